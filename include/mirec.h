/*
 * mirec.h — C ABI of libmirec.so, the MI355X (gfx950) engine for the
 * LightGCN propagation + BPR training hot path of
 * HiromasaYamanishi/furusato_recommend.
 *
 * Every entry point is extern "C", takes plain pointers and sizes, returns an
 * int status (0 = MIREC_OK) and never allocates device memory: the caller
 * (PyTorch's caching allocator on the Python side) owns every buffer and
 * passes scratch space explicitly.  Device entry points are stream-ordered on
 * the hipStream_t passed as `stream` (NULL = the legacy default stream), do
 * not synchronise the host and are safe to capture into a hipGraph.
 *
 * Reference interfaces each group replaces (paths under the reference repo):
 *   mirec_csr_*            model/lgcn.py:53-61 (symmetric edge list) and the
 *                          gcn_norm degree pass PyG's LGConv runs per call
 *                          (called at model/lgcn.py:66,82); restated in-repo
 *                          by model/radj.py:28-36.
 *   mirec_propagate        LGConv()(x, edge_index) at model/lgcn.py:82,
 *                          model/radj.py:39-44 (gather / scale / scatter-sum),
 *                          the layer mean of model/lgcn.py:78-86 and the
 *                          autograd backward of both.
 *   mirec_bpr_*            LightGCN.bpr_loss model/lgcn.py:98-118 + its
 *                          backward (stageOne, model/lgcn.py:127-133).
 *   mirec_adam_*           torch.optim.Adam created at model/lgcn.py:63,
 *                          stepped at model/lgcn.py:132.
 *   mirec_bpr_sample       UniformSample, negative_sample.py:98-134.
 */
#ifndef MIREC_H
#define MIREC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIREC_ABI_VERSION 1

enum mirec_status {
  MIREC_OK = 0,
  MIREC_ERR_ARG = 1,       /* null pointer / negative size / bad enum        */
  MIREC_ERR_DIM = 2,       /* embedding dim not in {4,8,16,32,64,128,256}    */
  MIREC_ERR_HIP = 3,       /* a HIP runtime call failed (mirec_last_hip_error) */
  MIREC_ERR_WORKSPACE = 4, /* caller-provided scratch space too small         */
  MIREC_ERR_RANGE = 5      /* an index is outside [0, n)                     */
};

typedef void *mirec_stream_t; /* hipStream_t */

const char *mirec_strerror(int code);
int mirec_abi_version(void);
int mirec_last_hip_error(void);
/* sizeof(mirec_csr_t), sizeof(mirec_prop_t), sizeof(mirec_adam_hparams_t):
 * lets FFI bindings verify their struct mirrors. */
int mirec_struct_sizes(size_t *csr, size_t *prop, size_t *adam_hparams);

/* ------------------------------------------------------------------------ */
/* Graph (host side, once per graph)                                         */
/* ------------------------------------------------------------------------ */

/* Destination-major CSR of the symmetric user–item graph of
 * model/lgcn.py:53-61: node ids are users [0, n_users) then items
 * n_users + [0, m_items).  Row u lists its items in edge order, row
 * n_users+i lists its users in edge order (stable, duplicates kept as
 * multi-edges exactly like the reference edge list).  dinv[v] =
 * deg(v)^-1/2, 0 for isolated nodes (gcn_norm, add_self_loops=False).
 * rowptr: [n_users+m_items+1], col: [2*n_edges], dinv: [n_users+m_items]. */
int mirec_csr_bipartite(const int64_t *train_user, const int64_t *train_item,
                        int64_t n_edges, int64_t n_users, int64_t m_items,
                        int64_t *rowptr, int32_t *col, float *dinv);

/* Generic stable CSR by destination from a COO edge list (edge_index[0] =
 * source, edge_index[1] = destination, the LGConv convention).  dinv (may
 * be NULL) = in-degree^-1/2 of every node (gcn_norm on `col`). */
int mirec_csr_from_coo(const int64_t *src, const int64_t *dst, int64_t nnz,
                       int64_t n_nodes, int64_t *rowptr, int32_t *col,
                       float *dinv);

/* Long-row schedule for load balance: rows with more than `split` entries
 * are cut into segments of `split` entries.  Call once with NULL outputs
 * to get the counts, then again with arrays of those sizes:
 * long_rows[n_long], long_segptr[n_long+1], seg_row[n_seg], seg_beg[n_seg]. */
int mirec_csr_long_rows(const int64_t *rowptr, int64_t n_rows, int32_t split,
                        int64_t *n_long, int64_t *n_seg, int32_t *long_rows,
                        int64_t *long_segptr, int32_t *seg_row,
                        int64_t *seg_beg);

/* Ingest (dataloader.py:93-150): parse an interaction file held in memory,
 * one line per user "uid i1 i2 ..." (spaces / tabs; empty lines skipped;
 * a line with only a uid counts as a line without items).  If stop_uid >= 0
 * parsing ends after the first line whose uid == stop_uid (the reference's
 * test-mode cut).  Call once with line_uid == NULL to get the counts and
 * maxima (-1 if none), then with line_uid[n_lines], line_off[n_lines + 1],
 * items[n_items]: line k has uid line_uid[k] and items
 * items[line_off[k] .. line_off[k+1]), in file order.  n_threads host
 * threads (buffers under 1 MiB use one).  MIREC_ERR_ARG on a malformed
 * token. */
int mirec_parse_interactions(const char *buf, int64_t len, int64_t stop_uid,
                             int32_t n_threads, int64_t *n_lines, int64_t *n_items,
                             int64_t *max_uid, int64_t *max_item, int64_t *line_uid,
                             int64_t *line_off, int64_t *items);

/* Device-resident CSR descriptor (all pointers are device pointers). */
typedef struct mirec_csr {
  const int64_t *rowptr;      /* [n_rows+1] */
  const int32_t *col;         /* [nnz] source node of each entry */
  const float *dinv;          /* [n_rows] deg^-1/2 (0 if deg == 0) */
  int64_t n_rows;
  int64_t nnz;
  int32_t split;              /* long-row threshold, 0 = none */
  int32_t _pad;
  int64_t n_long;
  int64_t n_seg;
  const int32_t *long_rows;   /* [n_long] */
  const int64_t *long_segptr; /* [n_long+1] */
  const int32_t *seg_row;     /* [n_seg] */
  const int64_t *seg_beg;     /* [n_seg] */
  /* optional (NULL = none): rows [0, n_sorted) with each row's entries sorted
   * ascending, entry rowptr[r] + j of the CSR at index rowptr[r] - rowptr[0]
   * + j (mirec_csr_sort_rows); the samplers' membership tests binary-search
   * them (the user rows of a bipartite graph) */
  const int32_t *col_sorted;
  int64_t n_sorted;
} mirec_csr_t;

/* Host: rows [0, n_rows) of (rowptr, col) with each row sorted ascending into
 * col_sorted [rowptr[n_rows] - rowptr[0]] (the csr's col_sorted). */
int mirec_csr_sort_rows(const int64_t *rowptr, const int32_t *col, int64_t n_rows,
                        int32_t *col_sorted);

/* ------------------------------------------------------------------------ */
/* Propagation: one LightGCN layer (CSR segment-gather SpMM + epilogue)      */
/* ------------------------------------------------------------------------ */

enum mirec_in_mode {
  MIREC_IN_PRESCALED = 0, /* x_in rows are already x~_j = dinv_j * x_j        */
  MIREC_IN_RAW = 1,       /* x_in rows are x_j; the kernel applies dinv_j     */
  MIREC_IN_SPARSE = 2,    /* input row j = seed_in[slot[j]] (0 if slot[j]<0),
                             kernel applies dinv_j                            */
  MIREC_IN_NONE = 3       /* no gather: y = 0 (epilogue only; L = 0 / MF)    */
};

typedef struct mirec_adam_hparams {
  float one_minus_beta1; /* 1 - beta1                      */
  float beta2;
  float one_minus_beta2; /* 1 - beta2                      */
  float neg_step_size;   /* -lr / (1 - beta1^t)            */
  float bc2_sqrt;        /* sqrt(1 - beta2^t)              */
  float eps;
} mirec_adam_hparams_t;

/* For every row i of the CSR:
 *   y_i   = dinv_i * sum_{j in row i} xin~_j                (Â x, fp32)
 *   z_i   = y_i + seed[slot_i]               (if seed != NULL and slot_i >= 0)
 *   xs_out_i = dinv_i * z_i                  (if xs_out != NULL; next layer)
 *   o_i   = (z_i + addend_i) / divisor + seed2[slot_i]
 *   out_i = o_i                 (if out != NULL and out_mask_i != 0)
 *   Adam(param_i, exp_avg_i, exp_avg_sq_i; grad = o_i)   (if param != NULL;
 *       then xs_out_i = dinv_i * param_i after the update)
 * `partial` is scratch of csr->n_seg * dim floats (may be NULL if n_seg==0).
 * Summation order per row is fixed by the CSR: results are deterministic. */
typedef struct mirec_prop {
  int32_t dim;
  int32_t in_mode;
  const float *x_in;    /* [n_rows, dim] (modes 0/1) */
  const int32_t *slot;  /* [n_rows] seed slot map, -1 = none */
  const float *seed_in; /* [*, dim] mode-2 input rows indexed by slot */
  const float *seed;    /* [*, dim] */
  const float *addend;  /* [n_rows, dim] */
  const float *seed2;   /* [*, dim] */
  float divisor;
  float _pad;
  float *out;           /* [n_rows, dim] */
  float *xs_out;        /* [n_rows, dim] */
  float *param;         /* fused Adam: [n_rows, dim] each */
  float *exp_avg;
  float *exp_avg_sq;
  mirec_adam_hparams_t adam;
  float *partial;       /* [n_seg, dim] scratch */
  const uint8_t *row_mask;  /* [n_rows] byte map: rows with byte 0 are
                               skipped (nothing written); NULL = all rows */
  const uint8_t *in_mask;   /* byte map over source nodes: only neighbours
                               with byte != 0 contribute (others are exact
                               zeros).  MIREC_IN_SPARSE filters by
                               slot[j] >= 0 when in_mask is NULL, else by
                               the byte map first (must cover the seeded
                               nodes; fewer slot reads when many neighbours
                               are seeded) */
  const uint8_t *out_mask;  /* byte map: rows with byte 0 skip the `out`
                               write and the addend read (their xs_out is
                               still written); ignored with fused Adam */
  const int32_t *row_list;  /* optional deduplicated row list (device); the
                               rows processed are row_list[0 .. *row_count);
                               needs row_mask = the same set (long rows) */
  const int32_t *row_count; /* device pointer to the list length */
  int64_t row_list_cap;     /* host upper bound of *row_count (grid size) */
  int32_t narrow_max;       /* rows of degree <= narrow_max are gathered one
                               per lane group (latency-bound short rows);
                               longer ones one per wave.  0 = always wave */
  int32_t _pad2;
  const int32_t *wide_list; /* optional second list (with row_list): rows
                               wide_list[0 .. *wide_count) are gathered by a
                               whole 256-thread workgroup each (4 waves split
                               the row, combined in LDS in a fixed order), so
                               a short list of long rows is not latency-bound */
  const int32_t *wide_count;
} mirec_prop_t;

int mirec_propagate(const mirec_csr_t *csr, const mirec_prop_t *p,
                    mirec_stream_t stream);

/* out = dinv ⊙ x row-wise (the pre-scaled layer-0 input x~_0). */
int mirec_prescale(const float *x, const float *dinv, int64_t n_rows,
                   int32_t dim, float *out, mirec_stream_t stream);

/* Row shards of the data-parallel `sharded` exchange (csrc/shard.hip;
 * replaces the reference's never-synchronised DDP, ddp_lgcn.py:663-673).
 * Rank r of W owns rows i ≡ r (mod W); slot s of rank r is row r + s·W; a
 * block of slots [slot0, slot0 + n_slots) is all-gathered through a
 * [W][n_slots][dim] staging buffer.  pack: stage_rank[s] = table[rank +
 * (slot0 + s)·W] (rows past n_rows give zero rows).  unpack: table[w +
 * (slot0 + s)·W] = stage[w][s] for every w != rank (rows past n_rows
 * skipped) and, with x0s (and dinv), x0s[row] = dinv[row] · stage[w][s]. */
int mirec_shard_pack(const float *table, int64_t n_rows, int32_t dim, int32_t world,
                     int32_t rank, int64_t slot0, int64_t n_slots, float *stage_rank,
                     mirec_stream_t stream);
int mirec_shard_unpack(const float *stage, int64_t n_rows, int32_t dim, int32_t world,
                       int32_t rank, int64_t slot0, int64_t n_slots, const float *dinv,
                       float *table, float *x0s, mirec_stream_t stream);

/* Frontier bitmaps of a key set S (keys[n_keys], entries outside [0, n_rows)
 * ignored; or, if keys == NULL, the 3*batch nodes of the triples users[b],
 * n_users+pos[b], n_users+neg[b]):  bm_self = S, bm_hop = S ∪ N(S).  Both
 * are byte maps of ceil(n_rows/4)*4 bytes (4-byte aligned), cleared first
 * (with one memset when bm_hop starts right after bm_self's 16-byte-rounded
 * size).  If self_list
 * is given it receives the distinct nodes of S (in no particular order) and
 * *self_count their number (capacity: n_keys or 3*batch).  zero_counts[0 ..
 * n_zero_counts) (<= 256, may be NULL / 0) are set to 0 with the maps — the
 * counters of the mirec_mask_compact calls that follow (counts_zeroed = 1):
 * adjacent, 16-byte aligned maps, S count and counters clear in one launch. */
int mirec_frontier(const mirec_csr_t *csr, const int32_t *keys, int64_t n_keys,
                   const int32_t *users, const int32_t *pos, const int32_t *neg,
                   int64_t batch, int64_t n_users, uint8_t *bm_self,
                   uint8_t *bm_hop, int32_t *self_list, int32_t *self_count,
                   int32_t *zero_counts, int32_t n_zero_counts, mirec_stream_t stream);

/* mirec_mask_compact of two byte maps in one launch (the step's S and F1 =
 * S ∪ N(S)), the degree split read from wide_bits (bit v of word v / 32:
 * degree of node v > narrow_max; built once per graph) instead of rowptr:
 * list_a / wide_a get map a's narrow / wide nodes, list_b / wide_b map b's;
 * counts[0..3] = their lengths (a narrow, a wide, b narrow, b wide), which
 * must be 0 on entry (mirec_frontier's zero_counts).  Lists ascending
 * within runs of 8 192 nodes; 16-byte aligned maps of >= n_rows bytes. */
int mirec_mask_compact_pair(const uint8_t *bm_a, const uint8_t *bm_b, const uint32_t *wide_bits,
                            int64_t n_rows, int32_t *list_a, int32_t *wide_a, int32_t *list_b,
                            int32_t *wide_b, int32_t *counts, mirec_stream_t stream);

/* Stable sort of n <= 8 192 (int32 key >= 0, int32 value) pairs: ascending
 * keys, equal keys in input order — bit for bit a stable radix sort's
 * result; vals_in NULL = the identity.  Two launches: every (key, index)
 * composite's rank counted over a grid of 256-entry blocks x 256-entry
 * chunks, then each pair written at its rank.  The sort of the BPR seed
 * grouping (mirec_bpr_seed: 3B node keys) and of small table-gradient
 * steps (mirec_table_grad_sorted); workspace: mirec_small_sort_workspace
 * bytes (ceil(n / 256) x n int32). */
int mirec_small_sort_workspace(int64_t n, size_t *bytes);
int mirec_small_sort_pairs(const int32_t *keys_in, const int32_t *vals_in, int32_t *keys_out,
                           int32_t *vals_out, int64_t n, void *workspace, size_t workspace_bytes,
                           mirec_stream_t stream);

/* Row lists of the nodes whose byte in the byte map bm[csr->n_rows] is
 * non-zero (16-byte aligned map): nodes of degree <= narrow_max (or all, if
 * wide_list is NULL) go to list[0 .. *count), the others to
 * wide_list[0 .. *wide_count); each list is ascending within runs of 4096
 * nodes, runs in no particular order (the result of a propagation does not
 * depend on list order).  Capacity: n_rows each.  Feeds the row_list /
 * wide_list of mirec_prop_t for the frontier-pruned launches.  The counts
 * are cleared first unless counts_zeroed (already 0 on this stream). */
int mirec_mask_compact(const mirec_csr_t *csr, const uint8_t *bm,
                       int32_t narrow_max, int32_t *list, int32_t *count,
                       int32_t *wide_list, int32_t *wide_count, int32_t counts_zeroed,
                       mirec_stream_t stream);

/* The ascending distinct ids of ids[0 .. n) that lie in [0, n_rows) and
 * outside [lo, hi) -> out[0 .. *count) (capacity n_rows): the rows a
 * data-parallel rank fetches from their owners before a GraphSAGE forward
 * (the fetch exchange of dist.DenseGradDataParallel; replaces torch.unique
 * of ddp-time bookkeeping, ddp_sage.py:754-878 has no exchange).  Byte map +
 * per-block counts + scan + ordered writes: no sort.  Workspace (16-byte
 * aligned): mirec_distinct_rows_workspace(n_rows) bytes. */
int64_t mirec_distinct_rows_workspace(int64_t n_rows);
int mirec_distinct_rows(const int32_t *ids, int64_t n, int64_t n_rows, int64_t lo,
                        int64_t hi, int32_t *out, int32_t *count, void *workspace,
                        size_t workspace_bytes, mirec_stream_t stream);
/* The same, skipping the ids whose byte in have[0 .. n_rows) is set, and
 * setting it for every id written: the pipelined exchange's read set of
 * micro-batch k without the rows fetched for micro-batches 0 .. k-1 (one
 * launch chain instead of a mask, a gather and a boolean compaction). */
int mirec_distinct_rows_unseen(const int32_t *ids, int64_t n, int64_t n_rows, int64_t lo,
                            int64_t hi, uint8_t *have, int32_t *out, int32_t *count,
                            void *workspace, size_t workspace_bytes, mirec_stream_t stream);

/* The rows r in [0, n_rows) with stamp[r] == gen (the rows a table gradient
 * of the sorted form wrote) ascending -> rows[0 .. counts[0]) (capacity
 * n_rows), and counts[1 + q] = those in owner block q of `parts` contiguous
 * blocks of n_rows / parts rows (the last to n_rows) — all on the device, no
 * host round trip: the pipelined fetch exchange's export of a micro-batch's
 * table-gradient rows (dist.DenseGradDataParallel; replaces torch.nonzero +
 * bincount).  Workspace: mirec_distinct_rows_workspace(n_rows) bytes. */
int mirec_stamped_rows(const int32_t *stamp, int64_t n_rows, int32_t gen, int32_t parts,
                       int32_t *rows, int32_t *counts, void *workspace,
                       size_t workspace_bytes, mirec_stream_t stream);

/* dst[ids[i], :] = src[i, :] for i < n (ids distinct; ids < 0 skipped);
 * dim % 4 == 0, src and dst 16-byte aligned: the install of the rows a rank
 * fetched into its local table (replaces index_copy_). */
int mirec_scatter_rows(const float *src, const int32_t *ids, int64_t n, int32_t dim,
                       float *dst, mirec_stream_t stream);

/* One source block of rows for mirec_owner_sum: ids[0 .. n) distinct,
 * rows [n, dim]. */
typedef struct mirec_row_block {
  const int32_t *ids;
  const float *rows;
  int64_t n;
} mirec_row_block_t;

/* out[r - lo, :] = sum over the blocks, IN BLOCK ORDER, of rows[i, :] where
 * ids[i] == r, for every r of the own block [lo, lo + n_own) (0 where no
 * block has r; ids outside the block ignored) — bitwise the sequence of
 * index_add_ launches it replaces (the owner side of the data-parallel
 * table-gradient exchange, dist.DenseGradDataParallel._owner_adam), in one
 * pass per 64 blocks.  Workspace: mirec_owner_sum_workspace(n_blocks, n_own)
 * bytes. */
int64_t mirec_owner_sum_workspace(int32_t n_blocks, int64_t n_own);
int mirec_owner_sum(const mirec_row_block_t *blocks, int32_t n_blocks, int64_t lo,
                    int64_t n_own, int32_t dim, void *workspace, size_t workspace_bytes,
                    float *out, mirec_stream_t stream);

/* out[i, :] = src[rows[i], :] for i < *count, the count read on the device
 * (capacity rows of out); dim % 4 == 0, src and out 16-byte aligned. */
int mirec_gather_rows_counted(const float *src, const int32_t *rows, const int32_t *count,
                              int64_t capacity, int32_t dim, float *out,
                              mirec_stream_t stream);

/* Capacity-bounded routing of a read set (the pipelined fetch exchange's
 * planner; replaces the per-read-set count read of ddp_sage.py:800-806's
 * exchange).  mirec_route_pack: ids ascending int32, *count (device) of them
 * valid, capacity = the ids buffer's length; writes one block per owner q
 * (contiguous row blocks of n_rows / parts, the last to n_rows) at
 * blocks + q*stride: blocks[q*stride] = the count of owner q's ids, then up
 * to cap of them (stride >= cap + 1; a count above cap is written as it is,
 * its ids past cap dropped: the host checks counts <= cap).  parts <= 256.
 * mirec_gather_rows_routed: the owner side over received blocks of that
 * layout: out[Σ_{p<q} min(c_p, cap) + j, :] = table[id_{q,j}, :], in source
 * order; out holds parts*cap rows of dim floats (ids outside [0, n_rows)
 * give zero rows). */
int mirec_route_pack(const int32_t *ids, const int32_t *count, int64_t capacity, int64_t n_rows,
                     int32_t parts, int32_t cap, int64_t stride, int32_t *blocks,
                     mirec_stream_t stream);
int mirec_gather_rows_routed(const float *table, int64_t n_rows, const int32_t *blocks,
                             int32_t parts, int32_t cap, int64_t stride, int32_t dim, float *out,
                             mirec_stream_t stream);

/* ------------------------------------------------------------------------ */
/* BPR (model/lgcn.py:98-133)                                                */
/* ------------------------------------------------------------------------ */

/* Scores of B triples from the layer-mean embeddings `out` [N, dim] and the
 * ego embeddings `emb` [N, dim] (users are rows [0, n_users), item ids are
 * offset by n_users).  Writes, per triple t:
 *   softplus[t] = softplus(<u,n> - <u,p>)          (torch threshold 20)
 *   coef[t]     = grad_scale * d mean(softplus) / d(neg - pos)
 *   reg[t]      = 1/2 (|u0|^2 + |p0|^2 + |n0|^2)
 * and the 3B seed keys/values (node id, occurrence index) consumed by
 * mirec_bpr_seed. */
int mirec_bpr_forward(const float *out, const float *emb, int64_t n_nodes,
                      int64_t n_users, int32_t dim, int64_t batch,
                      const int32_t *users, const int32_t *pos,
                      const int32_t *neg, float grad_scale, float *coef,
                      float *softplus, float *reg, int32_t *keys,
                      int32_t *vals, mirec_stream_t stream);

/* loss = mean(softplus) + decay * sum(reg) / B, written to loss_out[0];
 * if loss_accum != NULL also loss_accum[0] += loss (OneEpoch's aver_loss). */
int mirec_bpr_loss(const float *softplus, const float *reg, int64_t batch,
                   float decay, float *loss_out, float *loss_accum,
                   mirec_stream_t stream);

/* Scratch bytes mirec_bpr_seed needs for a batch of `batch` triples over a
 * graph of n_nodes nodes. */
int mirec_bpr_seed_workspace(int64_t batch, int64_t n_nodes, size_t *bytes);

/* Gradient seeds of the backward pass.  Sorts the 3B (node, occurrence)
 * pairs stably (mirec_small_sort_pairs up to 8 192 pairs, the device
 * library's radix sort above), marks the first position q of every distinct
 * node in `slot` (slot[node] = q; slot must be all -1 on entry) and writes
 *   seed_p[q] = (sum over the node's occurrences of dLoss/d out_node) / (L+1)
 *   seed_e[q] = decay * (#occurrences) * emb[node] / B   (reg term)
 * summed in occurrence order (deterministic).  keys_sorted[3B] keeps the
 * sorted node ids for mirec_bpr_seed_reset. */
int mirec_bpr_seed(const float *out, const float *emb, int64_t n_nodes,
                   int64_t n_users, int32_t dim, int64_t batch,
                   const int32_t *users, const int32_t *pos,
                   const int32_t *neg, const float *coef,
                   const int32_t *keys, const int32_t *vals, float decay,
                   float grad_scale, int32_t n_layers, int32_t *slot, float *seed_p,
                   float *seed_e, int32_t *keys_sorted, void *workspace,
                   size_t workspace_bytes, mirec_stream_t stream);

/* slot[keys_sorted[q]] = -1 for q in [0, n) (negative keys are skipped). */
int mirec_bpr_seed_reset(int32_t *slot, const int32_t *keys_sorted, int64_t n,
                         mirec_stream_t stream);

/* Dense pre-scaled seed rows: dense[v] = dinv[v] * seed[slot[v]] for the
 * listed nodes v = list[i], i < *count (device count, host bound cap), or
 * zeros when clear != 0 (restoring an all-zero table).  Feeds the first
 * backward layer as a PRESCALED input filtered by the S byte map. */
int mirec_seed_dense(const int32_t *list, const int32_t *count, int64_t cap,
                     const int32_t *slot, const float *dinv, const float *seed,
                     int32_t dim, float *dense, int32_t clear, mirec_stream_t stream);

/* Data-parallel sparse gradient exchange (dist.py).  The backward pass is
 * linear in the seeds, so the union batch's gradient is the backward of the
 * SUM of every rank's seeds: ranks all-gather their (node, seed_p, seed_e)
 * rows (3B each) instead of all-reducing the dense [N, D] gradient.
 * pack: keys_packed[q] = keys_sorted[q] at head positions, n_nodes elsewhere. */
int mirec_seed_pack(const int32_t *keys_sorted, int64_t n, int64_t n_nodes,
                    int32_t *keys_packed, mirec_stream_t stream);

int mirec_seed_merge_workspace(int64_t n, int64_t n_nodes, size_t *bytes);

/* merge: n gathered (key, row_p, row_e) entries (key == n_nodes: empty) →
 * per distinct node the sum of its rows in gathered order (deterministic,
 * identical on every rank), written at the node's first sorted position q;
 * slot[node] = q (slot must be all -1 on entry); keys_sorted[n] keeps the
 * sorted keys (-1 for empty entries) for mirec_bpr_seed_reset. */
int mirec_seed_merge(const int32_t *keys_packed, const float *rows_p,
                     const float *rows_e, int64_t n, int32_t dim,
                     int64_t n_nodes, int32_t *slot, float *seed_p,
                     float *seed_e, int32_t *keys_sorted, void *workspace,
                     size_t workspace_bytes, mirec_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Adam (torch.optim.Adam, amsgrad=False, weight_decay=0)                   */
/* ------------------------------------------------------------------------ */

int mirec_adam_dense(float *param, const float *grad, float *exp_avg,
                     float *exp_avg_sq, int64_t n,
                     const mirec_adam_hparams_t *h, mirec_stream_t stream);

/* Multi-tensor form for the small parameters of a model sharing one step
 * count: count (param, grad, exp_avg, exp_avg_sq, numel) tensors given as
 * host arrays of device pointers, one launch per 32 tensors.  Same update
 * as mirec_adam_dense. */
int mirec_adam_multi(int32_t count, float *const *params, const float *const *grads,
                     float *const *exp_avg, float *const *exp_avg_sq,
                     const int64_t *numel, const mirec_adam_hparams_t *hp,
                     mirec_stream_t stream);

/* The same two updates with the hyper-parameters read from DEVICE memory
 * when the kernel runs (h_device: one mirec_adam_hparams_t), so a captured
 * HIP graph replays each step with the scalars the host wrote there for
 * that step (bias corrections change every step). */
int mirec_adam_dense_dev(float *param, const float *grad, float *exp_avg,
                         float *exp_avg_sq, int64_t n,
                         const mirec_adam_hparams_t *h_device, mirec_stream_t stream);
int mirec_adam_multi_dev(int32_t count, float *const *params, const float *const *grads,
                         float *const *exp_avg, float *const *exp_avg_sq,
                         const int64_t *numel, const mirec_adam_hparams_t *h_device,
                         mirec_stream_t stream);

/* ------------------------------------------------------------------------ */
/* On-device BPR sampler (negative_sample.py:98-134 semantics)               */
/* ------------------------------------------------------------------------ */

/* Draws `batch` triples: u uniform over the users of shard `shard` (users
 * u with u % n_shards == shard; n_shards = 1 → all users), users with no
 * positives are redrawn, p uniform over u's CSR row (allPos order), n
 * uniform over [0, m_items) rejected while n is a positive of u.  Counter-
 * based: triple t of a call uses stream (seed, offset + t), so a batch is
 * reproducible and independent of the launch shape.  Item ids are returned
 * without the n_users offset.  err[0] is set to 1 if a draw exhausted its
 * retry budget (a user with every item as a positive). */
int mirec_bpr_sample(const mirec_csr_t *csr, int64_t n_users, int64_t m_items,
                     int64_t batch, uint64_t seed, uint64_t offset,
                     int32_t shard, int32_t n_shards, int32_t *users,
                     int32_t *pos, int32_t *neg, int32_t *err,
                     mirec_stream_t stream);

/* The ddp_lgcn.py epoch sampler (ddp_lgcn.py:33-35, 541-582): n_candidates
 * users drawn uniformly from the shard (users without positives are
 * skipped), a uniform positive each, and a candidate kept only if fewer than
 * `cap` earlier candidates (draw order) with the same positive item were kept
 * (POSITIVE_NUM_LIMIT = 3000); the kept ones (in draw order) draw a negative
 * not among the user's positives.  users / pos / neg: capacity n_candidates;
 * count[0] (device) = kept triples.  cand_u / cand_p (optional, [n]): every
 * candidate's user and positive (-1 = skipped).  Workspace:
 * mirec_bpr_sample_capped_workspace bytes. */
int mirec_bpr_sample_capped_workspace(int64_t n_candidates, int64_t m_items, size_t *bytes);

/* The same two samplers with per-user positive probabilities (the sample_pow
 * option of UniformSampling.sample_parallel, negative_sample.py:53-56:
 * np.random.choice(len(allPos[u]), p=probs[u])): pos_cdf[e - rowptr[0]]
 * is the inclusive cumulative probability of entry e within its user row
 * (rows 0 .. n_users - 1 of the CSR, i.e. the allPos order), non-decreasing
 * in the row, its last entry exactly 1.0, in float64 (mirec_pos_cdf_build makes
 * it on the host).  The positive is the first entry whose cumulative
 * probability exceeds a uniform draw on the 2^-53 grid (numpy's searchsorted
 * 'right' over its float64 CDF);
 * with pos_cdf = NULL they are the functions above (bit for bit). */
/* Host: cdf from probs[e - rowptr[0]] (float64, per user-row entry, each
 * non-empty row non-negative with a positive sum; normalised per row in
 * float64 as numpy's choice does).  MIREC_ERR_ARG on a negative / NaN entry
 * or a zero row. */
int mirec_pos_cdf_build(const int64_t *rowptr, int64_t n_users, const double *probs,
                        double *cdf);
int mirec_bpr_sample_ex(const mirec_csr_t *csr, const double *pos_cdf, int64_t n_users,
                        int64_t m_items, int64_t batch, uint64_t seed, uint64_t offset,
                        int32_t shard, int32_t n_shards, int32_t *users, int32_t *pos,
                        int32_t *neg, int32_t *err, mirec_stream_t stream);
int mirec_bpr_sample_capped(const mirec_csr_t *csr, int64_t n_users, int64_t m_items,
                            int64_t n_candidates, int32_t cap, uint64_t seed, uint64_t offset,
                            int32_t shard, int32_t n_shards, int32_t *users, int32_t *pos,
                            int32_t *neg, int32_t *count, int32_t *err, int32_t *cand_u,
                            int32_t *cand_p, void *workspace, size_t workspace_bytes,
                            mirec_stream_t stream);
int mirec_bpr_sample_capped_ex(const mirec_csr_t *csr, const double *pos_cdf, int64_t n_users,
                               int64_t m_items, int64_t n_candidates, int32_t cap,
                               uint64_t seed, uint64_t offset, int32_t shard, int32_t n_shards,
                               int32_t *users, int32_t *pos, int32_t *neg, int32_t *count,
                               int32_t *err, int32_t *cand_u, int32_t *cand_p, void *workspace,
                               size_t workspace_bytes, mirec_stream_t stream);

/* ------------------------------------------------------------------------ */
/* GraphSAGE hop ops (model/graphsage.py:311-324, neighbor_sampling.py)      */
/* ------------------------------------------------------------------------ */

/* Fixed-fanout sampling WITH replacement (neighbor_sampling.py:14-30):
 * children[t*k + c] = a uniform entry of the CSR row of nodes[t]
 * (counter RNG keyed by (seed, offset + t*k + c)); -1 if the row is empty. */
int mirec_sample_fanout(const mirec_csr_t *csr, const int32_t *nodes, int64_t n,
                        int32_t k, uint64_t seed, uint64_t offset,
                        int32_t *children, mirec_stream_t stream);

/* out[0, B) = users, out[B, 2B) = n_users + pos, out[2B, 3B) = n_users + neg
 * (the seed node ids of a BPR batch in a [users ; items] id table). */
int mirec_pack_seed_nodes(const int32_t *users, const int32_t *pos, const int32_t *neg,
                          int64_t batch, int64_t n_users, int32_t *out, mirec_stream_t stream);

/* Fixed-fanout sampling WITHOUT replacement (PyG NeighborSampler, the
 * sampler of model/graphsage.py:342-365): a node with at most k entries keeps
 * all of them in row order and -1 in the remaining slots; otherwise k
 * distinct entries of its row, uniformly (Floyd's algorithm on counter RNG
 * (seed, offset + t*k + j)).  Nodes without neighbours get k x -1 (their
 * mean is 0, as PyG's scatter-mean over no edges). */
int mirec_sample_fanout_norep(const mirec_csr_t *csr, const int32_t *nodes, int64_t n,
                              int32_t k, uint64_t seed, uint64_t offset, int32_t *children,
                              mirec_stream_t stream);

/* out[i, :] = table[ids[i], :] (zeros for ids[i] < 0); dim % 4 == 0. */
int mirec_gather_rows(const float *table, const int32_t *ids, int64_t n,
                      int32_t dim, float *out, mirec_stream_t stream);

/* table_grad[ids[i], :] += grad[i, :] (float atomics; ids < 0 skipped). */
int mirec_scatter_add_rows(const float *grad, const int32_t *ids, int64_t n,
                           int32_t dim, float *table_grad, mirec_stream_t stream);

/* out[t] = mean over the children c in [0,k) with valid[t*k+c] >= 0 (all if
 * valid == NULL) of dropout_p-dropout(x[t*k + c]); 0 if no valid child.
 * Dropout keeps an element with probability 1-p and scales it by 1/(1-p);
 * the mask is a hash of (seed, element index), so the backward recomputes
 * it.  dim % 4 == 0. */
int mirec_fanout_mean(const float *x, const int32_t *valid, int64_t n_targets,
                      int32_t k, int32_t dim, float dropout_p, uint64_t seed,
                      float *out, mirec_stream_t stream);

/* Backward of mirec_fanout_mean: grad_x[t*k + c] (written, not added). */
int mirec_fanout_mean_bwd(const float *grad_out, const int32_t *valid,
                          int64_t n_targets, int32_t k, int32_t dim,
                          float dropout_p, uint64_t seed, float *grad_x,
                          mirec_stream_t stream);

/* Fused leaf hop: out[t] = mean over the children c in [0,k) with
 * ids[t*k+c] >= 0 of dropout_p-dropout(table[ids[t*k+c]]) — the row gather
 * and mirec_fanout_mean in one pass (same dropout mask as gathering first
 * and calling mirec_fanout_mean).  The backward adds mask * grad_out[t] /
 * cnt into table_grad[ids[t*k+c]] (float atomics; k <= 64).  dim % 4 == 0. */
int mirec_fanout_mean_gather(const float *table, const int32_t *ids, int64_t n_targets,
                             int32_t k, int32_t dim, float dropout_p, uint64_t seed,
                             float *out, mirec_stream_t stream);
int mirec_fanout_mean_gather_bwd(const float *grad_out, const int32_t *ids,
                                 int64_t n_targets, int32_t k, int32_t dim,
                                 float dropout_p, uint64_t seed, float *table_grad,
                                 mirec_stream_t stream);

/* Deterministic form of mirec_fanout_mean_gather_bwd: the entries are
 * radix-sorted by child id and each id's contributions are summed in entry
 * order and added to its row once (no float atomics).  n_rows = rows of the
 * table (child ids < n_rows); workspace: ..._sorted_workspace bytes. */
int mirec_fanout_mean_gather_bwd_sorted_workspace(int64_t n_targets, int32_t k, int32_t n_rows,
                                                  size_t *bytes);
int mirec_fanout_mean_gather_bwd_sorted(const float *grad_out, const int32_t *ids,
                                        int64_t n_targets, int32_t k, int32_t dim,
                                        float dropout_p, uint64_t seed, int32_t n_rows,
                                        float *table_grad, void *workspace,
                                        size_t workspace_bytes, mirec_stream_t stream);

/* Deterministic id-table gradient (model/graphsage.py:311-337) and the Adam
 * step that consumes it (graphsage.py:388-397).  The table gradient of one
 * step is G[r] = c[slice(r)] * table[r] + S[r]: c = (c_user, c_item) the
 * norm-term coefficients dL/d|slice| / |slice| (device, 2 floats; rows
 * [0, n_user) are the user slice), S the sum of the tree's row
 * contributions, given as up to MIREC_TABLE_GRAD_MAX_GROUPS groups: entry
 * t*k + c of a group adds w_t * dropout(grad_out[t]) to row ids[t*k + c]
 * (ids < 0 skipped), with w_t = 1/(valid children of t) for a mean group
 * (the leaf hop's dropout-mean; mask element (t*k + c)*dim + col as in
 * mirec_fanout_mean_gather) and 1 otherwise (a plain row gather: k = 1,
 * dropout_p = 0). */
#define MIREC_TABLE_GRAD_MAX_GROUPS 8
typedef struct mirec_row_grad_group {
  const int32_t *ids;       /* [n_targets * k] row ids, -1 = none */
  const float *grad_out;    /* [n_targets, dim] */
  int64_t n_targets;
  int32_t k;
  int32_t mean;             /* 1: w_t = 1/cnt_t, 0: w_t = 1 */
  float dropout_p;
  int32_t _pad;
  uint64_t seed;
} mirec_row_grad_group_t;

/* sizeof(mirec_row_grad_group_t), for FFI struct-mirror checks. */
int64_t mirec_row_grad_group_size(void);

/* S for every touched row: the entries of all groups sorted by row id
 * (stable: mirec_small_sort_pairs up to 8 192 entries, the device library's
 * radix sort above), each id's contributions summed in entry order (runs longer than
 * a 64-entry chunk: per-chunk partials added in chunk order) — no float
 * atomics, bitwise repeatable.  Writes acc[r] = S[r] and stamp[r] = gen for
 * the touched rows only (nothing is cleared: a row belongs to this step iff
 * stamp[r] == gen).  acc [n_rows, dim], stamp [n_rows]; workspace:
 * mirec_table_grad_workspace bytes. */
int mirec_table_grad_workspace(const mirec_row_grad_group_t *groups, int32_t n_groups,
                               int32_t n_rows, int32_t dim, size_t *bytes);
int mirec_table_grad_sorted(const mirec_row_grad_group_t *groups, int32_t n_groups,
                            int32_t n_rows, int32_t dim, float *acc, int32_t *stamp, int32_t gen,
                            void *workspace, size_t workspace_bytes, mirec_stream_t stream);

/* The same S packed (the data-parallel exchanges' export): rows[j] = the
 * j-th touched row id ascending and vals[j] its row of S, j < counts[0];
 * counts[1 + p] = the touched rows in owner block p (rows [p N/P, (p + 1)
 * N/P), the last block to N = n_rows, P = parts) — all on the device, no
 * host sync.  The same sums bit for bit as mirec_table_grad_sorted; acc /
 * stamp are not touched.  rows / vals hold at least min(entries, n_rows)
 * rows; the workspace is mirec_table_grad_workspace's.  Replaces the
 * stamped-row scan + gather of the dense form for a routed step
 * (reference: the gradient all-reduce of ddp_sage.py:800-806). */
int mirec_table_grad_sorted_rows(const mirec_row_grad_group_t *groups, int32_t n_groups,
                                 int32_t n_rows, int32_t dim, int32_t parts, int32_t *rows,
                                 float *vals, int32_t *counts, void *workspace,
                                 size_t workspace_bytes, mirec_stream_t stream);

/* The same S in the atomic form, for plain groups only (k = 1, mean = 0,
 * dropout_p = 0): touched rows stamped and zeroed, then every gradient row
 * added with float atomics — two launches, no workspace; the summation
 * order of a repeated id is not fixed. */
int mirec_table_grad_atomic(const mirec_row_grad_group_t *groups, int32_t n_groups,
                            int32_t n_rows, int32_t dim, float *acc, int32_t *stamp, int32_t gen,
                            mirec_stream_t stream);

/* grad = G materialised (coef may be NULL = 0), [n_rows, dim]. */
int mirec_table_grad_dense(const float *table, const float *coef, int64_t n_user,
                           const float *acc, const int32_t *stamp, int32_t gen, int64_t n_rows,
                           int32_t dim, float *grad, mirec_stream_t stream);

/* Adam (torch.optim.Adam, as mirec_adam_dense) of the whole table with G
 * formed on the fly: param / exp_avg / exp_avg_sq read and written once,
 * the dense gradient never stored.  If sumsq and norms are given (sumsq:
 * mirec_adam_table_sumsq_floats floats), norms[0..1] = the L2 norms of the
 * UPDATED user / item slices (the next step's norm term), fixed order. */
int64_t mirec_adam_table_sumsq_floats(int64_t n_rows, int32_t dim);
int mirec_adam_table(float *param, float *exp_avg, float *exp_avg_sq, const float *coef,
                     int64_t n_user, const float *acc, const int32_t *stamp, int32_t gen,
                     int64_t n_rows, int32_t dim, const mirec_adam_hparams_t *h, float *sumsq,
                     float *norms, mirec_stream_t stream);
/* The owner's step of the data-parallel exchanges in one pass: S of the own
 * row block [lo, lo + n_own) from the source blocks exactly as
 * mirec_owner_sum forms it (block order), then mirec_adam_table on those
 * rows with every row stamped (param / exp_avg / exp_avg_sq point at row lo;
 * n_user = the block's user rows; sumsq / norms as there, sumsq of
 * mirec_adam_table_sumsq_floats(n_own, dim) floats) — S is never stored.
 * Bitwise the same parameters, moments and norms as mirec_owner_sum +
 * mirec_adam_table.  At most 64 blocks.  Workspace:
 * mirec_owner_sum_workspace(n_blocks, n_own) bytes.  (Reference: the Adam
 * step of the synchronised table gradient, ddp_sage.py:800-806.) */
int mirec_owner_adam(const mirec_row_block_t *blocks, int32_t n_blocks, int64_t lo,
                     int64_t n_own, int32_t dim, float *param, float *exp_avg,
                     float *exp_avg_sq, const float *coef, int64_t n_user,
                     const mirec_adam_hparams_t *h, float *sumsq, float *norms, void *workspace,
                     size_t workspace_bytes, mirec_stream_t stream);
/* mirec_adam_table with the hyper-parameters read from device memory when
 * the kernel runs (capturable in a HIP graph). */
int mirec_adam_table_dev(float *param, float *exp_avg, float *exp_avg_sq, const float *coef,
                         int64_t n_user, const float *acc, const int32_t *stamp, int32_t gen,
                         int64_t n_rows, int32_t dim, const mirec_adam_hparams_t *h_device,
                         float *sumsq, float *norms, mirec_stream_t stream);

/* coef[i] = norm[i*norm_stride] > 0 ? g[i*g_stride] / norm[i*norm_stride] : 0
 * for i < n (<= 1024): a table gradient's norm-term coefficients. */
int mirec_norm_coef(const float *g, int32_t g_stride, const float *norm, int32_t norm_stride,
                    int32_t n, float *coef, mirec_stream_t stream);

/* ------------------------------------------------------------------------ */
/* SASRec causal self-attention (model/sasrec.py:385-397), f32 MFMA          */
/* ------------------------------------------------------------------------ */

/* qkv: the packed in-projection output [batch, T, 3*heads*head_dim] (q | k |
 * v, head h = columns h*head_dim ..); out: [batch, T, heads*head_dim] =
 * softmax(q kᵀ / sqrt(head_dim) + causal mask) v per head.  T <= 64,
 * 1 <= head_dim <= 64. */
int mirec_attention_fwd(const float *qkv, int64_t batch, int32_t T, int32_t heads,
                        int32_t head_dim, float *out, mirec_stream_t stream);

/* Backward: dqkv [batch, T, 3*heads*head_dim] (written) from dout. */
int mirec_attention_bwd(const float *qkv, const float *dout, int64_t batch, int32_t T,
                        int32_t heads, int32_t head_dim, float *dqkv,
                        mirec_stream_t stream);

/* Packed (variable-length) form: sequence b is rows offsets[b] ..
 * offsets[b+1]-1 of qkv [n_tok, 3*heads*head_dim] / out / dout / dqkv
 * [n_tok, ...]; offsets (device, int32, batch+1 entries, non-decreasing)
 * with every length <= 64 (longer sequences are cut to their first 64
 * rows).  Padding positions past a sequence's length never influence its
 * earlier positions under the causal mask, so the padded and the packed
 * forms agree on every real row; the packed one skips the padding. */
int mirec_attention_varlen_fwd(const float *qkv, const int32_t *offsets, int64_t batch,
                               int32_t heads, int32_t head_dim, float *out,
                               mirec_stream_t stream);
int mirec_attention_varlen_bwd(const float *qkv, const float *dout, const int32_t *offsets,
                               int64_t batch, int32_t heads, int32_t head_dim,
                               float *dqkv, mirec_stream_t stream);

/* Packed form with the sequences ordered by length bucket: bucket_end (HOST
 * array of 4 non-decreasing counts; batch = bucket_end[3]) says sequences
 * [bucket_end[k-1], bucket_end[k]) have at most 16*(k+1) positions.  Each
 * bucket runs on a kernel whose workgroup holds only 16*(k+1) rows (one
 * wave per 16-row block, LDS sized to match), so short sequences neither
 * idle three waves nor reserve a 64-row LDS image.  A longer sequence placed
 * in a bucket is cut to the bucket's rows (an input error). */
int mirec_attention_bucketed_fwd(const float *qkv, const int32_t *offsets,
                                 const int64_t *bucket_end, int32_t heads, int32_t head_dim,
                                 float *out, mirec_stream_t stream);
int mirec_attention_bucketed_bwd(const float *qkv, const float *dout, const int32_t *offsets,
                                 const int64_t *bucket_end, int32_t heads, int32_t head_dim,
                                 float *dqkv, mirec_stream_t stream);

/* Backward with short sequences sharing a workgroup (one wave per 16-row
 * block, up to 4 blocks per workgroup): packs from
 * mirec_attention_length_order; head_dim % 4 == 0, <= 64.  Rows
 * [offsets[batch], n_rows) of dqkv (capacity padding) are zeroed. */
int mirec_attention_packed_bwd(const float *qkv, const float *dout, const int32_t *offsets,
                               const int32_t *packs, int64_t batch, int32_t heads,
                               int32_t head_dim, float *dqkv, int64_t n_rows,
                               mirec_stream_t stream);
/* The packed backward given the forward's statistic: lse [n, heads] as
 * mirec_attention_wave_fwd wrote it (base 2).  P = exp2(S scale log2 e -
 * lse) directly, with no max / sum reductions in the kernel.  Same packs,
 * layout and padding rows as mirec_attention_packed_bwd. */
int mirec_attention_packed_bwd_lse(const float *qkv, const float *lse, const float *dout,
                                   const int32_t *offsets, const int32_t *packs, int64_t batch,
                                   int32_t heads, int32_t head_dim, float *dqkv, int64_t n_rows,
                                   mirec_stream_t stream);

/* Packed form with the workgroups in a given sequence order (device int32
 * [batch], e.g. mirec_attention_length_order: longest first). */
int mirec_attention_ordered_fwd(const float *qkv, const int32_t *offsets, const int32_t *order,
                                int64_t batch, int32_t heads, int32_t head_dim, float *out,
                                mirec_stream_t stream);
int mirec_attention_ordered_bwd(const float *qkv, const float *dout, const int32_t *offsets,
                                const int32_t *order, int64_t batch, int32_t heads,
                                int32_t head_dim, float *dqkv, mirec_stream_t stream);

/* One wave per (sequence, head) (csrc/attn_wave.hip): no LDS, no barriers,
 * every operand loaded straight into its MFMA lane layout; head_dim 16, 32
 * or 64 (mirec_attention_wave_supported).  offsets == NULL: uniform batch
 * [batch, T, ...] (1 <= T <= 64); else packed as in the varlen form.  The
 * forward also writes lse [n_rows, heads] (BASE-2 log-sum-exp of each query's
 * scaled scores: log2 sum_k 2^(s_k * scale * log2 e), i.e. the natural lse times
 * log2 e); the backward takes out and lse from it and writes dqkv and delta
 * [n_rows, heads] (rowsum(dout ⊙ out), scratch), in two launches.  order
 * (optional, packed form): the sequences in the order their units run, from
 * mirec_attention_length_order (longest first, device int32 [batch]; the
 * forward with offsets and n_rows > 0 also zeroes out's rows [offsets[batch],
 * n_rows) (capacity padding); with
 * packs (optional, int32 [4 + 8 batch], 16-byte aligned) it also groups
 * that order into packs of at most 4 blocks of 16 positions for
 * mirec_attention_packed_bwd: packs[0] = count, packs[4 + 8p + 2s] and
 * packs[5 + 8p + 2s] = (first row, length) of the sequence in slot s of
 * pack p, (0, 0) when empty); with zero_buf it
 * also zeroes rows [offsets[batch], zero_rows) of that [zero_rows,
 * zero_width] buffer (the capacity padding of a packed batch's output). */
int mirec_attention_wave_supported(int32_t head_dim);
int mirec_attention_length_order(const int32_t *offsets, int64_t batch, int32_t *order,
                                 int32_t *packs, float *zero_buf, int64_t zero_rows,
                                 int32_t zero_width, mirec_stream_t stream);
int mirec_attention_wave_fwd(const float *qkv, const int32_t *offsets, const int32_t *order,
                             int64_t batch, int32_t T, int32_t heads, int32_t head_dim, float *out,
                             float *lse, int64_t n_rows, mirec_stream_t stream);
int mirec_attention_wave_bwd(const float *qkv, const float *out, const float *lse,
                             const float *dout, const int32_t *offsets, const int32_t *order,
                             int64_t batch, int32_t T, int32_t heads, int32_t head_dim,
                             float *dqkv, float *delta, mirec_stream_t stream);

/* Masked mean pool of the SASRec user tower (model/sasrec.py:399-413) on
 * packed sequences: out[b] = Σ_{r in [offsets[b], offsets[b+1])} x[r] /
 * length[b] (rows summed in a fixed order), x [n, d], out [B, d], d % 4 == 0,
 * d <= 1024.  Backward: grad_x[t] = grad_out[seg[t]] / length[seg[t]] for
 * the n_rows rows (0 where seg[t] is outside [0, B): capacity padding). */
int mirec_segment_mean(const float *x, const int32_t *offsets, const int64_t *length, int64_t B,
                       int32_t d, float *out, mirec_stream_t stream);
int mirec_segment_mean_bwd(const float *grad_out, const int64_t *seg, const int64_t *length,
                           int64_t n_rows, int64_t B, int32_t d, float *grad_x,
                           mirec_stream_t stream);

/* BPR loss on embedding rows (model/sasrec.py:423-435): x_r = <u_r, n_r> -
 * <u_r, p_r> (written to x_out[0..B); x_out holds 2B floats, the second half
 * scratch), loss[0] = mean_r softplus(x_r) + coef * extra[0] (extra: a
 * device scalar such as the embedding-norm term, or NULL); u, p, n [B, d].
 * Fixed summation order (deterministic).  Backward:
 * with g = g_loss[0] (device) and s_r = g sigmoid(x_r) / B: du = s (n - p),
 * dp = -s u, dn = s u, and g_extra[0] = g coef (if g_extra != NULL). */
int mirec_bpr_rows_loss(const float *u, const float *p, const float *n, int64_t B, int32_t d,
                        const float *extra, float coef, float *x_out, float *loss,
                        mirec_stream_t stream);
int mirec_bpr_rows_loss_bwd(const float *u, const float *p, const float *n, const float *x,
                            int64_t B, int32_t d, const float *g_loss, float coef, float *du,
                            float *dp, float *dn, float *g_extra, mirec_stream_t stream);

/* L2 norms of x[0, split) and x[split, n) -> norms[0], norms[1] (the
 * parameter-norm terms of model/graphsage.py:326-337 / model/sasrec.py:
 * 423-435 over an id table's user / item slices; split = n for one norm).
 * n % 4 == 0, split % 4 == 0, x 16-byte aligned; work:
 * mirec_slice_norms_work_floats() floats.  Fixed summation order. */
int64_t mirec_slice_norms_work_floats(void);
int mirec_slice_norms(const float *x, int64_t n, int64_t split, float *work, float *norms,
                      mirec_stream_t stream);

/* Weighted parameter-norm term (model/graphsage.py:326-337: all_param = 2
 * all_param + |p| over the parameters = Σ_k 2^(K-1-k) |p_k|):
 * total[0] = Σ_j extra_w[j] * extra[j] + Σ_k weights[k] * |xs[k]|₂ (extra:
 * norms already on the device, e.g. the id table's slices; xs: count small
 * device tensors of numel[k] floats, host array of pointers; weights /
 * extra_w: host arrays), norms[k] = |xs[k]|₂.  Fixed summation order.
 * Backward: grads[k] = g * weights[k] * xs[k] / |xs[k]| (written; 0 where the
 * norm is 0) and extra_grad[j] = g * extra_w[j], with g = g_total[0]
 * (device).  count, n_extra <= MIREC_NORM_TERMS_MAX. */
#define MIREC_NORM_TERMS_MAX 16
int mirec_norm_terms(const float *const *xs, const int64_t *numel, const float *weights,
                     int32_t count, const float *extra, const float *extra_w, int32_t n_extra,
                     float *norms, float *total, mirec_stream_t stream);
int mirec_norm_terms_bwd(const float *const *xs, float *const *grads, const int64_t *numel,
                         const float *weights, int32_t count, const float *norms,
                         const float *g_total, const float *extra_w, int32_t n_extra,
                         float *extra_grad, mirec_stream_t stream);
/* The same small-tensor gradients ADDED to grads[k] (the gradients the rest
 * of the backward already accumulated there): g_k += g * weights[k] * xs[k] /
 * |xs[k]|.  Run once the backward is done, so a parameter used by several
 * nodes is not summed by a separate elementwise kernel per use. */
int mirec_norm_terms_bwd_acc(const float *const *xs, float *const *grads, const int64_t *numel,
                             const float *weights, int32_t count, const float *norms,
                             const float *g_total, mirec_stream_t stream);

/* Per-step (positive, negative) pairs of a sequence batch: out[j] = a
 * uniform element of user users[j]'s sequence items[u][0, length[u]) (0 for
 * an empty one), out[B + j] = a uniform item in [0, m_items); counter-based
 * (seed, offset + j). */
int mirec_seq_sample(const int64_t *users, int64_t B, const int32_t *items, int32_t max_len,
                     const int64_t *length, int64_t m_items, uint64_t seed, uint64_t offset,
                     int64_t *out, mirec_stream_t stream);

/* Pack a SASRec batch into a fixed token capacity (the graph-captured step,
 * model/sasrec.py:449-455's pad_sequence without the padding): users [B]
 * (device int64), items [n_users, max_len] (int32, each user's last items),
 * length_tab [n_users] (int64), pos / neg [B] (int64).  Writes length[b] =
 * length_tab[users[b]], offsets[B+1] = the prefix sums clamped to capacity
 * (int32), ids_all[capacity + 2B] (int32) = the item id of every token row
 * (-1 past the last sequence) followed by pos and neg, and seg[capacity]
 * (int64) = the sequence of every row (B past the last sequence). */
int mirec_seq_pack(const int64_t *users, int64_t B, const int32_t *items, int32_t max_len,
                   const int64_t *length_tab, const int64_t *pos, const int64_t *neg,
                   int64_t capacity, int32_t *offsets, int64_t *length, int32_t *ids_all,
                   int64_t *seg, mirec_stream_t stream);

/* Zero rows [offsets[B], n_rows) of buf [n_rows, row_floats] (offsets on the
 * device): the capacity-padding rows of a packed batch, which the packed
 * attention kernels do not write. */
int mirec_zero_tail_rows(float *buf, const int32_t *offsets, int64_t B, int64_t n_rows,
                         int32_t row_floats, mirec_stream_t stream);

/* f32 MFMA GEMMs of the Linear layers on token rows (model/sasrec.py:385-421,
 * model/graphsage.py:311-324).  Row-major, device pointers, 16-byte aligned.
 *
 * Arithmetic (default build, MIREC_GEMM_X6): every f32 operand is split
 * exactly into three bf16 terms and each product is formed from the six
 * largest term products on bf16 MFMA with f32 accumulation — the error of
 * one f32 rounding per product.  Edge semantics differ from
 * an fp32 FMA chain: an infinite or NaN operand gives NaN (inf - inf in the
 * split), so an overflowed input yields NaN where fp32 would give +-inf; and
 * operands below ~2^-110 lose low-order bits (the third term underflows
 * bf16's range) — far below anything a finite, non-overflowing training step
 * feeds these GEMMs.  Building with -DMIREC_GEMM_X6=0 selects exact f32
 * v_mfma_f32_32x32x2_f32 products.
 *
 * C[n, No] = A[n, Kr] · B[No, Kr]ᵀ (+ bias[No] if bias != NULL): the forward
 * y = x Wᵀ + b, and the input gradient dX = dY W with B = Wᵀ (a [K, N] copy
 * of the weight).  Kr % 32 == 0, No % 128 == 0. */
int mirec_gemm_nt(const float *A, const float *B, const float *bias, float *C, int64_t n,
                  int32_t Kr, int32_t No, mirec_stream_t stream);

/* C[M, No] = A[n, M]ᵀ · B[n, No] summed over the n rows, and (if colsum !=
 * NULL) colsum[M] = Σ_rows A: the weight gradient dW = dYᵀ X and the bias
 * gradient db = Σ dY in one pass over dY.  M % 128 == 0, No % 128 == 0;
 * work: mirec_gemm_tn_work_floats(n, M, No) floats (per-slice partial
 * sums, added in a fixed order: deterministic). */
int64_t mirec_gemm_tn_work_floats(int64_t n, int32_t M, int32_t No);

/* out[c] = Σ_r A[r, c] over the n rows of a row-major [n, m] matrix, summed
 * in a fixed order (deterministic, capturable): the bias gradient db = Σ dY
 * of a Linear whose width the GEMM tiles do not take (nn.Linear backward,
 * model/sasrec.py:385-421), and the slice sum of the split weight gradient.
 * work: mirec_col_sums_work_floats(n, m) floats. */
int64_t mirec_col_sums_work_floats(int64_t n, int32_t m);
int mirec_col_sums(const float *A, int64_t n, int32_t m, float *out, float *work,
                   mirec_stream_t stream);
int mirec_gemm_tn(const float *A, const float *B, float *C, float *colsum, int64_t n, int32_t M,
                  int32_t No, float *work, mirec_stream_t stream);

/* Fused forms of the two GEMMs (the GraphSAGE hop h = relu(W [x ; aggr] + b),
 * model/graphsage.py:314-315, without materialising the concatenation):
 *   gemm_nt_ex: A2 != NULL: the A row is [A[r, 0:Ks) | A2[r, 0:Kr-Ks)] (row
 *     strides Ks and Kr-Ks; Ks % 32 == 0); Amask != NULL (single A only): A
 *     elements whose Amask element (same layout) is <= 0 read as 0 (the ReLU
 *     backward dY * (y > 0)); C2 != NULL: output columns [0, Ns) go to C (row
 *     stride Ns) and [Ns, No) to C2 (stride No-Ns; Ns % 128 == 0); relu != 0:
 *     max(., 0) after the bias.
 *   gemm_tn_ex: Amask as above on A; B2 != NULL: the B row is [B[r, 0:Ns) |
 *     B2[r, 0:No-Ns)] (Ns % 128 == 0); colsum = Σ of the masked A. */
int mirec_gemm_nt_ex(const float *A, const float *A2, int32_t Ks, const float *Amask,
                     const float *B, const float *bias, float *C, float *C2, int32_t Ns,
                     int32_t relu, int64_t n, int32_t Kr, int32_t No, mirec_stream_t stream);
/* C = A B with B [Kr, No] row-major (the input gradient dX = dY W of a
 * Linear, W used as stored: no transposed copy); Amask and the C / C2 split
 * as in gemm_nt_ex. */
int mirec_gemm_nn_ex(const float *A, const float *Amask, const float *B, float *C, float *C2,
                     int32_t Ns, int64_t n, int32_t Kr, int32_t No, mirec_stream_t stream);
int mirec_gemm_tn_ex(const float *A, const float *Amask, const float *B, const float *B2,
                     int32_t Ns, float *C, float *colsum, int64_t n, int32_t M, int32_t No,
                     float *work, mirec_stream_t stream);

/* Row tail of the SASRec block (model/sasrec.py:385-397 — the dropout,
 * residual add, ReLU and LayerNorm around the attention and the FFN), one
 * pass over the n x d token rows (d % 4 == 0, 4 <= d <= 1024):
 *   pre = (res ? res : 0) + dropout_p-dropout(z + (bias ? bias : 0))
 *   out = relu ? max(pre, 0) : pre                         (written if out)
 *   y   = (out - mean) * rstd * (gamma ? gamma : 1) + (beta ? beta : 0),
 *         rstd = 1 / sqrt(biased var + eps)                (written if y;
 *         mean / rstd [n] then required)
 * out may be NULL only when it equals z (no res / bias / relu / dropout).
 * The dropout mask is the counter hash of (seed, row * d + col) — the same
 * seed recomputes it in the backward.  seed_base (device, may be NULL): when
 * given, *seed_base is mixed into the mask key when the kernel runs, so a
 * captured HIP graph draws a fresh mask on every replay (the host writes a
 * new base before each replay; the backward reads the same base). */
int mirec_resnorm_fwd(const float *res, const float *z, const float *bias, const float *gamma,
                      const float *beta, int64_t n, int32_t d, int32_t relu, float dropout_p,
                      uint64_t seed, const uint64_t *seed_base, float eps, float *out, float *y,
                      float *mean, float *rstd, mirec_stream_t stream);

/* mirec_resnorm_fwd with z = A Wᵀ computed in the same kernel (A [n, Kr],
 * W [d, Kr] row-major, d = 128, Kr % 32 == 0): the Linear before a block
 * stage's row tail (model/sasrec.py:385-397 — attention out-projection and
 * FFN, their biases passed as `bias`), z never written.  out is required;
 * every other argument and output as in mirec_resnorm_fwd (identical
 * values: same per-row arithmetic); the backward is mirec_resnorm_bwd
 * followed by the Linear's gradients (mirec_gemm_nn_ex / mirec_gemm_tn). */
int mirec_gemm_resnorm(const float *A, const float *W, int64_t n, int32_t Kr, int32_t d,
                       const float *res, const float *bias, const float *gamma, const float *beta,
                       int32_t relu, float dropout_p, uint64_t seed, const uint64_t *seed_base,
                       float eps, float *out, float *y, float *mean, float *rstd,
                       mirec_stream_t stream);

/* Backward counterpart of mirec_gemm_resnorm: g_y = A W computed in the
 * kernel (A [n, Kr], W [Kr, d] row-major as stored — the input gradient of
 * the Linear that consumed this row tail's y — d = 128, Kr % 32 == 0), then
 * mirec_resnorm_bwd(g_y, g_out, out, mean, rstd, gamma, ...) (the same
 * per-row expressions; d_gamma / d_beta / d_bias, each optional, summed per 64-row
 * tile and then in tile order (work: mirec_gemm_nn_resnorm_bwd_work_floats
 * floats when any sum is asked).  g_y is never written. */
int64_t mirec_gemm_nn_resnorm_bwd_work_floats(int64_t n, int32_t d);
int mirec_gemm_nn_resnorm_bwd(const float *A, const float *W, int64_t n, int32_t Kr, int32_t d,
                              const float *g_out, const float *out, const float *mean,
                              const float *rstd, const float *gamma, int32_t relu,
                              float dropout_p, uint64_t seed, const uint64_t *seed_base,
                              float *d_res, float *d_z, float *work, float *d_gamma,
                              float *d_beta, float *d_bias, mirec_stream_t stream);
/* The fixed-order sum of [parts][3][d] column partials into d_gamma /
 * d_beta / d_bias (each optional): the second pass of the row-tail
 * backwards. */
int mirec_resnorm_reduce_partials(const float *work, int64_t parts, int32_t d, float *d_gamma,
                                  float *d_beta, float *d_bias, mirec_stream_t stream);

/* Floats of scratch mirec_resnorm_bwd needs for parameter gradients. */
int64_t mirec_resnorm_work_floats(int64_t n, int32_t d);

/* Backward of mirec_resnorm_fwd.  out: the forward's out (or z when out
 * was omitted); g_y / g_out: gradients of y / out (either may be NULL =
 * zero).  Writes d_res = d(pre) and d_z = d(z) = d(bias) per row (each
 * optional), and the column sums d_gamma = Σ g_y·x̂, d_beta = Σ g_y,
 * d_bias = Σ d_z (each optional; work then needs
 * mirec_resnorm_work_floats floats).  Sums are added in a fixed order. */
int mirec_resnorm_bwd(const float *g_y, const float *g_out, const float *out, const float *mean,
                      const float *rstd, const float *gamma, int64_t n, int32_t d, int32_t relu,
                      float dropout_p, uint64_t seed, const uint64_t *seed_base, float *d_res,
                      float *d_z, float *work, float *d_gamma, float *d_beta, float *d_bias,
                      mirec_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Evaluation (trainer.py:130-138)                                           */
/* ------------------------------------------------------------------------ */

/* scores [n_eval, m_items] row-major (a GEMM of user and item embeddings,
 * model/lgcn.py:124).  If csr != NULL, row b's train positives (the CSR row
 * of user users[b]: node ids n_users + item) are set to -1024 in place
 * (trainer.py:132-137).  Then the k best items of every row (score
 * descending, ties to the lower item id) go to topk_idx[b*k ..] and, if
 * topk_val != NULL, their scores to topk_val.  1 <= k <= 64. */
int mirec_topk_masked(float *scores, int64_t n_eval, int64_t m_items,
                      const int32_t *users, const mirec_csr_t *csr,
                      int64_t n_users, int32_t k, int32_t *topk_idx,
                      float *topk_val, mirec_stream_t stream);

/* Streaming evaluation: the top-k of user_emb[b] · item_embᵀ
 * per evaluated user b, the user's train positives (csr row users[b],
 * entries n_users + item) scoring -1024, WITHOUT materialising the
 * [n_eval, m_items] scores: MFMA score tiles are filtered into per-user
 * candidate lists as they are produced (two launches).  user_emb [n_eval,
 * dim], item_emb [m_items, dim], dim in {16, 32, 64, 128}, 1 <= k <= 32;
 * same order and ties as mirec_topk_masked.  workspace:
 * mirec_score_topk_workspace bytes. */
int64_t mirec_score_topk_workspace(int64_t n_eval, int64_t m_items, int32_t k);
int mirec_score_topk(const float *user_emb, int64_t n_eval, const float *item_emb,
                     int64_t m_items, int32_t dim, const int32_t *users, const mirec_csr_t *csr,
                     int64_t n_users, int32_t k, int32_t *topk_idx, float *topk_val,
                     void *workspace, size_t workspace_bytes, mirec_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Host (CPU) path of configuration C1 (model/MF.py BPR, "CPU single-process", */
/* BASELINE configs[0]): host pointers, no stream, n_threads worker threads.  */
/* ------------------------------------------------------------------------ */

/* mirec_bpr_sample on the host: the same counter streams, so the triples are
 * the device sampler's bit for bit (col_sorted / pos_cdf optional, as in
 * mirec_csr_t / mirec_bpr_sample_ex).  Replaces UniformSample,
 * negative_sample.py:98-134, for a CPU model. */
int mirec_cpu_bpr_sample(const int64_t *rowptr, const int32_t *col, const int32_t *col_sorted,
                         const double *pos_cdf, int64_t n_users, int64_t m_items, int64_t batch,
                         uint64_t seed, uint64_t offset, int32_t shard, int32_t n_shards,
                         int32_t *users, int32_t *pos, int32_t *neg, int32_t *err,
                         int32_t n_threads);

/* mirec_bpr_sample_capped_ex on the host (the ddp_lgcn.py epoch sampler for
 * a CPU model): the same candidate streams, so users / pos / neg (capacity
 * n_candidates), *count and the optional cand_u / cand_p equal the device
 * sampler's bit for bit; the keep decision is the reference's sequential
 * per-item count (ddp_lgcn.py:571-572).  *err = 1 if a negative draw
 * exhausted its retries.  No workspace. */
int mirec_cpu_bpr_sample_capped(const int64_t *rowptr, const int32_t *col,
                                const int32_t *col_sorted, const double *pos_cdf, int64_t n_users,
                                int64_t m_items, int64_t n_candidates, int32_t cap, uint64_t seed,
                                uint64_t offset, int32_t shard, int32_t n_shards, int32_t *users,
                                int32_t *pos, int32_t *neg, int32_t *count, int32_t *err,
                                int32_t *cand_u, int32_t *cand_p, int32_t n_threads);

/* One MF stageOne (model/MF.py:62-94: BPR loss + decay x reg, backward,
 * torch.optim.Adam over the whole table) on a [n_rows, dim] host table whose
 * item rows start at item_offset (= n_users): grad is a [n_rows, dim]
 * workspace; *loss_out = loss + decay reg (the value stageOne returns).
 * MIREC_ERR_RANGE if an id is outside its table slice. */
int mirec_cpu_bpr_step(float *table, float *exp_avg, float *exp_avg_sq, float *grad,
                       int64_t n_rows, int32_t dim, int64_t item_offset, const int32_t *users,
                       const int32_t *pos, const int32_t *neg, int64_t batch, float decay,
                       const mirec_adam_hparams_t *h, float *loss_out, int32_t n_threads);

/* The two halves of mirec_cpu_bpr_step (bitwise the same arithmetic): the
 * dense gradient of one batch's loss + decay reg, multiplied by grad_scale
 * (1 / world_size under data parallelism; 1 = the step's), into grad
 * (*loss_out unscaled); then torch.optim.Adam over n elements. */
int mirec_cpu_bpr_grad(const float *table, float *grad, int64_t n_rows, int32_t dim,
                       int64_t item_offset, const int32_t *users, const int32_t *pos,
                       const int32_t *neg, int64_t batch, float decay, float grad_scale,
                       float *loss_out, int32_t n_threads);
int mirec_cpu_adam(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                   const mirec_adam_hparams_t *h, int32_t n_threads);

#ifdef __cplusplus
}
#endif

#endif /* MIREC_H */
