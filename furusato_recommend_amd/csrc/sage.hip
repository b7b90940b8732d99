// GraphSAGE hot ops on gfx950 (model/graphsage.py:311-324 + the samplers of
// neighbor_sampling.py:14-30 / PyG NeighborSampler at graphsage.py:342-365).
//
// Sampling is fixed-fanout WITH replacement (the repo's uniform_neighbors),
// so every hop is a regular tree: level l+1 holds k children per level-l
// node, contiguous.  That turns PyG's scatter-mean over a sampled edge_index
// into a fixed-width segment mean — no CSR, no atomics in the forward.
//
//   mirec_sample_fanout   children[t*k + c] ~ U(CSR row of nodes[t]); -1 if
//                         the node has no neighbours (its mean is then 0)
//   mirec_gather_rows     out[i] = table[ids[i]] (0 for ids < 0)
//   mirec_scatter_add_rows  grad_table[ids[i]] += grad[i] (float atomics:
//                         the backward of the gather)
//   mirec_fanout_mean     out[t] = mean over valid c of dropout(x[t*k + c])
//   mirec_fanout_mean_bwd grad_x[t*k + c] = mask * grad_out[t] / cnt
//   mirec_fanout_mean_gather(_bwd)  the same with child rows gathered from
//                         the table by id (leaf hop: no materialised rows;
//                         backward scatter-adds into the table gradient)
// Dropout masks are a counter hash of (seed, element index), recomputed in
// the backward (nothing stored).
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace mirec {

__global__ __launch_bounds__(256) void sample_fanout_kernel(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col, int64_t n_rows,
    const int32_t *__restrict__ nodes, int64_t n, int32_t k, uint64_t seed, uint64_t offset,
    int32_t *__restrict__ children) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * k) return;
  const int64_t t = i / k;
  const int32_t v = nodes[t];
  int32_t out = -1;
  if (v >= 0 && v < n_rows) {
    const int64_t beg = rowptr[v], deg = rowptr[v + 1] - beg;
    if (deg > 0) {
      const uint64_t r = mix64(mix64(seed) ^ (offset + (uint64_t)i));
      out = col[beg + (int64_t)__umul64hi(r, (uint64_t)deg)];
    }
  }
  children[i] = out;
}

// Without replacement (PyG NeighborSampler's default, the sampler of
// model/graphsage.py:342-365): a node with deg <= k keeps all its entries
// (row order; the remaining slots are -1), otherwise k distinct entries by
// Floyd's algorithm (the chosen positions are kept in the output row itself
// while drawing, then mapped to node ids).  One thread per target node.
__global__ __launch_bounds__(256) void sample_fanout_norep_kernel(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col, int64_t n_rows,
    const int32_t *__restrict__ nodes, int64_t n, int32_t k, uint64_t seed, uint64_t offset,
    int32_t *__restrict__ children) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  int32_t *out = children + t * k;
  const int32_t v = nodes[t];
  const int64_t beg = (v >= 0 && v < n_rows) ? rowptr[v] : 0;
  const int64_t deg = (v >= 0 && v < n_rows) ? rowptr[v + 1] - beg : 0;
  if (deg <= k) {
    for (int c = 0; c < k; ++c) out[c] = c < deg ? col[beg + c] : -1;
    return;
  }
  const uint64_t key = mix64(seed);
  int m = 0;
  for (int64_t j = deg - k; j < deg; ++j, ++m) {
    const uint64_t r64 = mix64(key ^ (offset + (uint64_t)(t * k + m)));
    int32_t r = (int32_t)__umul64hi(r64, (uint64_t)(j + 1));  // uniform in [0, j]
    for (int q = 0; q < m; ++q)
      if (out[q] == r) {
        r = (int32_t)j;
        break;
      }
    out[m] = r;
  }
  for (int c = 0; c < k; ++c) out[c] = col[beg + out[c]];
}

// The same draws (same counter stream, same Floyd positions) with the chosen
// positions held in registers: k <= KMAX, the draw loop unrolled so the
// membership test is a chain of compares against earlier registers instead
// of re-reading the output row from global memory (the k (k-1) / 2 dependent
// loads per target made the 6144 x 25 root hop latency-bound: 67 us), and
// the k column loads of the final mapping issued together.
template <int KMAX>
__global__ __launch_bounds__(256) void sample_fanout_norep_reg_kernel(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col, int64_t n_rows,
    const int32_t *__restrict__ nodes, int64_t n, int32_t k, uint64_t seed, uint64_t offset,
    int32_t *__restrict__ children) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  int32_t *out = children + t * k;
  const int32_t v = nodes[t];
  const int64_t beg = (v >= 0 && v < n_rows) ? rowptr[v] : 0;
  const int64_t deg = (v >= 0 && v < n_rows) ? rowptr[v + 1] - beg : 0;
  int32_t sel[KMAX];
  if (deg <= k) {
#pragma unroll
    for (int c = 0; c < KMAX; ++c)
      if (c < k) sel[c] = c < deg ? col[beg + c] : -1;
  } else {
    const uint64_t key = mix64(seed);
#pragma unroll
    for (int m = 0; m < KMAX; ++m) {
      if (m < k) {
        const int64_t j = deg - k + m;
        const uint64_t r64 = mix64(key ^ (offset + (uint64_t)(t * k + m)));
        int32_t r = (int32_t)__umul64hi(r64, (uint64_t)(j + 1));  // uniform in [0, j]
        bool hit = false;
#pragma unroll
        for (int q = 0; q < m; ++q) hit |= sel[q] == r;
        sel[m] = hit ? (int32_t)j : r;
      }
    }
#pragma unroll
    for (int c = 0; c < KMAX; ++c)
      if (c < k) sel[c] = col[beg + sel[c]];
  }
#pragma unroll
  for (int c = 0; c < KMAX; ++c)
    if (c < k) out[c] = sel[c];
}

// out[r, :] = table[ids[r], :] (zeros for an id < 0); the row-mover shape
// of common.h
__global__ __launch_bounds__(256) void gather_rows_kernel(const float4 *__restrict__ table,
                                                          const int32_t *__restrict__ ids, int64_t n,
                                                          int32_t d4, int32_t lg,
                                                          float4 *__restrict__ out) {
  const int per = 256 >> lg;
  const int c = threadIdx.x & ((1 << lg) - 1);
  const int64_t r0 = (int64_t)blockIdx.x * per * kRowRounds + (threadIdx.x >> lg);
  const bool col = c < d4;
  int32_t id[kRowRounds];
#pragma unroll
  for (int k = 0; k < kRowRounds; ++k) id[k] = r0 + k * per < n ? ids[r0 + k * per] : -1;
  float4 x[kRowRounds];
#pragma unroll
  for (int k = 0; k < kRowRounds; ++k)
    x[k] = (col && id[k] >= 0) ? table[(int64_t)id[k] * d4 + c] : f4_zero();
#pragma unroll
  for (int k = 0; k < kRowRounds; ++k)
    if (col && r0 + k * per < n) out[(r0 + k * per) * d4 + c] = x[k];
}

__global__ __launch_bounds__(256) void scatter_add_rows_kernel(const float *__restrict__ grad,
                                                               const int32_t *__restrict__ ids,
                                                               int64_t n, int32_t d,
                                                               float *__restrict__ table_grad) {
  // one wave-instruction = 64 consecutive floats of one row (256 B): the
  // full-rate shape for global float atomics on gfx950
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * d) return;
  const int64_t r = i / d;
  const int32_t id = ids[r];
  if (id < 0) return;
  atomicAdd(table_grad + (int64_t)id * d + (i - r * d), grad[i]);
}

// one thread per (target, float4 column).  GATHER: child rows are
// table[valid[child]] (fused row gather, nothing materialised), else x rows.
template <bool GATHER>
__global__ __launch_bounds__(256) void fanout_mean_kernel(
    const float *__restrict__ x, const int32_t *__restrict__ valid, int64_t n_targets, int32_t k,
    int32_t d4, uint64_t key, uint32_t thresh, float scale, float *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_targets * d4) return;
  const int64_t t = i / d4;
  const int64_t c4 = i - t * d4;
  const int64_t d = (int64_t)d4 * 4;
  float4 acc = f4_zero();
  int cnt = 0;
  // children in batches of kFmBatch: every id, then every row of the batch
  // in flight at once (not one dependent id -> row round trip per child),
  // then masked and added in child order (the same sum as one at a time)
  constexpr int kFmBatch = 8;
  for (int c0 = 0; c0 < k; c0 += kFmBatch) {
    int32_t vid[kFmBatch];
#pragma unroll
    for (int u = 0; u < kFmBatch; ++u)
      vid[u] = (c0 + u < k && valid != nullptr) ? valid[t * k + c0 + u] : 0;
    float4 v[kFmBatch];
#pragma unroll
    for (int u = 0; u < kFmBatch; ++u) {
      const int64_t child = t * k + c0 + u;
      const bool ok = c0 + u < k && vid[u] >= 0;
      const int64_t row = GATHER ? (int64_t)vid[u] : child;
      v[u] = ok ? ld4(x + row * d + c4 * 4) : f4_zero();
    }
#pragma unroll
    for (int u = 0; u < kFmBatch; ++u) {
      const int64_t child = t * k + c0 + u;
      if (c0 + u < k && vid[u] >= 0) {
        ++cnt;
        float4 w = v[u];
        if (thresh != 0u) w = drop4(w, key, (uint64_t)(child * d + c4 * 4), thresh, scale);
        acc = f4_add(acc, w);
      }
    }
  }
  st4(out + i * 4, cnt > 0 ? f4_div(acc, (float)cnt) : f4_zero());
}

__global__ __launch_bounds__(256) void fanout_mean_bwd_kernel(
    const float *__restrict__ grad_out, const int32_t *__restrict__ valid, int64_t n_targets,
    int32_t k, int32_t d4, uint64_t key, uint32_t thresh, float scale,
    float *__restrict__ grad_x) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (child, float4)
  if (i >= n_targets * k * d4) return;  // whole d4-lane groups leave together
  const int64_t child = i / d4;
  const int64_t c4 = i - child * d4;
  const int64_t t = child / k;
  const int64_t d = (int64_t)d4 * 4;
  // valid children of target t: the d4 lanes of this child's group read the
  // k flags d4 at a time and count them by ballot (d4 a power of two <= 64,
  // so the groups are aligned inside the wave), instead of every lane
  // loading all k flags
  int cnt = k;
  if (valid != nullptr) {
    cnt = 0;
    if (d4 <= 64 && (d4 & (d4 - 1)) == 0) {
      const int lane = threadIdx.x & 63;
      const int gbase = lane & ~(d4 - 1);
      const unsigned long long gmask = (d4 == 64 ? ~0ull : ((1ull << d4) - 1ull)) << gbase;
      for (int j0 = 0; j0 < k; j0 += d4) {
        const int j = j0 + (int)c4;
        cnt += __popcll(__ballot(j < k && valid[t * k + j] >= 0) & gmask);
      }
    } else {
      for (int c = 0; c < k; ++c) cnt += valid[t * k + c] >= 0 ? 1 : 0;
    }
  }
  float4 g = f4_zero();
  if (valid == nullptr || valid[child] >= 0) {
    g = f4_div(ld4(grad_out + t * d + c4 * 4), (float)cnt);
    if (thresh != 0u) {
      g = drop4(g, key, (uint64_t)(child * d + c4 * 4), thresh, scale);
    }
  }
  st4(grad_x + i * 4, g);
}

// Backward of the fused gather + mean: table_grad[ids[child]] += mask *
// grad_out[t] / cnt.  One wave per target: the k child ids are read once
// (cnt by ballot), grad_out[t] stays in registers, and every valid child's
// row is added with one wave-instruction per 64 consecutive floats (the
// full-rate atomic shape).  Dropout element index = child * d + col, as in
// the unfused path.
__global__ __launch_bounds__(256) void fanout_mean_gather_bwd_kernel(
    const float *__restrict__ grad_out, const int32_t *__restrict__ ids, int64_t n_targets,
    int32_t k, int32_t d, uint64_t key, uint32_t thresh, float scale,
    float *__restrict__ table_grad) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (t >= n_targets) return;
  const int32_t myid = lane < k ? ids[t * k + lane] : -1;  // k <= 64 (checked on host)
  const unsigned long long valid = __ballot(myid >= 0);
  const int cnt = __popcll(valid);
  if (cnt == 0) return;
  const float inv = 1.f / (float)cnt;
  for (int c0 = 0; c0 < d; c0 += 64) {
    const int col = c0 + lane;
    const float g = col < d ? grad_out[t * d + col] * inv : 0.f;
    for (int c = 0; c < k; ++c) {
      if (!((valid >> c) & 1ull)) continue;  // wave-uniform
      const int32_t id = __shfl(myid, c);
      if (col < d) {
        float x = g;
        if (thresh != 0u)
          x = keep(key, (uint64_t)((t * k + c) * (int64_t)d + col), thresh) ? x * scale : 0.f;
        atomicAdd(table_grad + (int64_t)id * d + col, x);
      }
    }
  }
}

// Sorted form of the same backward (deterministic, no atomics): the leaf
// entries e = t*k + c are radix-sorted by child id (stable, so each id's
// entries stay in e order), then every run of equal ids is summed — mask *
// grad_out[t] / cnt_t, in that order — by exactly one wave and added to the
// id's row once.  Invalid entries (id < 0) sort to the key n_rows, last.
__global__ __launch_bounds__(256) void fanout_sort_prep_kernel(const int32_t *__restrict__ ids,
                                                               int64_t n_targets, int32_t k,
                                                               int32_t n_rows,
                                                               int32_t *__restrict__ keys,
                                                               int32_t *__restrict__ vals,
                                                               float *__restrict__ inv_cnt) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n_targets * k) {
    const int32_t id = ids[e];
    keys[e] = id >= 0 ? id : n_rows;
    vals[e] = (int32_t)e;
  }
  if (e < n_targets) {
    int cnt = 0;
    for (int c = 0; c < k; ++c) cnt += ids[e * k + c] >= 0 ? 1 : 0;
    inv_cnt[e] = cnt > 0 ? 1.f / (float)cnt : 0.f;
  }
}

// One wave per chunk of 64 sorted entries; a run belongs to the chunk that
// holds its head, and its owner keeps reading past the chunk end while the
// run continues.  Keys / entry ids / 1/cnt are loaded 64 at a time
// (coalesced) and broadcast with readlane; each lane sums 4 columns (d % 4
// == 0), with kSortBatch grad_out rows in flight before they are added in
// order.
constexpr int kSortBatch = 8;

__global__ __launch_bounds__(256) void fanout_sorted_sum_kernel(
    const float *__restrict__ grad_out, const int32_t *__restrict__ keys,
    const int32_t *__restrict__ vals, const float *__restrict__ inv_cnt, int64_t n, int32_t k,
    int32_t d, int32_t n_rows, uint64_t key, uint32_t thresh, float scale,
    float *__restrict__ table_grad) {
  constexpr int32_t kEnd = 0x7fffffff;  // key past the last entry
  const int lane = threadIdx.x & 63;
  const int64_t base = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64;
  if (base >= n) return;
  const int64_t end = base + 64 < n ? base + 64 : n;
  int64_t pos = base;
  if (base > 0) {  // skip the tail of a run whose head is in an earlier chunk
    const int32_t prev = keys[base - 1];
    const int32_t kl = base + lane < n ? keys[base + lane] : kEnd;
    const unsigned long long diff = __ballot(kl != prev);
    if (diff == 0ull) return;
    pos = base + (int64_t)__builtin_ctzll(diff);
  }
  if (pos >= end) return;
  const int32_t first = keys[pos];
  if (first >= n_rows) return;  // only invalid entries from here on
  for (int c0 = 0; c0 < d; c0 += 256) {
    const int col = c0 + 4 * lane;
    const bool act = col < d;
    int32_t cur = first;
    float4 acc = f4_zero();
    bool done = false;
    for (int64_t p = pos; !done; p += 64) {
      const int64_t j = p + lane;
      const int32_t kb = j < n ? keys[j] : kEnd;
      const int32_t vb = j < n ? vals[j] : 0;
      const float ib = inv_cnt[vb / k];
      for (int m0 = 0; m0 < 64 && !done; m0 += kSortBatch) {
        float4 x[kSortBatch];
        int32_t kk[kSortBatch], ee[kSortBatch];
#pragma unroll
        for (int u = 0; u < kSortBatch; ++u) {
          kk[u] = __builtin_amdgcn_readlane(kb, m0 + u);
          ee[u] = __builtin_amdgcn_readlane(vb, m0 + u);
          const float iv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ib), m0 + u));
          const int64_t t = ee[u] / k;
          x[u] = act ? f4_scale(iv, ld4(grad_out + t * d + col)) : f4_zero();
        }
#pragma unroll
        for (int u = 0; u < kSortBatch; ++u) {
          if (kk[u] != cur) {  // wave-uniform: the run `cur` ends here
            if (act) {
              float *row = table_grad + (int64_t)cur * d + col;
              st4(row, f4_add(ld4(row), acc));
            }
            if (p + m0 + u >= end || kk[u] >= n_rows) {
              done = true;
              break;
            }
            cur = kk[u];
            acc = f4_zero();
          }
          float4 v = x[u];
          if (thresh != 0u) {
            v = drop4(v, key, (uint64_t)((int64_t)ee[u] * d + col), thresh, scale);
          }
          acc = f4_add(acc, v);
        }
      }
    }
  }
}

// Workspace layout of the sorted backward: keys / vals in and out (int32),
// inv_cnt (float), then the radix sort's temporary storage.
static size_t fanout_sorted_layout(int64_t n_targets, int32_t k, int32_t n_rows,
                                   size_t *sort_off, size_t *sort_bytes, int *end_bit) {
  const int64_t n = n_targets * k;
  const auto up = [](size_t b) { return (b + 255) / 256 * 256; };
  size_t off = 4 * up(sizeof(int32_t) * n) + up(sizeof(float) * n_targets);
  int bits = 1;
  while (bits < 31 && ((int64_t)1 << bits) <= n_rows) ++bits;
  size_t tb = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (int32_t *)nullptr, (int32_t *)nullptr,
                                           (int32_t *)nullptr, (int32_t *)nullptr, (int)n, 0,
                                           bits);
  *sort_off = off;
  *sort_bytes = tb;
  *end_bit = bits;
  return off + up(tb);
}

}  // namespace mirec

extern "C" int mirec_fanout_mean_gather_bwd_sorted_workspace(int64_t n_targets, int32_t k,
                                                             int32_t n_rows, size_t *bytes) {
  using namespace mirec;
  MIREC_CHECK_ARG(bytes && n_targets >= 0 && k > 0 && n_rows > 0 &&
                  n_targets * (int64_t)k < ((int64_t)1 << 31));
  size_t so, sb;
  int eb;
  *bytes = fanout_sorted_layout(n_targets, k, n_rows, &so, &sb, &eb);
  return MIREC_OK;
}

extern "C" int mirec_fanout_mean_gather_bwd_sorted(const float *grad_out, const int32_t *ids,
                                                   int64_t n_targets, int32_t k, int32_t dim,
                                                   float dropout_p, uint64_t seed,
                                                   int32_t n_rows, float *table_grad,
                                                   void *workspace, size_t workspace_bytes,
                                                   mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(table_grad && n_targets >= 0 && k > 0 && dim > 0 && dim % 4 == 0 &&
                  n_rows > 0 && n_targets * (int64_t)k < ((int64_t)1 << 31));
  uint64_t key;
  uint32_t thresh;
  float scale;
  MIREC_CHECK_ARG(dropout_params(dropout_p, seed, &key, &thresh, &scale));
  if (n_targets == 0) return MIREC_OK;
  MIREC_CHECK_ARG(grad_out && ids && workspace);
  size_t sort_off, sort_bytes;
  int end_bit;
  const size_t need = fanout_sorted_layout(n_targets, k, n_rows, &sort_off, &sort_bytes, &end_bit);
  if (workspace_bytes < need) return MIREC_ERR_WORKSPACE;
  const int64_t n = n_targets * k;
  const size_t seg = (sizeof(int32_t) * n + 255) / 256 * 256;
  char *ws = static_cast<char *>(workspace);
  int32_t *keys_in = reinterpret_cast<int32_t *>(ws);
  int32_t *keys_out = reinterpret_cast<int32_t *>(ws + seg);
  int32_t *vals_in = reinterpret_cast<int32_t *>(ws + 2 * seg);
  int32_t *vals_out = reinterpret_cast<int32_t *>(ws + 3 * seg);
  float *inv_cnt = reinterpret_cast<float *>(ws + 4 * seg);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(fanout_sort_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     st, ids, n_targets, k, n_rows, keys_in, vals_in, inv_cnt);
  MIREC_LAUNCH_CHECK();
  MIREC_HIP(hipcub::DeviceRadixSort::SortPairs(ws + sort_off, sort_bytes, keys_in, keys_out,
                                               vals_in, vals_out, (int)n, 0, end_bit, st));
  const int64_t chunks = (n + 63) / 64;  // one wave per 64 sorted entries
  hipLaunchKernelGGL(fanout_sorted_sum_kernel, dim3((unsigned)((chunks + 3) / 4)), dim3(256), 0, st,
                     grad_out, keys_out, vals_out, inv_cnt, n, k, dim, n_rows, key, thresh, scale,
                     table_grad);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}


extern "C" int mirec_sample_fanout(const mirec_csr_t *csr, const int32_t *nodes, int64_t n,
                                   int32_t k, uint64_t seed, uint64_t offset, int32_t *children,
                                   mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(csr && csr->rowptr && csr->col && nodes && children && n >= 0 && k > 0);
  if (n == 0) return MIREC_OK;
  const int64_t tot = n * k;
  hipLaunchKernelGGL(sample_fanout_kernel, dim3((tot + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), csr->rowptr, csr->col, csr->n_rows,
                     nodes, n, k, seed, offset, children);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_sample_fanout_norep(const mirec_csr_t *csr, const int32_t *nodes, int64_t n,
                                         int32_t k, uint64_t seed, uint64_t offset,
                                         int32_t *children, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(csr && csr->rowptr && csr->col && nodes && children && n >= 0 && k > 0);
  if (n == 0) return MIREC_OK;
  const dim3 grid((unsigned)((n + 255) / 256));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define MIREC_NOREP(KM)                                                                         \
  hipLaunchKernelGGL(sample_fanout_norep_reg_kernel<KM>, grid, dim3(256), 0, st, csr->rowptr,  \
                     csr->col, csr->n_rows, nodes, n, k, seed, offset, children)
  if (k <= 8) MIREC_NOREP(8);
  else if (k <= 16) MIREC_NOREP(16);
  else if (k <= 32) MIREC_NOREP(32);
  else
    hipLaunchKernelGGL(sample_fanout_norep_kernel, grid, dim3(256), 0, st, csr->rowptr, csr->col,
                       csr->n_rows, nodes, n, k, seed, offset, children);
#undef MIREC_NOREP
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_gather_rows(const float *table, const int32_t *ids, int64_t n, int32_t dim,
                                 float *out, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(table && ids && out && n >= 0 && dim > 0 && dim % 4 == 0);
  if (n == 0) return MIREC_OK;
  MIREC_CHECK_ARG(((uintptr_t)table & 15u) == 0 && ((uintptr_t)out & 15u) == 0);
  const int lg = row_lg(dim / 4);
  MIREC_CHECK_ARG(lg <= 8);
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)row_blocks(n, lg)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float4 *>(table),
                     ids, n, dim / 4, lg, reinterpret_cast<float4 *>(out));
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_scatter_add_rows(const float *grad, const int32_t *ids, int64_t n,
                                      int32_t dim, float *table_grad, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(grad && ids && table_grad && n >= 0 && dim > 0);
  if (n == 0) return MIREC_OK;
  const int64_t tot = n * dim;
  hipLaunchKernelGGL(scatter_add_rows_kernel, dim3((tot + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), grad, ids, n, dim, table_grad);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_fanout_mean(const float *x, const int32_t *valid, int64_t n_targets,
                                 int32_t k, int32_t dim, float dropout_p, uint64_t seed,
                                 float *out, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(x && out && n_targets >= 0 && k > 0 && dim > 0 && dim % 4 == 0);
  uint64_t key;
  uint32_t thresh;
  float scale;
  MIREC_CHECK_ARG(dropout_params(dropout_p, seed, &key, &thresh, &scale));
  if (n_targets == 0) return MIREC_OK;
  const int64_t tot = n_targets * (dim / 4);
  hipLaunchKernelGGL(fanout_mean_kernel<false>, dim3((tot + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), x, valid, n_targets, k, dim / 4, key,
                     thresh, scale, out);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_fanout_mean_bwd(const float *grad_out, const int32_t *valid,
                                     int64_t n_targets, int32_t k, int32_t dim, float dropout_p,
                                     uint64_t seed, float *grad_x, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(grad_out && grad_x && n_targets >= 0 && k > 0 && dim > 0 && dim % 4 == 0);
  uint64_t key;
  uint32_t thresh;
  float scale;
  MIREC_CHECK_ARG(dropout_params(dropout_p, seed, &key, &thresh, &scale));
  if (n_targets == 0) return MIREC_OK;
  const int64_t tot = n_targets * k * (dim / 4);
  hipLaunchKernelGGL(fanout_mean_bwd_kernel, dim3((tot + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), grad_out, valid, n_targets, k,
                     dim / 4, key, thresh, scale, grad_x);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_fanout_mean_gather(const float *table, const int32_t *ids, int64_t n_targets,
                                        int32_t k, int32_t dim, float dropout_p, uint64_t seed,
                                        float *out, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(table && ids && out && n_targets >= 0 && k > 0 && dim > 0 && dim % 4 == 0);
  uint64_t key;
  uint32_t thresh;
  float scale;
  MIREC_CHECK_ARG(dropout_params(dropout_p, seed, &key, &thresh, &scale));
  if (n_targets == 0) return MIREC_OK;
  const int64_t tot = n_targets * (dim / 4);
  hipLaunchKernelGGL(fanout_mean_kernel<true>, dim3((tot + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), table, ids, n_targets, k, dim / 4,
                     key, thresh, scale, out);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_fanout_mean_gather_bwd(const float *grad_out, const int32_t *ids,
                                            int64_t n_targets, int32_t k, int32_t dim,
                                            float dropout_p, uint64_t seed, float *table_grad,
                                            mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(grad_out && ids && table_grad && n_targets >= 0 && k > 0 && dim > 0 &&
                  dim % 4 == 0);
  uint64_t key;
  uint32_t thresh;
  float scale;
  MIREC_CHECK_ARG(dropout_params(dropout_p, seed, &key, &thresh, &scale));
  if (n_targets == 0) return MIREC_OK;
  MIREC_CHECK_ARG(k <= 64);
  const int64_t tot = n_targets;  // one wave per target, 4 per block
  hipLaunchKernelGGL(fanout_mean_gather_bwd_kernel, dim3((tot + 3) / 4), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), grad_out, ids, n_targets, k, dim,
                     key, thresh, scale, table_grad);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

// Seed node ids of a BPR batch for the GraphSAGE tree: out = [users ;
// n_users + pos ; n_users + neg] (graphsage.py:326-337's user / item rows of
// the one id table), one launch.
__global__ __launch_bounds__(256) void pack_seed_nodes_kernel(const int32_t *__restrict__ users,
                                                              const int32_t *__restrict__ pos,
                                                              const int32_t *__restrict__ neg,
                                                              int64_t B, int64_t n_users,
                                                              int32_t *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * B) return;
  const int64_t part = i / B, j = i - part * B;
  out[i] = part == 0 ? users[j] : (int32_t)(n_users + (part == 1 ? pos[j] : neg[j]));
}

extern "C" int mirec_pack_seed_nodes(const int32_t *users, const int32_t *pos, const int32_t *neg,
                                     int64_t batch, int64_t n_users, int32_t *out,
                                     mirec_stream_t stream) {
  MIREC_CHECK_ARG(batch >= 0 && n_users >= 0 && n_users < INT32_MAX);
  if (batch == 0) return MIREC_OK;
  MIREC_CHECK_ARG(users && pos && neg && out);
  hipLaunchKernelGGL(pack_seed_nodes_kernel, dim3((unsigned)((3 * batch + 255) / 256)), dim3(256),
                     0, (hipStream_t)stream, users, pos, neg, batch, n_users, out);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}
