// Frontier bitmaps for pruned propagation.
//
// The BPR loss of a batch reads the layer-mean embedding only at the batch's
// nodes S (users, pos items, neg items; model/lgcn.py:88-96).  With L layers,
// layer L's output is needed only on S and layer L-1's only on
// F1 = S ∪ N(S); symmetrically the backward seeds live on S, so the first
// backward layer's output is non-zero only on F1.  This launch builds the
// two byte maps (1 byte per node, 1.1 MB at C2: L2-resident) from a key list
// or directly from the triples:
//   bm_self = S,  bm_hop = S ∪ N(S)
// One lane per key sets S membership with a 32-bit atomicOr, so the first
// setter appends the node to the deduplicated S list (one list atomic per
// block); then one wave per S node expands its CSR row with plain byte stores
// (idempotent: no atomics).  Rows longer than the CSR split are expanded by
// one wave per segment, so a hot item does not serialise the launch.
// mirec_mask_compact turns a byte map (F1) into a row list for the masked
// propagation launches.
#include <algorithm>

#include "common.h"

namespace mirec {

constexpr int kWaves = 4;

// Sets byte i of a byte map with a word atomicOr; true if this call set it.
__device__ __forceinline__ bool test_and_set(uint8_t *bm, int64_t i) {
  const uint32_t b = 1u << (8 * (i & 3));
  return (atomicOr(reinterpret_cast<uint32_t *>(bm) + (i >> 2), b) & b) == 0u;
}

// Reserves c list entries for this thread in a 256-thread block: one
// atomicAdd per block on `count` (not one per entry: same-address atomics
// serialise in one L2 channel).  Returns this thread's first offset; entries
// keep thread order inside the block.  Every thread of the block must call.
__device__ __forceinline__ int32_t block_reserve(int c, int32_t *count) {
  __shared__ int wsum[kWaves];
  __shared__ int base;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();  // a previous call's readers are done with wsum / base
  int incl = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(incl, d);
    if (lane >= d) incl += t;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) t += wsum[k];
    base = t > 0 ? atomicAdd(count, t) : 0;
  }
  __syncthreads();
  int off = base + incl - c;
  for (int k = 0; k < wid; ++k) off += wsum[k];
  return off;
}

__device__ __forceinline__ int64_t key_node(int64_t i, const int32_t *keys, int64_t n_keys,
                                            const int32_t *users, const int32_t *pos,
                                            const int32_t *neg, int64_t batch, int64_t n_users) {
  if (keys != nullptr) return i < n_keys ? (int64_t)keys[i] : -1;
  if (i >= 3 * batch) return -1;
  return i < batch ? (int64_t)users[i]
                   : (i < 2 * batch ? n_users + pos[i - batch] : n_users + neg[i - 2 * batch]);
}

// One lane per key: S membership (first setter appends the node to the
// deduplicated S list) and the node's own bm_hop byte.
__global__ __launch_bounds__(256) void frontier_self_kernel(
    int64_t n_rows, const int32_t *__restrict__ keys, int64_t n_keys,
    const int32_t *__restrict__ users, const int32_t *__restrict__ pos,
    const int32_t *__restrict__ neg, int64_t batch, int64_t n_users, uint8_t *bm_self,
    uint8_t *bm_hop, int32_t *self_list, int32_t *self_count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t node = key_node(i, keys, n_keys, users, pos, neg, batch, n_users);
  const bool valid = node >= 0 && node < n_rows;  // empty / sentinel entries
  const bool first = valid && test_and_set(bm_self, node);
  if (valid) bm_hop[node] = 1;
  const int32_t off = block_reserve(first ? 1 : 0, self_count);
  if (first) self_list[off] = (int32_t)node;
}

// The step's clears in one launch: both byte maps (uint4 stores), the S
// count and the row-list counters the following mask_compact calls fill
// (four memset launches before, ~5 us each on the C2 step).
__global__ __launch_bounds__(256) void frontier_clear_kernel(uint4 *__restrict__ maps, int64_t n16,
                                                             int32_t *__restrict__ self_count,
                                                             int32_t *__restrict__ zero,
                                                             int32_t n_zero) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t j = i; j < n16; j += (int64_t)gridDim.x * blockDim.x) maps[j] = make_uint4(0, 0, 0, 0);
  if (i == 0 && self_count != nullptr) *self_count = 0;
  if (i < n_zero) zero[i] = 0;
}

// One wave per S node: its CSR row's neighbours into bm_hop with plain byte
// stores (idempotent, no atomics).
__global__ __launch_bounds__(256) void frontier_expand_kernel(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col, int32_t split,
    const int32_t *__restrict__ self_list, const int32_t *__restrict__ self_count,
    uint8_t *bm_hop) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (i >= *self_count) return;
  const int64_t node = self_list[i];
  const int64_t beg = rowptr[node], end = rowptr[node + 1];
  if (split > 0 && end - beg > split) return;  // expanded per segment
  for (int64_t e = beg + lane; e < end; e += 64) bm_hop[col[e]] = 1;
}

// Without an S list: one wave per key does both (duplicates re-expand).
__global__ __launch_bounds__(256) void frontier_keys_kernel(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col, int64_t n_rows,
    int32_t split, const int32_t *__restrict__ keys, int64_t n_keys,
    const int32_t *__restrict__ users, const int32_t *__restrict__ pos,
    const int32_t *__restrict__ neg, int64_t batch, int64_t n_users, uint8_t *bm_self,
    uint8_t *bm_hop) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int64_t node = key_node(i, keys, n_keys, users, pos, neg, batch, n_users);
  if (node < 0 || node >= n_rows) return;
  if (lane == 0) {
    bm_self[node] = 1;
    bm_hop[node] = 1;
  }
  const int64_t beg = rowptr[node], end = rowptr[node + 1];
  if (split > 0 && end - beg > split) return;
  for (int64_t e = beg + lane; e < end; e += 64) bm_hop[col[e]] = 1;
}

__global__ __launch_bounds__(256) void frontier_segments_kernel(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const int32_t *__restrict__ seg_row, const int64_t *__restrict__ seg_beg, int64_t n_seg,
    int32_t split, const uint8_t *bm_self, uint8_t *bm_hop) {
  const int lane = threadIdx.x & 63;
  const int64_t sg = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (sg >= n_seg) return;
  const int64_t row = seg_row[sg];
  if (bm_self[row] == 0) return;
  const int64_t beg = seg_beg[sg];
  const int64_t end = min(beg + (int64_t)split, rowptr[row + 1]);
  for (int64_t e = beg + lane; e < end; e += 64) bm_hop[col[e]] = 1;
}

// Byte map -> row lists (narrow / wide by degree), ascending within a block.
// Each thread tests 16 bytes (one 16-B load of four map words).
__global__ __launch_bounds__(256) void mask_compact_kernel(
    const uint8_t *__restrict__ bm, const int64_t *__restrict__ rowptr, int64_t n,
    int32_t narrow_max, int32_t *list, int32_t *count, int32_t *wide_list,
    int32_t *wide_count) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b0 = t * 16;
  uint32_t w[4] = {0u, 0u, 0u, 0u};
  if (b0 + 16 <= n) {
    const uint4 v = *reinterpret_cast<const uint4 *>(bm + b0);
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  } else if (b0 < n) {
    for (int k = 0; b0 + k < n; ++k)
      if (bm[b0 + k]) w[k >> 2] |= 1u << (8 * (k & 3));
  }
  uint32_t set = 0u, wide = 0u;  // bit k: byte k set / node k goes wide
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if ((w[k >> 2] >> (8 * (k & 3))) & 0xffu) {
      set |= 1u << k;
      if (wide_list != nullptr && rowptr[b0 + k + 1] - rowptr[b0 + k] > narrow_max)
        wide |= 1u << k;
    }
  }
  const uint32_t narrow = set & ~wide;
  int32_t off = block_reserve(__popc(narrow), count);
  int32_t woff = wide_list != nullptr ? block_reserve(__popc(wide), wide_count) : 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if ((narrow >> k) & 1u) list[off++] = (int32_t)(b0 + k);
    if ((wide >> k) & 1u) wide_list[woff++] = (int32_t)(b0 + k);
  }
}

// Both frontier maps of a step in one launch (S and F1 = S ∪ N(S)): a thread
// takes 32 nodes — 32 bytes of each map and one word of the static wide-row
// bitmap (degree > narrow_max, built once per graph) instead of a rowptr
// pair per set node — and the workgroup reserves its four runs (S narrow /
// wide, F1 narrow / wide) with one block scan and four atomics on adjacent
// counters (zeroed by mirec_frontier).  Two launches of mask_compact_kernel
// before: 2 x 11.6 us per C2 step, mostly ~270 same-address reservations
// per counter (8192 nodes per workgroup now: ~135).
__device__ __forceinline__ uint32_t map_bits32(const uint8_t *__restrict__ bm, int64_t b0,
                                               int64_t n) {
  uint32_t set = 0u;
  if (b0 + 32 <= n) {
    const uint4 v0 = *reinterpret_cast<const uint4 *>(bm + b0);
    const uint4 v1 = *reinterpret_cast<const uint4 *>(bm + b0 + 16);
    const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
    for (int k = 0; k < 32; ++k)
      if ((w[k >> 2] >> (8 * (k & 3))) & 0xffu) set |= 1u << k;
  } else {
    for (int k = 0; b0 + k < n; ++k)
      if (bm[b0 + k]) set |= 1u << k;
  }
  return set;
}

__global__ __launch_bounds__(256) void mask_compact_pair_kernel(
    const uint8_t *__restrict__ bm_a, const uint8_t *__restrict__ bm_b,
    const uint32_t *__restrict__ wide_bits, int64_t n, int32_t *__restrict__ list_a,
    int32_t *__restrict__ wide_a, int32_t *__restrict__ list_b, int32_t *__restrict__ wide_b,
    int32_t *__restrict__ counts) {
  __shared__ int4 wsum[kWaves];
  __shared__ int4 base;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b0 = t * 32;
  uint32_t sa = 0u, sb = 0u, wd = 0u;
  if (b0 < n) {
    sa = map_bits32(bm_a, b0, n);
    sb = map_bits32(bm_b, b0, n);
    wd = wide_bits[t];
  }
  const uint32_t na = sa & ~wd, wa = sa & wd, nb = sb & ~wd, wb = sb & wd;
  // one block scan of the four counts (entries keep thread order)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int4 c = make_int4(__popc(na), __popc(wa), __popc(nb), __popc(wb)), incl = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int x = __shfl_up(incl.x, d), y = __shfl_up(incl.y, d);
    const int z = __shfl_up(incl.z, d), w = __shfl_up(incl.w, d);
    if (lane >= d) incl = make_int4(incl.x + x, incl.y + y, incl.z + z, incl.w + w);
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    int4 tot = make_int4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < kWaves; ++k)
      tot = make_int4(tot.x + wsum[k].x, tot.y + wsum[k].y, tot.z + wsum[k].z, tot.w + wsum[k].w);
    base = make_int4(tot.x ? atomicAdd(counts, tot.x) : 0, tot.y ? atomicAdd(counts + 1, tot.y) : 0,
                     tot.z ? atomicAdd(counts + 2, tot.z) : 0,
                     tot.w ? atomicAdd(counts + 3, tot.w) : 0);
  }
  __syncthreads();
  int4 off = make_int4(base.x + incl.x - c.x, base.y + incl.y - c.y, base.z + incl.z - c.z,
                       base.w + incl.w - c.w);
  for (int k = 0; k < wid; ++k)
    off = make_int4(off.x + wsum[k].x, off.y + wsum[k].y, off.z + wsum[k].z, off.w + wsum[k].w);
#pragma unroll 4
  for (int k = 0; k < 32; ++k) {
    const int32_t v = (int32_t)(b0 + k);
    if ((na >> k) & 1u) list_a[off.x++] = v;
    if ((wa >> k) & 1u) wide_a[off.y++] = v;
    if ((nb >> k) & 1u) list_b[off.z++] = v;
    if ((wb >> k) & 1u) wide_b[off.w++] = v;
  }
}

// ------------------------------------------------ distinct rows of an id list
// The ascending distinct ids of ids[0 .. n) in [0, n_rows) outside [lo, hi):
// the rows a data-parallel rank must fetch from their owners before the
// GraphSAGE forward (dist.DenseGradDataParallel, fetch exchange).  Marked in
// a byte map (plain byte stores: idempotent), counted per 4096-row block,
// block offsets scanned, then each block writes its ids in order — globally
// ascending (so each owner's ids are one contiguous run), no sort, no host
// round trip (torch.unique sorted all n ids: 1.76 M at C3).
constexpr int kDrBlock = 4096;  // rows per workgroup (256 threads x 16 bytes)

__global__ __launch_bounds__(256) void dr_mark_kernel(const int32_t *__restrict__ ids, int64_t n,
                                                      int64_t n_rows, int64_t lo, int64_t hi,
                                                      const uint8_t *__restrict__ have,
                                                      uint8_t *__restrict__ bm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t id = ids[i];
  if (id >= 0 && id < n_rows && (id < lo || id >= hi) && (have == nullptr || !have[id]))
    bm[id] = 1;
}

// set-byte bit mask of the 16 map bytes of thread t of block b
__device__ __forceinline__ uint32_t dr_bits(const uint8_t *__restrict__ bm, int64_t n_rows,
                                            int64_t b0) {
  uint32_t w[4] = {0u, 0u, 0u, 0u};
  if (b0 + 16 <= n_rows) {
    const uint4 v = *reinterpret_cast<const uint4 *>(bm + b0);
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  } else {
    for (int k = 0; b0 + k < n_rows; ++k)
      if (bm[b0 + k]) w[k >> 2] |= 1u << (8 * (k & 3));
  }
  uint32_t set = 0u;
#pragma unroll
  for (int k = 0; k < 16; ++k)
    if ((w[k >> 2] >> (8 * (k & 3))) & 0xffu) set |= 1u << k;
  return set;
}

// exclusive prefix of c over the 256 threads of the block; total in *tot
__device__ __forceinline__ int dr_block_scan(int c, int *tot) {
  __shared__ int wsum[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int before = 0, all = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    before += k < w ? wsum[k] : 0;
    all += wsum[k];
  }
  *tot = all;
  return before + x - c;
}

__global__ __launch_bounds__(256) void dr_count_kernel(const uint8_t *__restrict__ bm,
                                                       int64_t n_rows, int32_t *__restrict__ cnt) {
  const int64_t b0 = (int64_t)blockIdx.x * kDrBlock + 16 * threadIdx.x;
  const int c = b0 < n_rows ? __popc(dr_bits(bm, n_rows, b0)) : 0;
  int tot;
  dr_block_scan(c, &tot);
  if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

// one workgroup: cnt[0 .. nb) -> exclusive offsets in place, total in *count
__global__ __launch_bounds__(256) void dr_scan_kernel(int32_t *__restrict__ cnt, int64_t nb,
                                                      int32_t *__restrict__ count) {
  int carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += 256) {
    const int64_t b = b0 + threadIdx.x;
    const int c = b < nb ? cnt[b] : 0;
    int tot;
    const int ex = dr_block_scan(c, &tot);
    __syncthreads();  // every lane has read cnt[] of this round
    if (b < nb) cnt[b] = carry + ex;
    carry += tot;
    __syncthreads();  // wsum reused by the next round
  }
  if (threadIdx.x == 0) *count = carry;
}

__global__ __launch_bounds__(256) void dr_write_kernel(const uint8_t *__restrict__ bm,
                                                       int64_t n_rows,
                                                       const int32_t *__restrict__ off,
                                                       int32_t *__restrict__ out,
                                                       uint8_t *__restrict__ have) {
  const int64_t b0 = (int64_t)blockIdx.x * kDrBlock + 16 * threadIdx.x;
  const uint32_t set = b0 < n_rows ? dr_bits(bm, n_rows, b0) : 0u;
  int tot;
  int o = off[blockIdx.x] + dr_block_scan(__popc(set), &tot);
#pragma unroll
  for (int k = 0; k < 16; ++k)
    if ((set >> k) & 1u) {
      out[o++] = (int32_t)(b0 + k);
      if (have != nullptr) have[b0 + k] = 1;
    }
}

// ------------------------------------------ the stamped rows of a table gradient
// The rows a micro-batch's sorted table gradient wrote (stamp == gen,
// graphsage.TableGrad) ascending, the count and the count per owner block,
// all on the device: the pipelined fetch exchange exports micro-batch k's
// rows with no host round trip and reads the counts one micro-batch later
// (dist.DenseGradDataParallel._route_chunk).  The byte map is the stamp
// comparison; count / scan / ordered writes are the distinct-rows kernels.
__global__ __launch_bounds__(256) void sr_mark_kernel(const int32_t *__restrict__ stamp,
                                                      int64_t n_rows, int32_t gen,
                                                      uint8_t *__restrict__ bm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_rows) bm[i] = stamp[i] == gen ? 1 : 0;
}

// counts[1 + q] = rows in owner block q (q·per .. (q+1)·per, the last block
// to n_rows): two lower bounds in the ascending rows[0 .. counts[0])
__device__ __forceinline__ int32_t sr_lower_bound(const int32_t *__restrict__ rows, int32_t n,
                                                  int64_t v) {
  int32_t a = 0, b = n;
  while (a < b) {
    const int32_t m = (a + b) >> 1;
    if ((int64_t)rows[m] < v) a = m + 1;
    else b = m;
  }
  return a;
}

__global__ __launch_bounds__(256) void sr_parts_kernel(const int32_t *__restrict__ rows,
                                                       int64_t n_rows, int32_t parts,
                                                       int32_t *__restrict__ counts) {
  const int n = counts[0];
  const int64_t per = n_rows / parts;
  for (int q = threadIdx.x; q < parts; q += blockDim.x) {
    const int64_t lo = q * per, hi = q == parts - 1 ? n_rows : (q + 1) * per;
    counts[1 + q] = sr_lower_bound(rows, n, hi) - sr_lower_bound(rows, n, lo);
  }
}

// out[i, :] = src[rows[i], :] for i < *count (read on the device); the
// row-mover shape of common.h over a grid sized for the capacity
__global__ __launch_bounds__(256) void gather_counted_kernel(const float4 *__restrict__ src,
                                                             const int32_t *__restrict__ rows,
                                                             const int32_t *__restrict__ count,
                                                             int32_t d4, int32_t lg,
                                                             float4 *__restrict__ out) {
  const int64_t n = count[0];
  const int per = 256 >> lg;
  const int c = threadIdx.x & ((1 << lg) - 1);
  const int64_t r0 = (int64_t)blockIdx.x * per * kRowRounds + (threadIdx.x >> lg);
  if (r0 >= n || c >= d4) return;
  int32_t id[kRowRounds];
#pragma unroll
  for (int k = 0; k < kRowRounds; ++k) id[k] = r0 + k * per < n ? rows[r0 + k * per] : -1;
  float4 x[kRowRounds];
#pragma unroll
  for (int k = 0; k < kRowRounds; ++k)
    x[k] = id[k] >= 0 ? src[(int64_t)id[k] * d4 + c] : f4_zero();
#pragma unroll
  for (int k = 0; k < kRowRounds; ++k)
    if (r0 + k * per < n) out[(r0 + k * per) * d4 + c] = x[k];
}

// dst[ids[i], :] = src[i, :] (ids distinct, < 0 skipped): the install of
// fetched rows into the local table; the row-mover shape of common.h
__global__ __launch_bounds__(256) void scatter_rows_kernel(const float4 *__restrict__ src,
                                                           const int32_t *__restrict__ ids,
                                                           int64_t n, int32_t d4, int32_t lg,
                                                           float4 *__restrict__ dst) {
  const int per = 256 >> lg;
  const int c = threadIdx.x & ((1 << lg) - 1);
  const int64_t r0 = (int64_t)blockIdx.x * per * kRowRounds + (threadIdx.x >> lg);
  if (c >= d4) return;
  int32_t id[kRowRounds];
  float4 x[kRowRounds];
#pragma unroll
  for (int k = 0; k < kRowRounds; ++k) {
    const int64_t r = r0 + k * per;
    id[k] = r < n ? ids[r] : -1;
    x[k] = r < n ? src[r * d4 + c] : f4_zero();
  }
#pragma unroll
  for (int k = 0; k < kRowRounds; ++k)
    if (id[k] >= 0) dst[(int64_t)id[k] * d4 + c] = x[k];
}

// ------------------------------------------ capacity-bounded read-set routing
// A micro-batch's read set (ascending ids, its count on the device) as one
// fixed-capacity block per owner: block q at blocks + q·stride holds
// [count_q, the ids of owner block q, unused up to cap].  The id all-to-all
// then runs with equal splits and the counts travel in-band, so the planner
// of the pipelined fetch exchange (dist.DenseGradDataParallel._plan_fetch)
// enqueues every micro-batch's routing without reading a count on the host.
constexpr int kRouteMaxParts = 256;

__global__ __launch_bounds__(256) void rp_pack_kernel(const int32_t *__restrict__ ids,
                                                      const int32_t *__restrict__ count,
                                                      int64_t n_rows, int32_t parts, int32_t cap,
                                                      int64_t stride, int32_t *__restrict__ blocks) {
  __shared__ int32_t start[kRouteMaxParts + 1];
  const int32_t n = count[0];
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  if (blockIdx.x > 0 && i0 >= n) return;  // (whole block: no barrier below is reached)
  const int64_t per = n_rows / parts;
  for (int q = threadIdx.x; q <= parts; q += blockDim.x)
    start[q] = q == parts ? n : sr_lower_bound(ids, n, q * per);
  __syncthreads();
  if (blockIdx.x == 0)
    for (int q = threadIdx.x; q < parts; q += blockDim.x) blocks[q * stride] = start[q + 1] - start[q];
  for (int64_t i = i0 + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t id = ids[i];
    const int q = (int)min<int64_t>(id / per, parts - 1);
    const int64_t pos = i - start[q];
    if (pos < cap) blocks[q * stride + 1 + pos] = id;
  }
}

// The owner side: out = the rows of table for the ids of the received
// blocks, in source order (block q's rows at Σ_{p<q} min(count_p, cap)), on
// a grid sized for the capacity; rows past the total, and ids outside
// [0, n_rows) (zeros written), touch no table memory.
__global__ __launch_bounds__(256) void rp_gather_kernel(const float4 *__restrict__ table,
                                                        int64_t n_rows,
                                                        const int32_t *__restrict__ blocks,
                                                        int32_t parts, int32_t cap, int64_t stride,
                                                        int32_t d4, int32_t lg,
                                                        float4 *__restrict__ out) {
  __shared__ int32_t off[kRouteMaxParts + 1];
  if (threadIdx.x == 0) {
    int32_t s = 0;
    for (int q = 0; q < parts; ++q) {
      off[q] = s;
      s += min(max(blocks[q * stride], 0), cap);
    }
    off[parts] = s;
  }
  __syncthreads();
  const int64_t total = off[parts];
  const int per = 256 >> lg;
  const int c = threadIdx.x & ((1 << lg) - 1);
  const int64_t r0 = (int64_t)blockIdx.x * per * kRowRounds + (threadIdx.x >> lg);
  if (r0 >= total || c >= d4) return;
  int32_t id[kRowRounds];
#pragma unroll
  for (int k = 0; k < kRowRounds; ++k) {
    const int64_t r = r0 + k * per;
    id[k] = -1;
    if (r < total) {
      int a = 0, b = parts;  // the last q with off[q] <= r
      while (b - a > 1) {
        const int m = (a + b) >> 1;
        if (off[m] <= r) a = m;
        else b = m;
      }
      const int32_t v = blocks[a * stride + 1 + (r - off[a])];
      id[k] = v >= 0 && v < n_rows ? v : -2;
    }
  }
  float4 x[kRowRounds];
#pragma unroll
  for (int k = 0; k < kRowRounds; ++k) x[k] = id[k] >= 0 ? table[(int64_t)id[k] * d4 + c] : f4_zero();
#pragma unroll
  for (int k = 0; k < kRowRounds; ++k)
    if (id[k] != -1) out[(r0 + k * per) * d4 + c] = x[k];
}

}  // namespace mirec

extern "C" int64_t mirec_distinct_rows_workspace(int64_t n_rows) {
  using namespace mirec;
  if (n_rows < 0) return -1;
  const int64_t map = (n_rows + 15) / 16 * 16;
  const int64_t nb = (n_rows + kDrBlock - 1) / kDrBlock;
  return map + 4 * (nb + 1);
}

extern "C" int mirec_distinct_rows(const int32_t *ids, int64_t n, int64_t n_rows, int64_t lo,
                                   int64_t hi, int32_t *out, int32_t *count, void *workspace,
                                   size_t workspace_bytes, mirec_stream_t stream) {
  return mirec_distinct_rows_unseen(ids, n, n_rows, lo, hi, nullptr, out, count, workspace,
                                 workspace_bytes, stream);
}

extern "C" int mirec_distinct_rows_unseen(const int32_t *ids, int64_t n, int64_t n_rows, int64_t lo,
                                       int64_t hi, uint8_t *have, int32_t *out, int32_t *count,
                                       void *workspace, size_t workspace_bytes,
                                       mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(n >= 0 && n_rows >= 0 && out && count && workspace);
  MIREC_CHECK_ARG(n == 0 || ids);
  MIREC_CHECK_ARG(((uintptr_t)workspace & 15u) == 0);
  const int64_t need = mirec_distinct_rows_workspace(n_rows);
  if ((int64_t)workspace_bytes < need) return MIREC_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  uint8_t *bm = static_cast<uint8_t *>(workspace);
  const int64_t map = (n_rows + 15) / 16 * 16;
  int32_t *cnt = reinterpret_cast<int32_t *>(bm + map);
  const int64_t nb = (n_rows + kDrBlock - 1) / kDrBlock;
  if (nb == 0) {
    MIREC_HIP(hipMemsetAsync(count, 0, 4, st));
    return MIREC_OK;
  }
  MIREC_HIP(hipMemsetAsync(bm, 0, (size_t)map, st));
  if (n > 0) {
    hipLaunchKernelGGL(dr_mark_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ids, n,
                       n_rows, lo, hi, have, bm);
    MIREC_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(dr_count_kernel, dim3((unsigned)nb), dim3(256), 0, st, bm, n_rows, cnt);
  MIREC_LAUNCH_CHECK();
  hipLaunchKernelGGL(dr_scan_kernel, dim3(1), dim3(256), 0, st, cnt, nb, count);
  MIREC_LAUNCH_CHECK();
  hipLaunchKernelGGL(dr_write_kernel, dim3((unsigned)nb), dim3(256), 0, st, bm, n_rows, cnt, out,
                     have);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_stamped_rows(const int32_t *stamp, int64_t n_rows, int32_t gen,
                                  int32_t parts, int32_t *rows, int32_t *counts, void *workspace,
                                  size_t workspace_bytes, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(n_rows >= 0 && parts >= 1 && rows && counts && workspace);
  MIREC_CHECK_ARG(n_rows == 0 || stamp);
  MIREC_CHECK_ARG(((uintptr_t)workspace & 15u) == 0);
  const int64_t need = mirec_distinct_rows_workspace(n_rows);
  if ((int64_t)workspace_bytes < need) return MIREC_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t nb = (n_rows + kDrBlock - 1) / kDrBlock;
  if (nb == 0) {
    MIREC_HIP(hipMemsetAsync(counts, 0, 4 * (size_t)(1 + parts), st));
    return MIREC_OK;
  }
  uint8_t *bm = static_cast<uint8_t *>(workspace);
  int32_t *cnt = reinterpret_cast<int32_t *>(bm + (n_rows + 15) / 16 * 16);
  hipLaunchKernelGGL(sr_mark_kernel, dim3((unsigned)((n_rows + 255) / 256)), dim3(256), 0, st,
                     stamp, n_rows, gen, bm);
  MIREC_LAUNCH_CHECK();
  hipLaunchKernelGGL(dr_count_kernel, dim3((unsigned)nb), dim3(256), 0, st, bm, n_rows, cnt);
  MIREC_LAUNCH_CHECK();
  hipLaunchKernelGGL(dr_scan_kernel, dim3(1), dim3(256), 0, st, cnt, nb, counts);
  MIREC_LAUNCH_CHECK();
  hipLaunchKernelGGL(dr_write_kernel, dim3((unsigned)nb), dim3(256), 0, st, bm, n_rows, cnt, rows,
                     nullptr);
  MIREC_LAUNCH_CHECK();
  hipLaunchKernelGGL(sr_parts_kernel, dim3(1), dim3(256), 0, st, rows, n_rows, parts, counts);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_gather_rows_counted(const float *src, const int32_t *rows,
                                         const int32_t *count, int64_t capacity, int32_t dim,
                                         float *out, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(capacity >= 0 && dim > 0 && dim % 4 == 0 && count);
  MIREC_CHECK_ARG(capacity == 0 || (src && rows && out));
  MIREC_CHECK_ARG(((uintptr_t)src & 15u) == 0 && ((uintptr_t)out & 15u) == 0);
  if (capacity == 0) return MIREC_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int lg = row_lg(dim / 4);
  MIREC_CHECK_ARG(lg <= 8);
  hipLaunchKernelGGL(gather_counted_kernel, dim3((unsigned)row_blocks(capacity, lg)), dim3(256), 0,
                     st, reinterpret_cast<const float4 *>(src), rows, count, dim / 4, lg,
                     reinterpret_cast<float4 *>(out));
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_route_pack(const int32_t *ids, const int32_t *count, int64_t capacity,
                                int64_t n_rows, int32_t parts, int32_t cap, int64_t stride,
                                int32_t *blocks, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(count && blocks && capacity >= 0 && n_rows >= 0 && cap >= 0);
  MIREC_CHECK_ARG(capacity == 0 || ids);
  MIREC_CHECK_ARG(parts >= 1 && parts <= kRouteMaxParts && stride >= (int64_t)cap + 1);
  MIREC_CHECK_ARG(n_rows >= parts);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t nb = std::min<int64_t>(std::max<int64_t>((capacity + 255) / 256, 1), 4096);
  hipLaunchKernelGGL(rp_pack_kernel, dim3((unsigned)nb), dim3(256), 0, st, ids, count, n_rows,
                     parts, cap, stride, blocks);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_gather_rows_routed(const float *table, int64_t n_rows, const int32_t *blocks,
                                        int32_t parts, int32_t cap, int64_t stride, int32_t dim,
                                        float *out, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(table && blocks && out && n_rows >= 0 && cap >= 0 && dim > 0 && dim % 4 == 0);
  MIREC_CHECK_ARG(parts >= 1 && parts <= kRouteMaxParts && stride >= (int64_t)cap + 1);
  MIREC_CHECK_ARG(((uintptr_t)table & 15u) == 0 && ((uintptr_t)out & 15u) == 0);
  const int64_t slots = (int64_t)parts * cap;
  if (slots == 0) return MIREC_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int lg = row_lg(dim / 4);
  MIREC_CHECK_ARG(lg <= 8);
  hipLaunchKernelGGL(rp_gather_kernel, dim3((unsigned)row_blocks(slots, lg)), dim3(256), 0, st,
                     reinterpret_cast<const float4 *>(table), n_rows, blocks, parts, cap, stride,
                     dim / 4, lg, reinterpret_cast<float4 *>(out));
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_frontier(const mirec_csr_t *c, const int32_t *keys, int64_t n_keys,
                              const int32_t *users, const int32_t *pos, const int32_t *neg,
                              int64_t batch, int64_t n_users, uint8_t *bm_self,
                              uint8_t *bm_hop, int32_t *self_list, int32_t *self_count,
                              int32_t *zero_counts, int32_t n_zero_counts,
                              mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(c && c->rowptr && c->col && bm_self && bm_hop);
  MIREC_CHECK_ARG(keys != nullptr || (users && pos && neg && batch >= 0 && n_users >= 0));
  MIREC_CHECK_ARG(self_list == nullptr || self_count != nullptr);
  MIREC_CHECK_ARG(n_zero_counts >= 0 && n_zero_counts <= 256 &&
                  (n_zero_counts == 0 || zero_counts != nullptr));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const size_t bytes = (size_t)((c->n_rows + 3) / 4) * 4;  // whole words (test_and_set)
  const size_t bytes16 = (bytes + 15) / 16 * 16;
  int32_t *sc = self_list != nullptr ? self_count : nullptr;
  if (bm_hop == bm_self + bytes16 && ((uintptr_t)bm_self & 15u) == 0) {
    // adjacent, 16-B aligned maps: everything cleared by one launch
    const int64_t n16 = (int64_t)(2 * bytes16 / 16);
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n16 + 255) / 256, 1024));
    hipLaunchKernelGGL(frontier_clear_kernel, dim3(blocks), dim3(256), 0, st,
                       reinterpret_cast<uint4 *>(bm_self), n16, sc, zero_counts, n_zero_counts);
    MIREC_LAUNCH_CHECK();
  } else {
    MIREC_HIP(hipMemsetAsync(bm_self, 0, bytes, st));
    MIREC_HIP(hipMemsetAsync(bm_hop, 0, bytes, st));
    if (sc != nullptr) MIREC_HIP(hipMemsetAsync(sc, 0, 4, st));
    if (n_zero_counts > 0) MIREC_HIP(hipMemsetAsync(zero_counts, 0, 4 * (size_t)n_zero_counts, st));
  }
  const int64_t n = keys != nullptr ? n_keys : 3 * batch;
  const int32_t split = c->n_seg > 0 ? c->split : 0;
  if (self_list != nullptr) {
    if (n > 0) {
      hipLaunchKernelGGL(frontier_self_kernel, dim3((n + 255) / 256), dim3(256), 0, st, c->n_rows,
                         keys, n_keys, users, pos, neg, batch, n_users, bm_self, bm_hop,
                         self_list, self_count);
      MIREC_LAUNCH_CHECK();
      hipLaunchKernelGGL(frontier_expand_kernel, dim3((n + kWaves - 1) / kWaves), dim3(256), 0,
                         st, c->rowptr, c->col, split, self_list, self_count, bm_hop);
      MIREC_LAUNCH_CHECK();
    }
  } else if (n > 0) {
    hipLaunchKernelGGL(frontier_keys_kernel, dim3((n + kWaves - 1) / kWaves), dim3(256), 0, st,
                       c->rowptr, c->col, c->n_rows, split, keys, n_keys, users, pos, neg, batch,
                       n_users, bm_self, bm_hop);
    MIREC_LAUNCH_CHECK();
  }
  if (c->n_seg > 0 && n > 0) {
    hipLaunchKernelGGL(frontier_segments_kernel, dim3((c->n_seg + kWaves - 1) / kWaves), dim3(256),
                       0, st, c->rowptr, c->col, c->seg_row, c->seg_beg, c->n_seg, c->split,
                       bm_self, bm_hop);
    MIREC_LAUNCH_CHECK();
  }
  return MIREC_OK;
}

extern "C" int mirec_mask_compact(const mirec_csr_t *c, const uint8_t *bm, int32_t narrow_max,
                                  int32_t *list, int32_t *count, int32_t *wide_list,
                                  int32_t *wide_count, int32_t counts_zeroed,
                                  mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(c && c->rowptr && bm && list && count && c->n_rows >= 0);
  MIREC_CHECK_ARG(wide_list == nullptr || wide_count != nullptr);
  MIREC_CHECK_ARG(((uintptr_t)bm & 15u) == 0);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (counts_zeroed) {
    // (cleared by the caller on this stream, e.g. mirec_frontier's zero_counts)
  } else if (wide_count == count + 1) {  // adjacent counters: one clear
    MIREC_HIP(hipMemsetAsync(count, 0, 8, st));
  } else {
    MIREC_HIP(hipMemsetAsync(count, 0, 4, st));
    if (wide_count != nullptr) MIREC_HIP(hipMemsetAsync(wide_count, 0, 4, st));
  }
  const int64_t threads = (c->n_rows + 15) / 16;
  if (threads > 0) {
    hipLaunchKernelGGL(mask_compact_kernel, dim3((threads + 255) / 256), dim3(256), 0, st, bm,
                       c->rowptr, c->n_rows, narrow_max, list, count, wide_list, wide_count);
    MIREC_LAUNCH_CHECK();
  }
  return MIREC_OK;
}

extern "C" int mirec_mask_compact_pair(const uint8_t *bm_a, const uint8_t *bm_b,
                                       const uint32_t *wide_bits, int64_t n_rows,
                                       int32_t *list_a, int32_t *wide_a, int32_t *list_b,
                                       int32_t *wide_b, int32_t *counts, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(bm_a && bm_b && wide_bits && list_a && wide_a && list_b && wide_b && counts &&
                  n_rows >= 0);
  MIREC_CHECK_ARG((((uintptr_t)bm_a | (uintptr_t)bm_b) & 15u) == 0);
  const int64_t threads = (n_rows + 31) / 32;
  if (threads == 0) return MIREC_OK;
  hipLaunchKernelGGL(mask_compact_pair_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256),
                     0, reinterpret_cast<hipStream_t>(stream), bm_a, bm_b, wide_bits, n_rows,
                     list_a, wide_a, list_b, wide_b, counts);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_scatter_rows(const float *src, const int32_t *ids, int64_t n, int32_t dim,
                                  float *dst, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(n >= 0 && dim > 0 && dim % 4 == 0);
  if (n == 0) return MIREC_OK;
  MIREC_CHECK_ARG(src && ids && dst);
  MIREC_CHECK_ARG(((uintptr_t)src & 15u) == 0 && ((uintptr_t)dst & 15u) == 0);
  const int lg = row_lg(dim / 4);
  MIREC_CHECK_ARG(lg <= 8);
  hipLaunchKernelGGL(scatter_rows_kernel, dim3((unsigned)row_blocks(n, lg)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float4 *>(src),
                     ids, n, dim / 4, lg, reinterpret_cast<float4 *>(dst));
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

