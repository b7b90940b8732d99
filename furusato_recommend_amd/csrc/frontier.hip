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
// One wave per key expands its CSR row with plain byte stores (idempotent:
// no atomics); S membership is set with one 32-bit atomicOr per key so the
// first setter can append the node to the deduplicated S list.  Rows longer
// than the CSR split are expanded by one wave per segment (second kernel),
// so a hot item does not serialise the launch.
#include "common.h"

namespace mirec {

constexpr int kWaves = 4;

// Sets byte i of a byte map with a word atomicOr; true if this call set it.
__device__ __forceinline__ bool test_and_set(uint8_t *bm, int64_t i) {
  const uint32_t b = 1u << (8 * (i & 3));
  return (atomicOr(reinterpret_cast<uint32_t *>(bm) + (i >> 2), b) & b) == 0u;
}

__global__ __launch_bounds__(256) void frontier_keys_kernel(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col, int64_t n_rows,
    int32_t split, const int32_t *__restrict__ keys, int64_t n_keys,
    const int32_t *__restrict__ users, const int32_t *__restrict__ pos,
    const int32_t *__restrict__ neg, int64_t batch, int64_t n_users, uint8_t *bm_self,
    uint8_t *bm_hop, int32_t *self_list, int32_t *self_count) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  int64_t node;
  if (keys != nullptr) {
    if (i >= n_keys) return;
    node = keys[i];
  } else {
    if (i >= 3 * batch) return;
    node = i < batch ? (int64_t)users[i]
                     : (i < 2 * batch ? n_users + pos[i - batch] : n_users + neg[i - 2 * batch]);
  }
  if (node < 0 || node >= n_rows) return;  // empty / sentinel entries
  if (lane == 0) {
    if (test_and_set(bm_self, node) && self_list != nullptr)
      self_list[atomicAdd(self_count, 1)] = (int32_t)node;
    bm_hop[node] = 1;
  }
  const int64_t beg = rowptr[node], end = rowptr[node + 1];
  if (split > 0 && end - beg > split) return;  // expanded per segment
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

}  // namespace mirec

extern "C" int mirec_frontier(const mirec_csr_t *c, const int32_t *keys, int64_t n_keys,
                              const int32_t *users, const int32_t *pos, const int32_t *neg,
                              int64_t batch, int64_t n_users, uint8_t *bm_self,
                              uint8_t *bm_hop, int32_t *self_list, int32_t *self_count,
                              mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(c && c->rowptr && c->col && bm_self && bm_hop);
  MIREC_CHECK_ARG(keys != nullptr || (users && pos && neg && batch >= 0 && n_users >= 0));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const size_t bytes = (size_t)((c->n_rows + 3) / 4) * 4;  // whole words (test_and_set)
  MIREC_HIP(hipMemsetAsync(bm_self, 0, bytes, st));
  MIREC_HIP(hipMemsetAsync(bm_hop, 0, bytes, st));
  MIREC_CHECK_ARG(self_list == nullptr || self_count != nullptr);
  if (self_count != nullptr) MIREC_HIP(hipMemsetAsync(self_count, 0, 4, st));
  const int64_t n = keys != nullptr ? n_keys : 3 * batch;
  if (n > 0) {
    hipLaunchKernelGGL(frontier_keys_kernel, dim3((n + kWaves - 1) / kWaves), dim3(256), 0, st,
                       c->rowptr, c->col, c->n_rows, c->n_seg > 0 ? c->split : 0, keys, n_keys,
                       users, pos, neg, batch, n_users, bm_self, bm_hop, self_list, self_count);
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
