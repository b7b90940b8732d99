// Stable sort of up to 8 192 (int32 key, int32 value) pairs in two
// launches: the BPR seed grouping of every LightGCN step (3B = 6 144 node
// keys, bpr.hip; reference: the per-node gradient rows of the BPR batch,
// model/lgcn.py:96-123).  The device library's radix sort spends six
// launches of ~5 us on it (32 us of the C2 step).
//
// Each pair becomes one unique 64-bit composite (key << 32 | input index),
// so ascending composites ARE the stable order and ties never arise, and a
// composite's final position is its rank: the number of composites below
// it.  Launch 1 counts them over a grid of (256 entries) x (256-entry
// chunks): a workgroup stages one chunk in LDS and each thread compares its
// composite with all of it (broadcast reads), writing one partial count —
// n^2 / 2^16 workgroups, the whole chip busy; launch 2 adds each entry's
// partial counts and writes it at its rank.  (A one-workgroup bitonic
// network in LDS, and the same with the elements in registers and the
// short stages on lane shuffles, both measured ~78 us at 6 144 keys: one CU,
// latency-bound; a tile + rank-merge form for 64 K entries was no faster
// than the library's merge sort either.)
#include "common.h"
#include "smallsort.h"

namespace mirec {
namespace {

constexpr int kB = 256;

__device__ __forceinline__ uint64_t composite(const int32_t *__restrict__ keys, int64_t i) {
  return ((uint64_t)(uint32_t)keys[i] << 32) | (uint64_t)(uint32_t)i;
}

// part[c * n + i] = #{composites of chunk c below entry i's}
__global__ __launch_bounds__(kB) void ss_count_kernel(const int32_t *__restrict__ keys, int64_t n,
                                                      int32_t *__restrict__ part) {
  __shared__ uint64_t s[kB];
  const int64_t c0 = (int64_t)blockIdx.y * kB;
  const int len = (int)(n - c0 < kB ? n - c0 : kB);
  if ((int)threadIdx.x < len) s[threadIdx.x] = composite(keys, c0 + threadIdx.x);
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  const uint64_t x = composite(keys, i);
  int cnt = 0;
#pragma unroll 8
  for (int j = 0; j < len; ++j) cnt += s[j] < x ? 1 : 0;
  part[(int64_t)blockIdx.y * n + i] = cnt;
}

__global__ __launch_bounds__(kB) void ss_place_kernel(const int32_t *__restrict__ keys,
                                                      const int32_t *__restrict__ vals, int64_t n,
                                                      int n_chunks,
                                                      const int32_t *__restrict__ part,
                                                      int32_t *__restrict__ keys_out,
                                                      int32_t *__restrict__ vals_out) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  int r = 0;
#pragma unroll 8
  for (int c = 0; c < n_chunks; ++c) r += part[(int64_t)c * n + i];  // (loads in flight together)
  keys_out[r] = keys[i];
  vals_out[r] = vals ? vals[i] : (int32_t)i;
}

}  // namespace

size_t small_sort_workspace(int64_t n) {
  const int64_t chunks = (n + kB - 1) / kB;
  return (size_t)(chunks * n) * sizeof(int32_t);
}

hipError_t small_sort_pairs(void *ws, size_t ws_bytes, const int32_t *keys_in, int32_t *keys_out,
                            const int32_t *vals_in, int32_t *vals_out, int64_t n,
                            hipStream_t st) {
  if (n < 0 || n > kSmallSortMax) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  if (keys_in == nullptr || keys_out == nullptr || vals_out == nullptr || ws == nullptr ||
      ws_bytes < small_sort_workspace(n))
    return hipErrorInvalidValue;
  int32_t *part = static_cast<int32_t *>(ws);
  const int chunks = (int)((n + kB - 1) / kB);
  hipLaunchKernelGGL(ss_count_kernel, dim3((unsigned)chunks, (unsigned)chunks), dim3(kB), 0, st,
                     keys_in, n, part);
  hipLaunchKernelGGL(ss_place_kernel, dim3((unsigned)chunks), dim3(kB), 0, st, keys_in, vals_in, n,
                     chunks, part, keys_out, vals_out);
  return hipGetLastError();
}

}  // namespace mirec

extern "C" int mirec_small_sort_workspace(int64_t n, size_t *bytes) {
  using namespace mirec;
  MIREC_CHECK_ARG(bytes && n >= 0 && n <= kSmallSortMax);
  *bytes = small_sort_workspace(n);
  return MIREC_OK;
}

extern "C" int mirec_small_sort_pairs(const int32_t *keys_in, const int32_t *vals_in,
                                      int32_t *keys_out, int32_t *vals_out, int64_t n,
                                      void *workspace, size_t workspace_bytes,
                                      mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(n >= 0 && n <= kSmallSortMax);
  if (n == 0) return MIREC_OK;
  MIREC_CHECK_ARG(keys_in && keys_out && vals_out);
  if (workspace_bytes < small_sort_workspace(n)) return MIREC_ERR_WORKSPACE;
  MIREC_HIP(small_sort_pairs(workspace, workspace_bytes, keys_in, keys_out, vals_in, vals_out, n,
                             reinterpret_cast<hipStream_t>(stream)));
  return MIREC_OK;
}
