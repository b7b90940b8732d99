// Row shards of the data-parallel `sharded` exchange (dist.DataParallel):
// rank r owns the rows i ≡ r (mod W) — slot s of rank r is row r + s·W — and
// a block of slots [s0, s0 + ns) covers the rows [s0·W, (s0 + ns)·W).  The
// block's all-gather output is a [W][ns][D] staging buffer.
//
//   mirec_shard_pack    stage_r[s][:] = table[r + (s0 + s)·W][:]  (this
//                       rank's finished rows into its slot of the buffer)
//   mirec_shard_unpack  table[w + (s0 + s)·W][:] = stage[w][s][:] for every
//                       other rank w, and with x0s also x0s[row] = dinv[row] ·
//                       that row: the next forward's pre-scaled layer-0
//                       input for the rows another rank updated (this rank's
//                       own rows got theirs from the fused Adam), so no
//                       prescale pass over the whole table follows.
// float4 per thread, grid-stride; rows past n_rows (the ragged last block)
// are zero in the buffer and skipped on the way back.
#include "common.h"

namespace mirec {

__global__ __launch_bounds__(256) void shard_pack_kernel(const float *__restrict__ table,
                                                         int64_t n_rows, int32_t d4, int32_t W,
                                                         int32_t r, int64_t s0, int64_t ns,
                                                         float *__restrict__ stage_r) {
  const int64_t n4 = ns * d4, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const int64_t s = i / d4, c = i - s * d4, row = r + (s0 + s) * W;
    st4(stage_r + 4 * i, row < n_rows ? ld4(table + row * 4 * d4 + 4 * c) : f4_zero());
  }
}

__global__ __launch_bounds__(256) void shard_unpack_kernel(
    const float *__restrict__ stage, int64_t n_rows, int32_t d4, int32_t W, int32_t r, int64_t s0,
    int64_t ns, const float *__restrict__ dinv, float *__restrict__ table,
    float *__restrict__ x0s) {
  const int64_t per = ns * d4, n4 = (int64_t)W * per, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const int64_t w = i / per, k = i - w * per, s = k / d4, c = k - s * d4;
    const int64_t row = w + (s0 + s) * W;
    if (w == r || row >= n_rows) continue;
    const float4 v = ld4(stage + 4 * i);
    st4(table + row * 4 * d4 + 4 * c, v);
    if (x0s != nullptr) st4(x0s + row * 4 * d4 + 4 * c, f4_scale(dinv[row], v));
  }
}

static unsigned grid_of(int64_t n4) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n4 + 255) / 256, 256 * 16));
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_shard_pack(const float *table, int64_t n_rows, int32_t dim, int32_t world,
                                int32_t rank, int64_t slot0, int64_t n_slots, float *stage_rank,
                                mirec_stream_t stream) {
  MIREC_CHECK_ARG(table && stage_rank && n_rows >= 0 && dim > 0 && dim % 4 == 0 && world >= 1 &&
                  rank >= 0 && rank < world && slot0 >= 0 && n_slots >= 0);
  MIREC_CHECK_ARG(((uintptr_t)table | (uintptr_t)stage_rank) % 16 == 0);
  const int64_t n4 = n_slots * (dim / 4);
  if (n4 == 0) return MIREC_OK;
  hipLaunchKernelGGL(shard_pack_kernel, dim3(grid_of(n4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), table, n_rows, dim / 4, world, rank,
                     slot0, n_slots, stage_rank);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_shard_unpack(const float *stage, int64_t n_rows, int32_t dim, int32_t world,
                                  int32_t rank, int64_t slot0, int64_t n_slots, const float *dinv,
                                  float *table, float *x0s, mirec_stream_t stream) {
  MIREC_CHECK_ARG(stage && table && n_rows >= 0 && dim > 0 && dim % 4 == 0 && world >= 1 &&
                  rank >= 0 && rank < world && slot0 >= 0 && n_slots >= 0);
  MIREC_CHECK_ARG(x0s == nullptr || dinv != nullptr);
  MIREC_CHECK_ARG(((uintptr_t)stage | (uintptr_t)table | (uintptr_t)x0s) % 16 == 0);
  const int64_t n4 = (int64_t)world * n_slots * (dim / 4);
  if (n4 == 0) return MIREC_OK;
  hipLaunchKernelGGL(shard_unpack_kernel, dim3(grid_of(n4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), stage, n_rows, dim / 4, world, rank,
                     slot0, n_slots, dinv, table, x0s);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}
