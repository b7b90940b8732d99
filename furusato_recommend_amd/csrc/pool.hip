// Masked mean pool of the SASRec user tower (model/sasrec.py:399-413: the
// mean of the block output over the first `length` positions of each
// sequence) on packed sequences, where the positions of sequence b are the
// contiguous rows offsets[b] .. offsets[b+1]-1: a segment mean, one wave per
// sequence, rows summed in order (deterministic; no atomics).  The backward
// spreads grad_out[b] / length[b] over the sequence's rows; rows of no
// sequence (seg == B: capacity padding) get zero.
#include "common.h"

namespace mirec {

// 64 lanes x float4 = 256 columns per pass; d <= 1024.
__global__ __launch_bounds__(64) void segment_mean_kernel(const float *__restrict__ x,
                                                          const int32_t *__restrict__ offsets,
                                                          const int64_t *__restrict__ length,
                                                          int32_t d, float *__restrict__ out) {
  const int64_t b = blockIdx.x;
  const int r0 = offsets[b], r1 = offsets[b + 1];
  const float inv = 1.f / (float)length[b];
  for (int c = 4 * threadIdx.x; c < d; c += 256) {
    float4 a = f4_zero();
    for (int r = r0; r < r1; ++r) a = f4_add(a, ld4(x + (int64_t)r * d + c));
    st4(out + b * d + c, make_float4(a.x * inv, a.y * inv, a.z * inv, a.w * inv));
  }
}

// Row t of grad_x = grad_out[seg[t]] / length[seg[t]] (0 when seg[t] == B).
__global__ __launch_bounds__(256) void segment_mean_bwd_kernel(const float *__restrict__ g,
                                                               const int64_t *__restrict__ seg,
                                                               const int64_t *__restrict__ length,
                                                               int64_t n_rows, int64_t B,
                                                               int32_t d, float *__restrict__ gx) {
  const int d4 = d / 4;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_rows * d4) return;
  const int64_t t = e / d4;
  const int c = 4 * (int)(e - t * d4);
  const int64_t b = seg[t];
  float4 v = f4_zero();
  if (b >= 0 && b < B) {
    const float inv = 1.f / (float)length[b];
    v = ld4(g + b * d + c);
    v = make_float4(v.x * inv, v.y * inv, v.z * inv, v.w * inv);
  }
  st4(gx + t * d + c, v);
}

// Zero rows [offsets[B], n_rows) of a [n_rows, row_floats] buffer: the
// capacity-padding rows the packed kernels leave unwritten.
__global__ __launch_bounds__(256) void zero_tail_rows_kernel(float *__restrict__ buf,
                                                             const int32_t *__restrict__ offsets,
                                                             int64_t B, int64_t n_rows,
                                                             int32_t row_floats) {
  const int64_t r0 = offsets[B];
  const int64_t total = (n_rows - r0) * row_floats;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x)
    buf[r0 * row_floats + e] = 0.f;
}

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_zero_tail_rows(float *buf, const int32_t *offsets, int64_t B, int64_t n_rows,
                                    int32_t row_floats, mirec_stream_t stream) {
  MIREC_CHECK_ARG(B >= 0 && n_rows >= 0 && row_floats > 0);
  if (n_rows == 0) return MIREC_OK;
  MIREC_CHECK_ARG(buf && offsets);
  hipLaunchKernelGGL(zero_tail_rows_kernel, dim3(256), dim3(256), 0, (hipStream_t)stream, buf,
                     offsets, B, n_rows, row_floats);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_segment_mean(const float *x, const int32_t *offsets, const int64_t *length,
                                  int64_t B, int32_t d, float *out, mirec_stream_t stream) {
  MIREC_CHECK_ARG(B >= 0 && d > 0 && d % 4 == 0 && d <= 1024);
  if (B == 0) return MIREC_OK;
  MIREC_CHECK_ARG(x && offsets && length && out);
  hipLaunchKernelGGL(segment_mean_kernel, dim3((unsigned)B), dim3(64), 0, (hipStream_t)stream,
                     x, offsets, length, d, out);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_segment_mean_bwd(const float *grad_out, const int64_t *seg,
                                      const int64_t *length, int64_t n_rows, int64_t B,
                                      int32_t d, float *grad_x, mirec_stream_t stream) {
  MIREC_CHECK_ARG(n_rows >= 0 && B >= 0 && d > 0 && d % 4 == 0);
  if (n_rows == 0) return MIREC_OK;
  MIREC_CHECK_ARG(seg && grad_x && (B == 0 || (grad_out && length)));
  const int64_t total = n_rows * (d / 4);
  hipLaunchKernelGGL(segment_mean_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, grad_out, seg, length, n_rows, B, d, grad_x);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}
