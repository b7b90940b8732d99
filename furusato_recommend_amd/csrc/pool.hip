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
// One wave per sequence: lanes 0-31 sum the even rows and lanes 32-63 the
// odd rows of a 128-column slice (4 rows of each in flight per lane), then
// the two partials are added — a fixed order, so reruns are bitwise equal.
__global__ __launch_bounds__(256) void segment_mean_kernel(const float *__restrict__ x,
                                                           const int32_t *__restrict__ offsets,
                                                           const int64_t *__restrict__ length,
                                                           int64_t B, int32_t d,
                                                           float *__restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63, half = lane >> 5;
  const int r0 = offsets[b], r1 = offsets[b + 1];
  const float inv = 1.f / (float)length[b];
  for (int c0 = 0; c0 < d; c0 += 128) {
    const int c = c0 + 4 * (lane & 31);
    const bool on = c < d;
    float4 a = f4_zero();
    for (int r = r0 + half; r < r1; r += 8) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = (on && r + 2 * u < r1) ? ld4(x + (int64_t)(r + 2 * u) * d + c) : f4_zero();
#pragma unroll
      for (int u = 0; u < 4; ++u) a = f4_add(a, v[u]);
    }
    a.x += __shfl_xor(a.x, 32);
    a.y += __shfl_xor(a.y, 32);
    a.z += __shfl_xor(a.z, 32);
    a.w += __shfl_xor(a.w, 32);
    if (on && half == 0) st4(out + b * d + c, make_float4(a.x * inv, a.y * inv, a.z * inv, a.w * inv));
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

// BPR loss on embedding rows (model/sasrec.py:423-435): x_r = <u_r, n_r> -
// <u_r, p_r>, loss = mean_r softplus(x_r) + coef * extra[0] (extra: the
// embedding-norm term, or NULL).  Pass 1: one wave per row writes x_r and
// softplus(x_r) (torch's: beta 1, threshold 20); pass 2: one workgroup adds
// the B terms in a fixed order (deterministic).
__device__ __forceinline__ float softplus20(float x) { return x > 20.f ? x : log1pf(expf(x)); }

__global__ __launch_bounds__(256) MIREC_NO_PK_F32 void bpr_rows_kernel(const float *__restrict__ u,
                                                       const float *__restrict__ p,
                                                       const float *__restrict__ n, int64_t B,
                                                       int32_t d, float *__restrict__ x_out,
                                                       float *__restrict__ sp_out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  float sp = 0.f, sn = 0.f;
  for (int c = lane; c < d; c += 64) {
    const float uv = u[r * d + c];
    sp += uv * p[r * d + c];
    sn += uv * n[r * d + c];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sp += __shfl_xor(sp, o);
    sn += __shfl_xor(sn, o);
  }
  if (lane == 0) {
    const float x = sn - sp;
    x_out[r] = x;
    sp_out[r] = softplus20(x);
  }
}

__global__ __launch_bounds__(1024) void bpr_rows_sum_kernel(const float *__restrict__ sp,
                                                            int64_t B,
                                                            const float *__restrict__ extra,
                                                            float coef, float *__restrict__ loss) {
  __shared__ float part[1024];
  float a = 0.f;
  for (int64_t r = threadIdx.x; r < B; r += 1024) a += sp[r];
  part[threadIdx.x] = a;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = part[0] / (float)B + (extra ? coef * extra[0] : 0.f);
}

// s_r = g * sigmoid(x_r) / B;  du = s (n - p), dp = -s u, dn = s u;
// g_extra = g * coef.
__global__ __launch_bounds__(256) void bpr_rows_loss_bwd_kernel(
    const float *__restrict__ u, const float *__restrict__ p, const float *__restrict__ n,
    const float *__restrict__ x, int64_t B, int32_t d, const float *__restrict__ g_loss,
    float coef, float *__restrict__ du, float *__restrict__ dp, float *__restrict__ dn,
    float *__restrict__ g_extra) {
  const float g = g_loss[0];
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e == 0 && g_extra) g_extra[0] = g * coef;
  if (e >= B * d) return;
  const int64_t r = e / d;
  const float s = g / (1.f + expf(-x[r])) / (float)B;
  const float uv = u[e], pv = p[e], nv = n[e];
  du[e] = s * (nv - pv);
  dp[e] = -s * uv;
  dn[e] = s * uv;
}

// Packing of a SASRec batch into a token capacity (graph-captured step):
// pass 1 (one workgroup) gathers the users' lengths and scans them into
// offsets (clamped to the capacity) and converts the positive / negative
// ids; pass 2 (one lane per token row) finds the row's sequence by binary
// search over the offsets and writes its item id (-1 and seg = B for rows
// past the last sequence).
__global__ __launch_bounds__(1024) void seq_pack_scan_kernel(
    const int64_t *__restrict__ users, int64_t B, const int64_t *__restrict__ length_tab,
    const int64_t *__restrict__ pos, const int64_t *__restrict__ neg, int64_t capacity,
    int32_t *__restrict__ offsets, int64_t *__restrict__ length, int32_t *__restrict__ ids_all) {
  __shared__ int64_t part[1024];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) {
    carry = 0;
    offsets[0] = 0;
  }
  __syncthreads();
  for (int64_t base = 0; base < B; base += 1024) {
    const int64_t b = base + threadIdx.x;
    int64_t len = 0;
    if (b < B) {
      len = length_tab[users[b]];
      length[b] = len;
      ids_all[capacity + b] = (int32_t)pos[b];
      ids_all[capacity + B + b] = (int32_t)neg[b];
    }
    part[threadIdx.x] = len;
    __syncthreads();
    for (int s = 1; s < 1024; s <<= 1) {  // inclusive Hillis-Steele scan
      const int64_t v = (int)threadIdx.x >= s ? part[threadIdx.x - s] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
    }
    if (b < B) offsets[b + 1] = (int32_t)min(carry + part[threadIdx.x], capacity);
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void seq_pack_rows_kernel(
    const int64_t *__restrict__ users, int64_t B, const int32_t *__restrict__ items,
    int32_t max_len, int64_t capacity, const int32_t *__restrict__ offsets,
    int32_t *__restrict__ ids_all, int64_t *__restrict__ seg) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= capacity) return;
  int64_t lo = 0, hi = B;  // first b with offsets[b + 1] > t, or B
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (offsets[mid + 1] > t) hi = mid;
    else lo = mid + 1;
  }
  if (lo < B) {
    const int64_t k = t - offsets[lo];
    ids_all[t] = items[users[lo] * max_len + k];
    seg[t] = lo;
  } else {
    ids_all[t] = -1;
    seg[t] = B;
  }
}

// L2 norms of x[0, split) and x[split, n) (the user / item slices of an id
// table: the parameter-norm term of model/graphsage.py:326-337 and
// model/sasrec.py:423-435).  Pass 1: each workgroup sums the squares of a
// fixed stride of float4 per slice into its partial pair; pass 2: one
// workgroup adds the partials in block order and takes the roots
// (deterministic).  split % 4 == 0, n % 4 == 0.
constexpr int kNormBlocks = 1024;
__global__ __launch_bounds__(256) void slice_sumsq_kernel(const float *__restrict__ x, int64_t n4,
                                                          int64_t split4,
                                                          float *__restrict__ partial) {
  __shared__ float red[2][256];
  float a = 0.f, b = 0.f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n4; e += (int64_t)kNormBlocks * 256) {
    const float4 v = ld4(x + 4 * e);
    const float s = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    if (e < split4) a += s;
    else b += s;
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = red[0][0];
    partial[2 * blockIdx.x + 1] = red[1][0];
  }
}

__global__ __launch_bounds__(256) void slice_norm_final_kernel(const float *__restrict__ partial,
                                                               float *__restrict__ norms) {
  __shared__ float red[2][256];
  float a = 0.f, b = 0.f;
  for (int k = threadIdx.x; k < kNormBlocks; k += 256) {
    a += partial[2 * k];
    b += partial[2 * k + 1];
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    norms[0] = sqrtf(red[0][0]);
    norms[1] = sqrtf(red[1][0]);
  }
}

// Parameter-norm term of the GraphSAGE loss (model/graphsage.py:326-337:
// all_param = 2 all_param + |p| over the parameters, i.e. the weighted sum
// Σ 2^(K-1-k) |p_k|) over a few small tensors plus norms already on the
// device (the id table's slices).  One 1024-thread workgroup: each tensor's
// sum of squares in a fixed order (strided partials, then a tree), total
// accumulated in term order after the extra terms (deterministic).
constexpr int kMaxNormTerms = MIREC_NORM_TERMS_MAX;
struct NormTermArgs {
  const float *x[kMaxNormTerms];
  float *g[kMaxNormTerms];
  int64_t off[kMaxNormTerms + 1];
  float w[kMaxNormTerms];
  float ew[kMaxNormTerms];
  int32_t count, n_extra;
};

__global__ __launch_bounds__(1024) void norm_terms_kernel(NormTermArgs a,
                                                          const float *__restrict__ extra,
                                                          float *__restrict__ norms,
                                                          float *__restrict__ total) {
  __shared__ float red[1024];
  float tot = 0.f;
  for (int j = 0; j < a.n_extra; ++j) tot += a.ew[j] * extra[j];
  for (int k = 0; k < a.count; ++k) {
    const int64_t n = a.off[k + 1] - a.off[k];
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < n; i += 1024) {
      const float v = a.x[k][i];
      s += v * v;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int h = 512; h > 0; h >>= 1) {
      if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
      __syncthreads();
    }
    const float nk = sqrtf(red[0]);
    tot += a.w[k] * nk;
    if (threadIdx.x == 0) norms[k] = nk;
    __syncthreads();
  }
  if (threadIdx.x == 0) total[0] = tot;
}

// g_k[i] = g * w_k * x_k[i] / |x_k| (0 where |x_k| = 0, as torch's norm
// backward); extra_grad[j] = g * ew_j.  One thread per element of the
// concatenation (+ n_extra).
__global__ __launch_bounds__(256) void norm_terms_bwd_kernel(NormTermArgs a,
                                                             const float *__restrict__ norms,
                                                             const float *__restrict__ g_total,
                                                             float *__restrict__ extra_grad,
                                                             int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const float g = g_total[0];
  const int64_t tot = a.off[a.count];
  if (i < tot) {
    int k = 0;
    while (a.off[k + 1] <= i) ++k;
    const int64_t j = i - a.off[k];
    const float nk = norms[k];
    const float v = nk > 0.f ? g * a.w[k] * (a.x[k][j] / nk) : 0.f;
    if (accumulate) a.g[k][j] += v;
    else a.g[k][j] = v;
  } else if (i < tot + a.n_extra) {
    extra_grad[i - tot] = g * a.ew[i - tot];
  }
}

}  // namespace mirec

using namespace mirec;

extern "C" int64_t mirec_slice_norms_work_floats(void) { return 2 * kNormBlocks; }

extern "C" int mirec_slice_norms(const float *x, int64_t n, int64_t split, float *work,
                                 float *norms, mirec_stream_t stream) {
  MIREC_CHECK_ARG(x && work && norms && n >= 0 && split >= 0 && split <= n);
  MIREC_CHECK_ARG(n % 4 == 0 && split % 4 == 0 && (uintptr_t)x % 16 == 0);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(slice_sumsq_kernel, dim3(kNormBlocks), dim3(256), 0, st, x, n / 4, split / 4,
                     work);
  MIREC_LAUNCH_CHECK();
  hipLaunchKernelGGL(slice_norm_final_kernel, dim3(1), dim3(256), 0, st, work, norms);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_seq_pack(const int64_t *users, int64_t B, const int32_t *items,
                              int32_t max_len, const int64_t *length_tab, const int64_t *pos,
                              const int64_t *neg, int64_t capacity, int32_t *offsets,
                              int64_t *length, int32_t *ids_all, int64_t *seg,
                              mirec_stream_t stream) {
  MIREC_CHECK_ARG(B > 0 && max_len > 0 && capacity >= 0 && capacity < (int64_t)1 << 31);
  MIREC_CHECK_ARG(users && items && length_tab && pos && neg && offsets && length && ids_all &&
                  (capacity == 0 || seg));
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(seq_pack_scan_kernel, dim3(1), dim3(1024), 0, st, users, B, length_tab, pos,
                     neg, capacity, offsets, length, ids_all);
  MIREC_LAUNCH_CHECK();
  if (capacity > 0) {
    hipLaunchKernelGGL(seq_pack_rows_kernel, dim3((unsigned)((capacity + 255) / 256)), dim3(256),
                       0, st, users, B, items, max_len, capacity, offsets, ids_all, seg);
    MIREC_LAUNCH_CHECK();
  }
  return MIREC_OK;
}

extern "C" int mirec_bpr_rows_loss(const float *u, const float *p, const float *n, int64_t B,
                                   int32_t d, const float *extra, float coef, float *x_out,
                                   float *loss, mirec_stream_t stream) {
  MIREC_CHECK_ARG(B > 0 && d > 0 && u && p && n && x_out && loss);
  hipStream_t st = (hipStream_t)stream;
  // x_out holds 2B floats: x, then the per-row softplus terms
  hipLaunchKernelGGL(bpr_rows_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, u, p, n, B,
                     d, x_out, x_out + B);
  MIREC_LAUNCH_CHECK();
  hipLaunchKernelGGL(bpr_rows_sum_kernel, dim3(1), dim3(1024), 0, st, x_out + B, B, extra, coef,
                     loss);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_bpr_rows_loss_bwd(const float *u, const float *p, const float *n,
                                       const float *x, int64_t B, int32_t d, const float *g_loss,
                                       float coef, float *du, float *dp, float *dn,
                                       float *g_extra, mirec_stream_t stream) {
  MIREC_CHECK_ARG(B > 0 && d > 0 && u && p && n && x && g_loss && du && dp && dn);
  const int64_t total = B * d;
  hipLaunchKernelGGL(bpr_rows_loss_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256),
                     0, (hipStream_t)stream, u, p, n, x, B, d, g_loss, coef, du, dp, dn, g_extra);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

static int norm_args(const float *const *xs, float *const *grads, const int64_t *numel,
                     const float *weights, int32_t count, const float *extra_w, int32_t n_extra,
                     NormTermArgs *a) {
  MIREC_CHECK_ARG(count >= 0 && count <= kMaxNormTerms && n_extra >= 0 &&
                  n_extra <= kMaxNormTerms && (count == 0 || (xs && numel && weights)) &&
                  (n_extra == 0 || extra_w));
  *a = NormTermArgs{};
  a->count = count;
  a->n_extra = n_extra;
  for (int k = 0; k < count; ++k) {
    MIREC_CHECK_ARG(xs[k] && numel[k] >= 0);
    a->x[k] = xs[k];
    a->g[k] = grads ? grads[k] : nullptr;
    a->w[k] = weights[k];
    a->off[k + 1] = a->off[k] + numel[k];
  }
  for (int j = 0; j < n_extra; ++j) a->ew[j] = extra_w[j];
  return MIREC_OK;
}

extern "C" int mirec_norm_terms(const float *const *xs, const int64_t *numel, const float *weights,
                                int32_t count, const float *extra, const float *extra_w,
                                int32_t n_extra, float *norms, float *total,
                                mirec_stream_t stream) {
  NormTermArgs a;
  const int rc = norm_args(xs, nullptr, numel, weights, count, extra_w, n_extra, &a);
  if (rc != MIREC_OK) return rc;
  MIREC_CHECK_ARG(total && (count == 0 || norms) && (n_extra == 0 || extra));
  hipLaunchKernelGGL(norm_terms_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, a, extra,
                     norms, total);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

static int norm_terms_bwd(const float *const *xs, float *const *grads, const int64_t *numel,
                          const float *weights, int32_t count, const float *norms,
                          const float *g_total, const float *extra_w, int32_t n_extra,
                          float *extra_grad, int accumulate, mirec_stream_t stream) {
  NormTermArgs a;
  const int rc = norm_args(xs, grads, numel, weights, count, extra_w, n_extra, &a);
  if (rc != MIREC_OK) return rc;
  MIREC_CHECK_ARG(g_total && (count == 0 || (grads && norms)) && (n_extra == 0 || extra_grad));
  for (int k = 0; k < count; ++k) MIREC_CHECK_ARG(grads[k]);
  const int64_t tot = a.off[count] + n_extra;
  if (tot == 0) return MIREC_OK;
  hipLaunchKernelGGL(norm_terms_bwd_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, a, norms, g_total, extra_grad, accumulate);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_norm_terms_bwd(const float *const *xs, float *const *grads,
                                    const int64_t *numel, const float *weights, int32_t count,
                                    const float *norms, const float *g_total,
                                    const float *extra_w, int32_t n_extra, float *extra_grad,
                                    mirec_stream_t stream) {
  return norm_terms_bwd(xs, grads, numel, weights, count, norms, g_total, extra_w, n_extra,
                        extra_grad, 0, stream);
}

extern "C" int mirec_norm_terms_bwd_acc(const float *const *xs, float *const *grads,
                                        const int64_t *numel, const float *weights,
                                        int32_t count, const float *norms, const float *g_total,
                                        mirec_stream_t stream) {
  return norm_terms_bwd(xs, grads, numel, weights, count, norms, g_total, nullptr, 0, nullptr, 1,
                        stream);
}

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
  hipLaunchKernelGGL(segment_mean_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, x, offsets, length, B, d, out);
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

// BPR pairs of a sequence batch on the device: out[j] = a uniformly drawn
// item of user users[j]'s sequence (items[u][0, length[u])), out[B + j] = a
// uniform item in [0, m_items) — the (positive, negative) of UniformSample
// over the users' interactions (the SASRec benchmark's per-step pairs).
// Counter-based: element j's draws are mix64(key + 2 (offset + j) + {0, 1}).
__global__ __launch_bounds__(256) void seq_sample_kernel(const int64_t *__restrict__ users,
                                                         int64_t B,
                                                         const int32_t *__restrict__ items,
                                                         int32_t max_len,
                                                         const int64_t *__restrict__ length,
                                                         int64_t m_items, uint64_t key,
                                                         uint64_t offset,
                                                         int64_t *__restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= B) return;
  const uint64_t c = key + 2 * (offset + (uint64_t)j);
  const int64_t u = users[j];
  const int64_t len = length[u];
  const int64_t k = len > 0 ? (int64_t)__umul64hi(mix64(c), (uint64_t)len) : 0;
  out[j] = len > 0 ? (int64_t)items[u * max_len + k] : 0;
  out[B + j] = (int64_t)__umul64hi(mix64(c + 1), (uint64_t)m_items);
}

extern "C" int mirec_seq_sample(const int64_t *users, int64_t B, const int32_t *items,
                                int32_t max_len, const int64_t *length, int64_t m_items,
                                uint64_t seed, uint64_t offset, int64_t *out,
                                mirec_stream_t stream) {
  MIREC_CHECK_ARG(B >= 0 && max_len > 0 && m_items > 0);
  if (B == 0) return MIREC_OK;
  MIREC_CHECK_ARG(users && items && length && out);
  hipLaunchKernelGGL(seq_sample_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, users, B, items, max_len, length, m_items,
                     mix64(seed ^ 0x5EC5A3B1E0D7F00Dull), offset, out);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}
