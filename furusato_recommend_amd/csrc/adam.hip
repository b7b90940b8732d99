// Dense single-pass Adam (torch.optim.Adam, amsgrad=False, weight_decay=0),
// the optimizer of model/lgcn.py:63 stepped at model/lgcn.py:132.  One pass
// reads param/grad/m/v and writes param/m/v as float4 (7 x 4 B per element:
// HBM-bound).  Used by the data-parallel path after the gradient all-reduce;
// the single-GPU path fuses the same update into the last backward
// propagation epilogue (prop.hip) and never materialises the gradient.
#include "common.h"

namespace mirec {

// Hyper-parameters by value, or read from device memory when hp != NULL
// (the *_dev entry points: a captured HIP graph replays with the step's
// scalars written there by the host before each replay).
__device__ __forceinline__ mirec_adam_hparams_t hparams(mirec_adam_hparams_t h,
                                                        const mirec_adam_hparams_t *hp) {
  return hp ? *hp : h;
}

__global__ __launch_bounds__(256) void adam_dense_kernel(float *__restrict__ param,
                                                         const float *__restrict__ grad,
                                                         float *__restrict__ m,
                                                         float *__restrict__ v, int64_t n4,
                                                         mirec_adam_hparams_t hv,
                                                         const mirec_adam_hparams_t *hp) {
  const mirec_adam_hparams_t h = hparams(hv, hp);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 p = ld4(param + 4 * i), g = ld4(grad + 4 * i), a = ld4(m + 4 * i),
           b = ld4(v + 4 * i);
    adam1(p.x, a.x, b.x, g.x, h);
    adam1(p.y, a.y, b.y, g.y, h);
    adam1(p.z, a.z, b.z, g.z, h);
    adam1(p.w, a.w, b.w, g.w, h);
    st4(param + 4 * i, p);
    st4(m + 4 * i, a);
    st4(v + 4 * i, b);
  }
}

__global__ void adam_tail_kernel(float *param, const float *grad, float *m, float *v,
                                 int64_t begin, int64_t n, mirec_adam_hparams_t hv,
                                 const mirec_adam_hparams_t *hp) {
  const mirec_adam_hparams_t h = hparams(hv, hp);
  const int64_t i = begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) adam1(param[i], m[i], v[i], grad[i], h);
}

// Multi-tensor Adam: up to kAdamMulti (param, grad, m, v) tensors with the
// same hyper-parameters in one launch (the pointer table travels in the
// kernel arguments).  Work item i is float i of the concatenation; the
// tensor is found by a scan of the prefix offsets (<= 32 entries).
constexpr int kAdamMulti = 32;
struct AdamMultiArgs {
  float *p[kAdamMulti];
  const float *g[kAdamMulti];
  float *m[kAdamMulti];
  float *v[kAdamMulti];
  int64_t off[kAdamMulti + 1];
  int32_t count;
  mirec_adam_hparams_t h;
  const mirec_adam_hparams_t *hp;
};

__global__ __launch_bounds__(256) void adam_multi_kernel(AdamMultiArgs a) {
  const mirec_adam_hparams_t h = hparams(a.h, a.hp);
  const int64_t total = a.off[a.count];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    int t = 0;
    while (a.off[t + 1] <= i) ++t;
    const int64_t j = i - a.off[t];
    float pv = a.p[t][j], mv = a.m[t][j], vv = a.v[t][j];
    adam1(pv, mv, vv, a.g[t][j], h);
    a.p[t][j] = pv;
    a.m[t][j] = mv;
    a.v[t][j] = vv;
  }
}

}  // namespace mirec

static int adam_multi(int32_t count, float *const *params, const float *const *grads,
                      float *const *exp_avg, float *const *exp_avg_sq, const int64_t *numel,
                      const mirec_adam_hparams_t *h, const mirec_adam_hparams_t *h_dev,
                      mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(count >= 0 && (h || h_dev) &&
                  (count == 0 || (params && grads && exp_avg && exp_avg_sq && numel)));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int32_t b = 0; b < count; b += kAdamMulti) {
    AdamMultiArgs a;
    a.count = std::min(kAdamMulti, count - b);
    a.h = h ? *h : mirec_adam_hparams_t{};
    a.hp = h_dev;
    a.off[0] = 0;
    for (int t = 0; t < a.count; ++t) {
      MIREC_CHECK_ARG(params[b + t] && grads[b + t] && exp_avg[b + t] && exp_avg_sq[b + t] &&
                      numel[b + t] >= 0);
      a.p[t] = params[b + t];
      a.g[t] = grads[b + t];
      a.m[t] = exp_avg[b + t];
      a.v[t] = exp_avg_sq[b + t];
      a.off[t + 1] = a.off[t] + numel[b + t];
    }
    const int64_t total = a.off[a.count];
    if (total == 0) continue;
    const int64_t blocks = std::min<int64_t>((total + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(adam_multi_kernel, dim3(blocks), dim3(256), 0, st, a);
    MIREC_LAUNCH_CHECK();
  }
  return MIREC_OK;
}

static int adam_dense(float *param, const float *grad, float *exp_avg, float *exp_avg_sq,
                      int64_t n, const mirec_adam_hparams_t *h, const mirec_adam_hparams_t *h_dev,
                      mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && (h || h_dev) && n >= 0);
  const mirec_adam_hparams_t hv = h ? *h : mirec_adam_hparams_t{};
  MIREC_CHECK_ARG(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg |
                   (uintptr_t)exp_avg_sq) % 16 == 0);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n4 = n / 4;
  if (n4 > 0) {
    // enough workgroups to keep ~8 float4 streams per CU in flight at
    // table sizes (a 4096-block grid-stride loop measured 3.9 TB/s)
    const int64_t blocks = std::min<int64_t>((n4 + 255) / 256, 65536);
    hipLaunchKernelGGL(adam_dense_kernel, dim3(blocks), dim3(256), 0, st, param, grad, exp_avg,
                       exp_avg_sq, n4, hv, h_dev);
    MIREC_LAUNCH_CHECK();
  }
  if (n4 * 4 < n) {
    hipLaunchKernelGGL(adam_tail_kernel, dim3(1), dim3(64), 0, st, param, grad, exp_avg,
                       exp_avg_sq, n4 * 4, n, hv, h_dev);
    MIREC_LAUNCH_CHECK();
  }
  return MIREC_OK;
}

extern "C" int mirec_adam_dense(float *param, const float *grad, float *exp_avg, float *exp_avg_sq,
                                int64_t n, const mirec_adam_hparams_t *h,
                                mirec_stream_t stream) {
  return adam_dense(param, grad, exp_avg, exp_avg_sq, n, h, nullptr, stream);
}

extern "C" int mirec_adam_dense_dev(float *param, const float *grad, float *exp_avg,
                                    float *exp_avg_sq, int64_t n,
                                    const mirec_adam_hparams_t *h_device, mirec_stream_t stream) {
  return adam_dense(param, grad, exp_avg, exp_avg_sq, n, nullptr, h_device, stream);
}

extern "C" int mirec_adam_multi(int32_t count, float *const *params, const float *const *grads,
                                float *const *exp_avg, float *const *exp_avg_sq,
                                const int64_t *numel, const mirec_adam_hparams_t *h,
                                mirec_stream_t stream) {
  return adam_multi(count, params, grads, exp_avg, exp_avg_sq, numel, h, nullptr, stream);
}

extern "C" int mirec_adam_multi_dev(int32_t count, float *const *params,
                                    const float *const *grads, float *const *exp_avg,
                                    float *const *exp_avg_sq, const int64_t *numel,
                                    const mirec_adam_hparams_t *h_device,
                                    mirec_stream_t stream) {
  return adam_multi(count, params, grads, exp_avg, exp_avg_sq, numel, nullptr, h_device, stream);
}
