// Shared helpers for the gfx950 kernels of libmirec.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mirec.h"

namespace mirec {

// Last HIP error seen by any entry point (exposed by mirec_last_hip_error).
extern thread_local int g_last_hip_error;

#define MIREC_CHECK_ARG(cond)                                                  \
  do {                                                                         \
    if (!(cond)) return MIREC_ERR_ARG;                                         \
  } while (0)

#define MIREC_LAUNCH_CHECK()                                                   \
  do {                                                                         \
    hipError_t e_ = hipGetLastError();                                         \
    if (e_ != hipSuccess) {                                                    \
      ::mirec::g_last_hip_error = (int)e_;                                     \
      return MIREC_ERR_HIP;                                                    \
    }                                                                          \
  } while (0)

#define MIREC_HIP(call)                                                        \
  do {                                                                         \
    hipError_t e_ = (call);                                                    \
    if (e_ != hipSuccess) {                                                    \
      ::mirec::g_last_hip_error = (int)e_;                                     \
      return MIREC_ERR_HIP;                                                    \
    }                                                                          \
  } while (0)

inline bool dim_supported(int d) {
  return d == 4 || d == 8 || d == 16 || d == 32 || d == 64 || d == 128 ||
         d == 256;
}

__device__ __forceinline__ float4 f4_zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

__device__ __forceinline__ float4 f4_add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 f4_sub(float4 a, float4 b) {
  return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
}
__device__ __forceinline__ float4 f4_scale(float s, float4 a) {
  return make_float4(s * a.x, s * a.y, s * a.z, s * a.w);
}
__device__ __forceinline__ float4 f4_fma(float s, float4 a, float4 c) {
  return make_float4(fmaf(s, a.x, c.x), fmaf(s, a.y, c.y), fmaf(s, a.z, c.z),
                     fmaf(s, a.w, c.w));
}
__device__ __forceinline__ float4 f4_div(float4 a, float d) {
  return make_float4(a.x / d, a.y / d, a.z / d, a.w / d);
}
__device__ __forceinline__ float f4_dot(float4 a, float4 b) {
  return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}
__device__ __forceinline__ float4 ld4(const float *p) {
  return *reinterpret_cast<const float4 *>(p);
}
__device__ __forceinline__ void st4(float *p, float4 v) {
  *reinterpret_cast<float4 *>(p) = v;
}
// Row movers (gather / scatter / counted gather of [n, d] float rows): a
// 256-thread block takes kRowRounds rounds of 256 >> lg rows, 1 << lg lanes
// per row (lg = ceil log2 (d / 4); lanes past d / 4 idle), every thread
// loading the ids of all its rows first, then all its rows — kRowRounds x 16
// B in flight per lane instead of one dependent (id, row) pair — and no
// 64-bit division in the index math.
constexpr int kRowRounds = 4;
inline int row_lg(int64_t d4) {
  int lg = 0;
  while ((int64_t(1) << lg) < d4) ++lg;
  return lg;
}
inline int64_t row_blocks(int64_t n, int lg) {
  const int64_t per = int64_t(256 >> lg) * kRowRounds;
  return (n + per - 1) / per;
}

__device__ __forceinline__ float4 f4_shfl_xor(float4 v, int m) {
  return make_float4(__shfl_xor(v.x, m), __shfl_xor(v.y, m),
                     __shfl_xor(v.z, m), __shfl_xor(v.w, m));
}

// Sum a float over the LPR-lane group a lane belongs to (groups are
// contiguous, aligned runs of LPR lanes inside the 64-lane wave).
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int m = 1; m < LPR; m <<= 1) v += __shfl_xor(v, m);
  return v;
}

// Softmax exponentials in the base-2 domain (attention.hip, attn_wave.hip):
// scores are scaled by scale * log2(e) once, so every exponential is ONE
// v_exp_f32 (libm expf without fast-math is a ~14-instruction range-reduced
// sequence) and a log-sum-exp is kept as lse2 = max2 + log2(sum), one
// v_log_f32.  exp2(-inf) = 0 keeps the causal mask; arguments are <= 0 and
// an underflow to 0 (v_exp_f32 flushes results below 2^-126) is a
// probability below 1e-38, zero in any f32 sum it enters.
constexpr float kLog2e = 1.4426950408889634f;
__device__ __forceinline__ float exp2_hw(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float log2_hw(float x) { return __builtin_amdgcn_logf(x); }

// Kernels with no MFMA of their own that run on the SASRec / GraphSAGE
// streams next to MFMA kernels are compiled without packed-f32 VALU ops:
// a v_pk_*_f32 whose op_sel feeds a pair's HIGH dword to the low lane
// returns 0 in the upper lanes while MFMAs execute on the same SIMD — any
// wave's, not only its own (tools/op_sel_repro.hip).  The
// attribute is a device-compilation feature switch (the host pass has no
// such feature).
#if defined(__HIP_DEVICE_COMPILE__)
#define MIREC_NO_PK_F32 __attribute__((target("no-packed-fp32-ops")))
#else
#define MIREC_NO_PK_F32
#endif

// Counter-hash dropout shared by the fused kernels: the four elements of an
// aligned quad (idx >> 2) share one mix64(key + quad); element idx & 3 takes
// its 16-bit slice and is kept iff slice >= thresh = round(p * 2^16); kept
// values are scaled by 1 / (1 - p).  The backward recomputes the mask from
// (seed, idx).  One hash per float4 (the kernels' unit) instead of per
// element: the hashing was the ALU floor of the dropout-mean gathers.
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ bool keep(uint64_t key, uint64_t idx, uint32_t thresh) {
  const uint64_t h = mix64(key + (idx >> 2));
  return (uint32_t)((h >> (16 * (idx & 3))) & 0xffffu) >= thresh;
}

// v * mask * scale for the quad with hash input hq = key + quad index.
__device__ __forceinline__ float4 drop4_hq(float4 v, uint64_t hq, uint32_t thresh, float scale) {
  const uint64_t h = mix64(hq);
  v.x = (uint32_t)(h & 0xffffu) >= thresh ? v.x * scale : 0.f;
  v.y = (uint32_t)((h >> 16) & 0xffffu) >= thresh ? v.y * scale : 0.f;
  v.z = (uint32_t)((h >> 32) & 0xffffu) >= thresh ? v.z * scale : 0.f;
  v.w = (uint32_t)(h >> 48) >= thresh ? v.w * scale : 0.f;
  return v;
}

// v * mask * scale for elements idx .. idx + 3 (idx % 4 == 0): one hash.
__device__ __forceinline__ float4 drop4(float4 v, uint64_t key, uint64_t idx, uint32_t thresh,
                                        float scale) {
  return drop4_hq(v, key + (idx >> 2), thresh, scale);
}

// The mask key of a launch: the host key, mixed with *key_base (device, a
// captured graph's per-replay seed base) when given.
__device__ __forceinline__ uint64_t run_key(uint64_t key, const uint64_t *key_base) {
  return key_base ? mix64(key ^ *key_base) : key;
}

static inline bool dropout_params(float p, uint64_t seed, uint64_t *key, uint32_t *thresh, float *scale) {
  if (!(p >= 0.f && p < 1.f)) return false;
  *key = mix64(seed ^ 0xA24BAED4963EE407ull);
  *thresh = (uint32_t)((double)p * 65536.0 + 0.5);
  *scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  if (p > 0.f && *thresh == 0u) *thresh = 1u;
  if (*thresh > 65535u) *thresh = 65535u;
  return true;
}

// One element of torch.optim.Adam (amsgrad=False, weight_decay=0): every
// Adam kernel uses this one expression, written with explicit fmas so the
// compiler's contraction choices cannot differ between kernels (fused and
// unfused steps agree bitwise).
__device__ __forceinline__ void adam1(float &p, float &m, float &v, float g,
                                      const mirec_adam_hparams_t &h) {
  m = fmaf(h.one_minus_beta1, g - m, m);
  v = fmaf(v, h.beta2, h.one_minus_beta2 * (g * g));
  const float denom = sqrtf(v) / h.bc2_sqrt + h.eps;
  p = fmaf(h.neg_step_size, m / denom, p);
}

// ---- exact three-term bf16 split of f32 operands (gemm.hip, attention.hip)
// x = x_h + x_m + x_l, each term rounded to nearest; the residuals are exact
// in f32 (error analysis: gemm.hip, "f32 products on bf16 MFMA").
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Split3 {
  bf16x8 h, m, l;
};

// packed RNE (a in the low half)
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

// x[0..7] -> three bf16x8 planes (element e of every plane is x[e]'s term)
__device__ __forceinline__ Split3 split3(const float (&x)[8]) {
  u32x4 H, M, L;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float a = x[2 * p], b = x[2 * p + 1];
    const uint32_t ph = pk_bf16(a, b);
    const float ra = a - __uint_as_float(ph << 16), rb = b - __uint_as_float(ph & 0xffff0000u);
    const uint32_t pm = pk_bf16(ra, rb);
    const float sa = ra - __uint_as_float(pm << 16), sb = rb - __uint_as_float(pm & 0xffff0000u);
    H[p] = ph;
    M[p] = pm;
    L[p] = pk_bf16(sa, sb);
  }
  return Split3{__builtin_bit_cast(bf16x8, H), __builtin_bit_cast(bf16x8, M),
                __builtin_bit_cast(bf16x8, L)};
}

typedef float f32x16 __attribute__((ext_vector_type(16)));

// C += A·B over one 16-deep k block: lane (i, h) supplies row / column i's
// 8 k values of its half (any k order, the same for A and B)
__device__ __forceinline__ f32x16 mfma_x6(const Split3 &a, const Split3 &b, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, b.h, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.l, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.m, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.h, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.m, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.h, c, 0, 0, 0);
  return c;
}

// The k order of a lane half h inside a 16-deep block: element e < 4 is k =
// 4 h + e, e >= 4 is 8 + 4 h + (e - 4) — two float4 reads of a [row][k] LDS
// row, and on a [k][col] image the two halves' rows are 4 apart (32 banks at
// the row strides used here), as in the f32 form's sub-chunks.
__device__ __forceinline__ int x6_k(int h, int e) { return 4 * h + (e & 3) + 8 * (e >> 2); }

}  // namespace mirec
