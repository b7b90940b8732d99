// SASRec causal self-attention core on gfx950 MFMA (model/sasrec.py:385-397:
// torch.nn.MultiheadAttention with a causal mask, T <= 50).
//
// One 256-thread workgroup (4 waves) per (sequence b, head h).  The T <= 64
// rows of Q, K, V for the head are staged in LDS (row stride dh+1: no bank
// conflicts on column reads), then every product is a handful of 32x32 tiles
// of v_mfma_f32_32x32x2_f32 — exact f32 FMAs (bitwise a k-ordered fmaf
// chain), so the 1e-4 fp32 parity holds without any reduced precision:
//   S = Q Kᵀ · 1/sqrt(dh) (+ causal -inf)   4 tiles, one per wave
//   P = softmax_rows(S)                     4 lanes per row, in LDS
//   O = P V                                 2 x dh/32 tiles
// Backward (recomputes S, P): dV = Pᵀ dO, dP = dO Vᵀ,
// dS = P ⊙ (dP − rowsum(dP ⊙ P)) / sqrt(dh), dQ = dS K, dK = dSᵀ Q.
// q/k/v are read straight from the packed in-projection output [B, T, 3d]
// (head h = columns h*dh .. h*dh+dh of each third) and O / dQKV are written
// in the same packed layouts, so the surrounding Linear layers are plain
// library GEMMs.  Any head dim <= 64: it is zero-padded to 32 or 64 in LDS.
#include <algorithm>

#include "common.h"

namespace mirec {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kT = 64;  // padded sequence tile

// 32x32 tile D += A·B over K (multiple of 2) with operands in LDS:
//   A(i, k) = TA ? A[k*lda + i] : A[i*lda + k]
//   B(k, j) = TB ? B[j*ldb + k] : B[k*ldb + j]
// lane l feeds A(i=l&31, k=2s+(l>>5)) and B(k=2s+(l>>5), j=l&31).
template <bool TA, bool TB>
__device__ __forceinline__ f32x16 mfma_tile(const float *A, int lda, const float *B, int ldb,
                                            int K, f32x16 acc, int lane) {
  const int r = lane & 31, h = lane >> 5;
  for (int s = 0; s < K; s += 2) {
    const int k = s + h;
    const float a = TA ? A[k * lda + r] : A[r * lda + k];
    const float b = TB ? B[r * ldb + k] : B[k * ldb + r];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
  return acc;
}

__device__ __forceinline__ int acc_row(int reg, int lane) {
  return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// Load rows [0, T) of NT heads (packed [B, T, *] tensors with row strides
// rs[t]) into LDS tiles [kT][ld] (zero rows T..kT-1 and columns dh..DPAD-1).
// Every load of all NT tiles is issued before the first LDS store, so the
// workgroup pays one HBM latency, not one per element.  float4 loads when
// dh % 4 == 0 (then rows are 16-byte aligned), scalar otherwise.
template <int DPAD, int NT>
__device__ __forceinline__ void load_heads(float *const (&dst)[NT], const float *const (&src)[NT],
                                           const int64_t (&rs)[NT], int ld, int T, int dh) {
  if ((dh & 3) == 0) {
    constexpr int C4 = DPAD / 4;
    constexpr int PER = kT * C4 / 256;
    float4 v[NT][PER];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int e = threadIdx.x + q * 256, i = e / C4, c = e % C4;
        v[t][q] = (i < T && 4 * c < dh) ? ld4(src[t] + (int64_t)i * rs[t] + 4 * c) : f4_zero();
      }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int e = threadIdx.x + q * 256, i = e / C4, c = e % C4;
        float *d = dst[t] + i * ld + 4 * c;
        d[0] = v[t][q].x;
        d[1] = v[t][q].y;
        d[2] = v[t][q].z;
        d[3] = v[t][q].w;
      }
  } else {
    constexpr int PER = kT * DPAD / 256;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float v[PER];
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int e = threadIdx.x + q * 256, i = e / DPAD, c = e % DPAD;
        v[q] = (i < T && c < dh) ? src[t][(int64_t)i * rs[t] + c] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int e = threadIdx.x + q * 256, i = e / DPAD, c = e % DPAD;
        dst[t][i * ld + c] = v[q];
      }
    }
  }
}

// S = scale * Q Kᵀ with the causal mask, written to sS [kT][kT+1]; then
// row softmax in place (P).  Rows >= T are computed too (finite, unused).
// sS may alias sQ (the products are in registers before it is written).
__device__ void scores_softmax(const float *sQ, const float *sK, int ld, float *sS, int dpad,
                               float scale) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qi = w >> 1, qj = w & 1;
  f32x16 acc = mfma_tile<false, true>(sQ + 32 * qi * ld, ld, sK + 32 * qj * ld, ld, dpad,
                                      zero16(), lane);
  if ((const float *)sS == sQ) __syncthreads();  // every wave is done reading sQ
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = 32 * qi + acc_row(r, lane), j = 32 * qj + (lane & 31);
    sS[i * (kT + 1) + j] = j > i ? -INFINITY : acc[r] * scale;
  }
  __syncthreads();
  // 4 lanes per row, 16 columns each
  const int row = threadIdx.x >> 2, part = threadIdx.x & 3;
  float *srow = sS + row * (kT + 1) + part * 16;
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < 16; ++c) m = fmaxf(m, srow[c]);
  m = fmaxf(m, __shfl_xor(m, 1));
  m = fmaxf(m, __shfl_xor(m, 2));
  float e[16], sum = 0.f;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    e[c] = expf(srow[c] - m);
    sum += e[c];
  }
  sum += __shfl_xor(sum, 1);
  sum += __shfl_xor(sum, 2);
  const float inv = 1.f / sum;
#pragma unroll
  for (int c = 0; c < 16; ++c) srow[c] = e[c] * inv;
  __syncthreads();
}

// Rows of sequence b: [row0, row0 + T) — uniform (b*T, T) or from offsets.
__device__ __forceinline__ void seq_rows(const int32_t *offsets, int b, int &T, int64_t &row0) {
  if (offsets == nullptr) {
    row0 = (int64_t)b * T;
  } else {
    row0 = offsets[b];
    T = min(offsets[b + 1] - offsets[b], kT);
  }
}

template <int DPAD>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const float *__restrict__ qkv,
                                                       float *__restrict__ out, int T, int H,
                                                       int dh, float scale,
                                                       const int32_t *__restrict__ offsets) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int ld = DPAD + 1;
  // P overwrites Q: [sQ | sS] [sK] [sV]
  constexpr int qs = kT * ld > kT * (kT + 1) ? kT * ld : kT * (kT + 1);
  float *sQ = smem, *sS = smem, *sK = smem + qs, *sV = sK + kT * ld;
  const int b = blockIdx.x / H, h = blockIdx.x - (blockIdx.x / H) * H;
  const int d = H * dh;
  const int64_t rs = 3 * (int64_t)d;
  int64_t row0;
  seq_rows(offsets, b, T, row0);
  const float *base = qkv + row0 * rs + h * dh;
  {
    float *const dst[3] = {sQ, sK, sV};
    const float *const src[3] = {base, base + d, base + 2 * d};
    const int64_t strides[3] = {rs, rs, rs};
    load_heads<DPAD, 3>(dst, src, strides, ld, T, dh);
  }
  __syncthreads();
  scores_softmax(sQ, sK, ld, sS, DPAD, scale);
  // O = P V: tiles (oi, oj) over 2 x DPAD/32, strided over the 4 waves
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int ntiles = 2 * (DPAD / 32);
  for (int t = w; t < ntiles; t += 4) {
    const int oi = t & 1, oj = t >> 1;
    f32x16 acc = mfma_tile<false, false>(sS + 32 * oi * (kT + 1), kT + 1, sV + 32 * oj, ld, kT,
                                         zero16(), lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = 32 * oi + acc_row(r, lane), c = 32 * oj + (lane & 31);
      if (i < T && c < dh) out[(row0 + i) * d + h * dh + c] = acc[r];
    }
  }
}

template <int DPAD>
__global__ __launch_bounds__(256) void attn_bwd_kernel(const float *__restrict__ qkv,
                                                       const float *__restrict__ dout,
                                                       float *__restrict__ dqkv, int T, int H,
                                                       int dh, float scale,
                                                       const int32_t *__restrict__ offsets) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int dpad = DPAD;
  constexpr int ld = DPAD + 1;
  float *sQ = smem, *sK = sQ + kT * ld, *sV = sK + kT * ld, *sO = sV + kT * ld;
  float *sP = sO + kT * ld, *sD = sP + kT * (kT + 1);
  const int b = blockIdx.x / H, h = blockIdx.x - (blockIdx.x / H) * H;
  const int d = H * dh;
  const int64_t rs = 3 * (int64_t)d;
  int64_t row0;
  seq_rows(offsets, b, T, row0);
  const float *base = qkv + row0 * rs + h * dh;
  {
    float *const dst[4] = {sQ, sK, sV, sO};
    const float *const src[4] = {base, base + d, base + 2 * d, dout + row0 * d + h * dh};
    const int64_t strides[4] = {rs, rs, rs, (int64_t)d};  // sO = dO
    load_heads<DPAD, 4>(dst, src, strides, ld, T, dh);
  }
  __syncthreads();
  scores_softmax(sQ, sK, ld, sP, dpad, scale);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float *gbase = dqkv + row0 * rs + h * dh;
  // dV = Pᵀ dO  (rows j, cols c; K = i)
  constexpr int ntiles = 2 * (dpad / 32);
  for (int t = w; t < ntiles; t += 4) {
    const int ti = t & 1, tj = t >> 1;
    f32x16 acc = mfma_tile<true, false>(sP + 32 * ti, kT + 1, sO + 32 * tj, ld, kT, zero16(), lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = 32 * ti + acc_row(r, lane), c = 32 * tj + (lane & 31);
      if (j < T && c < dh) gbase[(int64_t)j * rs + 2 * d + c] = acc[r];
    }
  }
  // dP = dO Vᵀ (K = dpad) -> sD, one 32x32 tile per wave
  {
    const int qi = w >> 1, qj = w & 1;
    f32x16 acc = mfma_tile<false, true>(sO + 32 * qi * ld, ld, sV + 32 * qj * ld, ld, dpad,
                                        zero16(), lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = 32 * qi + acc_row(r, lane), j = 32 * qj + (lane & 31);
      sD[i * (kT + 1) + j] = acc[r];
    }
  }
  __syncthreads();
  // dS = P ⊙ (dP − Σ_j dP P) · scale, in place in sD (4 lanes per row)
  {
    const int row = threadIdx.x >> 2, part = threadIdx.x & 3;
    float *prow = sP + row * (kT + 1) + part * 16;
    float *drow = sD + row * (kT + 1) + part * 16;
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) dot += prow[c] * drow[c];
    dot += __shfl_xor(dot, 1);
    dot += __shfl_xor(dot, 2);
#pragma unroll
    for (int c = 0; c < 16; ++c) drow[c] = prow[c] * (drow[c] - dot) * scale;
  }
  __syncthreads();
  for (int t = w; t < 2 * ntiles; t += 4) {
    const bool is_q = t < ntiles;
    const int tt = is_q ? t : t - ntiles;
    const int ti = tt & 1, tj = tt >> 1;
    f32x16 acc;
    if (is_q)  // dQ = dS K: rows i, cols k, K = j
      acc = mfma_tile<false, false>(sD + 32 * ti * (kT + 1), kT + 1, sK + 32 * tj, ld, kT,
                                    zero16(), lane);
    else  // dK = dSᵀ Q: rows j, cols k, K = i
      acc = mfma_tile<true, false>(sD + 32 * ti, kT + 1, sQ + 32 * tj, ld, kT, zero16(), lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = 32 * ti + acc_row(r, lane), c = 32 * tj + (lane & 31);
      if (i < T && c < dh) gbase[(int64_t)i * rs + (is_q ? 0 : d) + c] = acc[r];
    }
  }
}

// Dynamic LDS above 64 KiB needs an explicit opt-in per kernel (once).
static int allow_big_lds() {
  static int rc = -1;
  if (rc < 0) {
    rc = 0;
    const void *fns[4] = {(const void *)attn_fwd_kernel<32>, (const void *)attn_fwd_kernel<64>,
                          (const void *)attn_bwd_kernel<32>, (const void *)attn_bwd_kernel<64>};
    for (const void *f : fns)
      if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
          hipSuccess)
        rc = 1;
  }
  return rc;
}

static int attn_smem(int dpad, bool bwd) {
  const int ld = dpad + 1;
  const int qs = std::max(kT * ld, kT * (kT + 1));  // forward: P overwrites Q
  return (int)sizeof(float) * (bwd ? (4 * kT * ld + 2 * kT * (kT + 1)) : (qs + 2 * kT * ld));
}

static int launch_fwd(const float *qkv, const int32_t *offsets, int64_t batch, int T,
                      int heads, int head_dim, float *out, hipStream_t st) {
  if (batch == 0) return MIREC_OK;
  if (allow_big_lds() != 0) return MIREC_ERR_HIP;
  const float scale = 1.f / sqrtf((float)head_dim);
  const dim3 grid((unsigned)(batch * heads));
  if (head_dim <= 32)
    hipLaunchKernelGGL(attn_fwd_kernel<32>, grid, dim3(256), attn_smem(32, false), st, qkv, out,
                       T, heads, head_dim, scale, offsets);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), attn_smem(64, false), st, qkv, out,
                       T, heads, head_dim, scale, offsets);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

static int launch_bwd(const float *qkv, const float *dout, const int32_t *offsets,
                      int64_t batch, int T, int heads, int head_dim, float *dqkv,
                      hipStream_t st) {
  if (batch == 0) return MIREC_OK;
  if (allow_big_lds() != 0) return MIREC_ERR_HIP;
  const float scale = 1.f / sqrtf((float)head_dim);
  const dim3 grid((unsigned)(batch * heads));
  if (head_dim <= 32)
    hipLaunchKernelGGL(attn_bwd_kernel<32>, grid, dim3(256), attn_smem(32, true), st, qkv, dout,
                       dqkv, T, heads, head_dim, scale, offsets);
  else
    hipLaunchKernelGGL(attn_bwd_kernel<64>, grid, dim3(256), attn_smem(64, true), st, qkv, dout,
                       dqkv, T, heads, head_dim, scale, offsets);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

}  // namespace mirec

extern "C" int mirec_attention_fwd(const float *qkv, int64_t batch, int32_t T, int32_t heads,
                                   int32_t head_dim, float *out, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(qkv && out && batch >= 0 && T >= 1 && T <= kT && heads >= 1);
  MIREC_CHECK_ARG(head_dim >= 1 && head_dim <= 64);
  return launch_fwd(qkv, nullptr, batch, T, heads, head_dim, out,
                    reinterpret_cast<hipStream_t>(stream));
}

extern "C" int mirec_attention_bwd(const float *qkv, const float *dout, int64_t batch, int32_t T,
                                   int32_t heads, int32_t head_dim, float *dqkv,
                                   mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(qkv && dout && dqkv && batch >= 0 && T >= 1 && T <= kT && heads >= 1);
  MIREC_CHECK_ARG(head_dim >= 1 && head_dim <= 64);
  return launch_bwd(qkv, dout, nullptr, batch, T, heads, head_dim, dqkv,
                    reinterpret_cast<hipStream_t>(stream));
}

extern "C" int mirec_attention_varlen_fwd(const float *qkv, const int32_t *offsets,
                                          int64_t batch, int32_t heads, int32_t head_dim,
                                          float *out, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(qkv && offsets && out && batch >= 0 && heads >= 1);
  MIREC_CHECK_ARG(head_dim >= 1 && head_dim <= 64);
  return launch_fwd(qkv, offsets, batch, kT, heads, head_dim, out,
                    reinterpret_cast<hipStream_t>(stream));
}

extern "C" int mirec_attention_varlen_bwd(const float *qkv, const float *dout,
                                          const int32_t *offsets, int64_t batch, int32_t heads,
                                          int32_t head_dim, float *dqkv, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(qkv && dout && offsets && dqkv && batch >= 0 && heads >= 1);
  MIREC_CHECK_ARG(head_dim >= 1 && head_dim <= 64);
  return launch_bwd(qkv, dout, offsets, batch, kT, heads, head_dim, dqkv,
                    reinterpret_cast<hipStream_t>(stream));
}
