// SASRec causal self-attention core on gfx950 MFMA (model/sasrec.py:385-397:
// torch.nn.MultiheadAttention with a causal mask, T <= 50).
//
// One 256-thread workgroup (4 waves) per (sequence b, head h), sequences of
// up to 64 positions cut into nb = ceil(T/16) blocks of 16.  Every product is
// built from v_mfma_f32_16x16x4_f32 tiles — exact f32 FMAs, so the 1e-4 fp32
// parity holds without reduced precision — and only the causal (lower
// triangular) block pairs are computed, so a sequence of length T costs
// ~nb(nb+1)/2 tile pairs, not a padded 64 x 64 square.
//
// The scores are kept TRANSPOSED, Sᵀ = K Qᵀ (keys on the accumulator rows,
// queries on the lanes): the softmax over keys is then a per-lane reduction
// plus two lane shuffles, and Pᵀ sits in registers in exactly the layout the
// next MFMA takes as its B operand (Oᵀ = Vᵀ Pᵀ sums over Pᵀ's row index), so
// P never goes through LDS in the forward.  The contraction over head dims in
// Sᵀ uses a permuted dim order (lane group g owns dims g*DPAD/4 ..), which
// lets each lane hold its query row segment as a few float4 registers.
//
// Forward, wave w = query block w:   Sᵀ_kb = K_kb Q_wᵀ (kb <= w), scale,
//   causal mask, column softmax -> Pᵀ; Oᵀ = Σ_kb Vᵀ_kb Pᵀ_kb; store O rows.
// Backward, phase A (wave w = query block w): recompute Pᵀ; dPᵀ = V dOᵀ;
//   δ_q = Σ_k P dP; dSᵀ = Pᵀ ⊙ (dPᵀ − δ) / sqrt(dh); dQᵀ = Kᵀ dSᵀ -> store;
//   Pᵀ, dSᵀ tiles -> LDS.  Phase B (wave w = key block w): dVᵀ = Σ_q dOᵀ P,
//   dKᵀ = Σ_q Qᵀ dS over the query blocks >= w -> store.
// LDS (head dim padded to DPAD = 32 / 64): forward K, V (35 KB at DPAD 64);
// backward K, V (later reused for Q, dO) + Pᵀ, dSᵀ (76 KB): 4 / 2
// workgroups per CU.  Row strides are chosen so the strided operand reads
// and the tile writes hit 64 distinct banks.
// q/k/v are read straight from the packed in-projection output (head h =
// columns h*dh .. of each third); O / dQKV are written in the same layout.
// Sequences come either as a uniform [B, T, 3d] batch or packed by offsets.
#include <algorithm>

#include "common.h"

namespace mirec {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kT = 64;  // longest sequence
constexpr int kB = 16;  // block edge = MFMA tile edge
constexpr int kLdP = kT + 4;  // Pᵀ / dSᵀ row stride (≡ 4 mod 64 floats)

template <int DPAD>
struct AttnShape {
  static constexpr int Q4 = DPAD / 4;     // dims per lane group in the S products
  static constexpr int NCB = DPAD / kB;   // 16-dim output blocks
  static constexpr int LDK = DPAD + 4;    // K / V row stride (4 rows ≡ 16 mod 64)
  static constexpr int LDQ = DPAD == 64 ? 80 : 48;  // Q / dO (phase B) row stride
};

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// Rows of sequence b: [row0, row0 + T) — uniform (b*T, T) or from offsets.
__device__ __forceinline__ void seq_rows(const int32_t *offsets, int b, int &T, int64_t &row0) {
  if (offsets == nullptr) {
    row0 = (int64_t)b * T;
  } else {
    row0 = offsets[b];
    T = min(offsets[b + 1] - offsets[b], kT);
  }
}

// Rows [0, R) of two head slices (row stride rs) into LDS tiles with row
// stride LD: rows >= T and columns >= dh are zero (padding must be finite:
// a masked score still multiplies a V row).  All loads are issued before
// the first LDS store.  float4 when dh % 4 == 0 (rows 16-byte aligned).
template <int DPAD, int LD>
__device__ __forceinline__ void load_pair(float *d0, float *d1, const float *s0, const float *s1,
                                          int64_t rs, int T, int R, int dh) {
  constexpr int C4 = DPAD / 4;
  constexpr int PER = kT * C4 / 256;
  if ((dh & 3) == 0) {
    float4 v0[PER], v1[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = threadIdx.x + q * 256, i = e / C4, c = e % C4;
      const bool ok = i < T && 4 * c < dh;
      v0[q] = ok ? ld4(s0 + (int64_t)i * rs + 4 * c) : f4_zero();
      v1[q] = ok ? ld4(s1 + (int64_t)i * rs + 4 * c) : f4_zero();
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = threadIdx.x + q * 256, i = e / C4, c = e % C4;
      if (i < R) {
        st4(d0 + i * LD + 4 * c, v0[q]);
        st4(d1 + i * LD + 4 * c, v1[q]);
      }
    }
  } else {
    constexpr int PS = kT * DPAD / 256;
    float v0[PS], v1[PS];
#pragma unroll
    for (int q = 0; q < PS; ++q) {
      const int e = threadIdx.x + q * 256, i = e / DPAD, c = e % DPAD;
      const bool ok = i < T && c < dh;
      v0[q] = ok ? s0[(int64_t)i * rs + c] : 0.f;
      v1[q] = ok ? s1[(int64_t)i * rs + c] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < PS; ++q) {
      const int e = threadIdx.x + q * 256, i = e / DPAD, c = e % DPAD;
      if (i < R) {
        d0[i * LD + c] = v0[q];
        d1[i * LD + c] = v1[q];
      }
    }
  }
}

// A lane's Q4 dims [c0, c0 + Q4) of one row (zero if !valid or past dh).
template <int Q4>
__device__ __forceinline__ void load_seg(const float *row, int c0, int dh, bool valid,
                                         float (&v)[Q4]) {
  if (valid && (dh & 3) == 0) {
#pragma unroll
    for (int t = 0; t < Q4; t += 4) {
      const float4 x = (c0 + t < dh) ? ld4(row + c0 + t) : f4_zero();
      v[t] = x.x;
      v[t + 1] = x.y;
      v[t + 2] = x.z;
      v[t + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int t = 0; t < Q4; ++t) v[t] = (valid && c0 + t < dh) ? row[c0 + t] : 0.f;
  }
}

// Store the 4 dims [c, c+4) held in a tile register group to row `row`.
__device__ __forceinline__ void store4(float *row, int c, int dh, f32x4 x) {
  if ((dh & 3) == 0) {
    if (c < dh) st4(row + c, make_float4(x[0], x[1], x[2], x[3]));
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (c + r < dh) row[c + r] = x[r];
  }
}

// Pᵀ for query block w (key blocks 0..w) in registers: s[kb][r] =
// P[query 16w + j][key 16kb + 4g + r] (j = lane & 15, g = lane >> 4).
template <int DPAD>
__device__ __forceinline__ void scores_softmax(const float *sK, const float (&q)[DPAD / 4], int w,
                                               int T, float scale, f32x4 (&s)[4]) {
  using S = AttnShape<DPAD>;
  const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) s[kb] = zero4();
#pragma unroll
  for (int t = 0; t < S::Q4; ++t) {
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
      if (kb <= w) s[kb] = mfma16(sK[(kB * kb + j) * S::LDK + g * S::Q4 + t], q[t], s[kb]);
  }
  const int qi = kB * w + j;
  float m = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    if (kb > w) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = kB * kb + 4 * g + r;
      const float v = (key > qi || key >= T) ? -INFINITY : s[kb][r] * scale;
      s[kb][r] = v;
      m = fmaxf(m, v);
    }
  }
  m = fmaxf(m, __shfl_xor(m, 16));
  m = fmaxf(m, __shfl_xor(m, 32));
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    if (kb > w) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = expf(s[kb][r] - m);
      s[kb][r] = e;
      sum += e;
    }
  }
  sum += __shfl_xor(sum, 16);
  sum += __shfl_xor(sum, 32);
  const float inv = 1.f / sum;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    if (kb > w) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) s[kb][r] *= inv;
  }
}

template <int DPAD>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const float *__restrict__ qkv,
                                                       float *__restrict__ out, int T, int H,
                                                       int dh, float scale,
                                                       const int32_t *__restrict__ offsets) {
  using S = AttnShape<DPAD>;
  __shared__ __attribute__((aligned(16))) float sK[kT * S::LDK];
  __shared__ __attribute__((aligned(16))) float sV[kT * S::LDK];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int b = blockIdx.x / H, h = blockIdx.x - (blockIdx.x / H) * H;
  const int d = H * dh;
  const int64_t rs = 3 * (int64_t)d;
  int64_t row0;
  seq_rows(offsets, b, T, row0);
  const int nb = (T + kB - 1) / kB;
  const float *base = qkv + row0 * rs + h * dh;
  load_pair<DPAD, S::LDK>(sK, sV, base + d, base + 2 * d, rs, T, kB * nb, dh);
  const int qi = kB * w + j;
  float q[S::Q4];
  load_seg<S::Q4>(base + (int64_t)qi * rs, g * S::Q4, dh, w < nb && qi < T, q);
  __syncthreads();
  if (w >= nb) return;  // no barrier below
  f32x4 p[4];
  scores_softmax<DPAD>(sK, q, w, T, scale, p);
  f32x4 o[S::NCB];
#pragma unroll
  for (int cb = 0; cb < S::NCB; ++cb) o[cb] = zero4();
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    if (kb > w) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float *vrow = sV + (kB * kb + 4 * g + r) * S::LDK + j;
#pragma unroll
      for (int cb = 0; cb < S::NCB; ++cb) o[cb] = mfma16(vrow[kB * cb], p[kb][r], o[cb]);
    }
  }
  if (qi < T) {
    float *orow = out + (row0 + qi) * d + h * dh;
#pragma unroll
    for (int cb = 0; cb < S::NCB; ++cb) store4(orow, kB * cb + 4 * g, dh, o[cb]);
  }
}

template <int DPAD>
__global__ __launch_bounds__(256) void attn_bwd_kernel(const float *__restrict__ qkv,
                                                       const float *__restrict__ dout,
                                                       float *__restrict__ dqkv, int T, int H,
                                                       int dh, float scale,
                                                       const int32_t *__restrict__ offsets) {
  using S = AttnShape<DPAD>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int kv = 2 * kT * S::LDK, qd = 2 * kT * S::LDQ;
  constexpr int region = kv > qd ? kv : qd;
  float *sK = smem, *sV = smem + kT * S::LDK;           // phase A
  float *sQ = smem, *sDO = smem + kT * S::LDQ;          // phase B (same region)
  float *sP = smem + region, *sDS = sP + kT * kLdP;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int b = blockIdx.x / H, h = blockIdx.x - (blockIdx.x / H) * H;
  const int d = H * dh;
  const int64_t rs = 3 * (int64_t)d;
  int64_t row0;
  seq_rows(offsets, b, T, row0);
  const int nb = (T + kB - 1) / kB;
  const float *base = qkv + row0 * rs + h * dh;
  float *gbase = dqkv + row0 * rs + h * dh;
  load_pair<DPAD, S::LDK>(sK, sV, base + d, base + 2 * d, rs, T, kB * nb, dh);
  const int qi = kB * w + j;
  const bool qvalid = w < nb && qi < T;
  float q[S::Q4], dov[S::Q4];
  load_seg<S::Q4>(base + (int64_t)qi * rs, g * S::Q4, dh, qvalid, q);
  load_seg<S::Q4>(dout + (row0 + qi) * d + h * dh, g * S::Q4, dh, qvalid, dov);
  __syncthreads();
  // ---------------------------------------------------- phase A: query block w
  if (w < nb) {
    f32x4 p[4], dp[4];
    scores_softmax<DPAD>(sK, q, w, T, scale, p);
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) dp[kb] = zero4();
#pragma unroll
    for (int t = 0; t < S::Q4; ++t) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
        if (kb <= w) dp[kb] = mfma16(sV[(kB * kb + j) * S::LDK + g * S::Q4 + t], dov[t], dp[kb]);
    }
    float delta = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      if (kb > w) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) delta += p[kb][r] * dp[kb][r];
    }
    delta += __shfl_xor(delta, 16);
    delta += __shfl_xor(delta, 32);
    // dSᵀ (in dp), then dQᵀ = Kᵀ dSᵀ
    f32x4 dq[S::NCB];
#pragma unroll
    for (int cb = 0; cb < S::NCB; ++cb) dq[cb] = zero4();
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      if (kb > w) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dp[kb][r] = p[kb][r] * (dp[kb][r] - delta) * scale;
        const int key = kB * kb + 4 * g + r;
        sP[key * kLdP + qi] = p[kb][r];
        sDS[key * kLdP + qi] = dp[kb][r];
        const float *krow = sK + key * S::LDK + j;
#pragma unroll
        for (int cb = 0; cb < S::NCB; ++cb) dq[cb] = mfma16(krow[kB * cb], dp[kb][r], dq[cb]);
      }
    }
    if (qi < T) {
      float *row = gbase + (int64_t)qi * rs;
#pragma unroll
      for (int cb = 0; cb < S::NCB; ++cb) store4(row, kB * cb + 4 * g, dh, dq[cb]);
    }
  }
  __syncthreads();  // K / V no longer read; Pᵀ, dSᵀ complete
  if (w < nb) {
#pragma unroll
    for (int t = 0; t < S::Q4; ++t) {
      sQ[qi * S::LDQ + g * S::Q4 + t] = q[t];
      sDO[qi * S::LDQ + g * S::Q4 + t] = dov[t];
    }
  }
  __syncthreads();
  // ------------------------------------------------------ phase B: key block w
  if (w < nb) {
    const int kb = w;
    f32x4 dv[S::NCB], dk[S::NCB];
#pragma unroll
    for (int cb = 0; cb < S::NCB; ++cb) {
      dv[cb] = zero4();
      dk[cb] = zero4();
    }
    const int key = kB * kb + j;
    for (int q0 = kB * kb; q0 < kB * nb; q0 += 4) {
      const int qq = q0 + g;
      const float pb = sP[key * kLdP + qq];
      const float db = sDS[key * kLdP + qq];
      const float *dorow = sDO + qq * S::LDQ + j;
      const float *qrow = sQ + qq * S::LDQ + j;
#pragma unroll
      for (int cb = 0; cb < S::NCB; ++cb) {
        dv[cb] = mfma16(dorow[kB * cb], pb, dv[cb]);
        dk[cb] = mfma16(qrow[kB * cb], db, dk[cb]);
      }
    }
    if (key < T) {
      float *row = gbase + (int64_t)key * rs;
#pragma unroll
      for (int cb = 0; cb < S::NCB; ++cb) {
        store4(row + d, kB * cb + 4 * g, dh, dk[cb]);
        store4(row + 2 * d, kB * cb + 4 * g, dh, dv[cb]);
      }
    }
  }
}

template <int DPAD>
constexpr int bwd_smem() {
  using S = AttnShape<DPAD>;
  constexpr int kv = 2 * kT * S::LDK, qd = 2 * kT * S::LDQ;
  return (int)sizeof(float) * ((kv > qd ? kv : qd) + 2 * kT * kLdP);
}

// Dynamic LDS above 64 KiB needs an explicit opt-in per kernel (once).
static int allow_big_lds() {
  static int rc = -1;
  if (rc < 0) {
    rc = 0;
    const void *fns[2] = {(const void *)attn_bwd_kernel<32>, (const void *)attn_bwd_kernel<64>};
    for (const void *f : fns)
      if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
          hipSuccess)
        rc = 1;
  }
  return rc;
}

static int launch_fwd(const float *qkv, const int32_t *offsets, int64_t batch, int T,
                      int heads, int head_dim, float *out, hipStream_t st) {
  if (batch == 0) return MIREC_OK;
  const float scale = 1.f / sqrtf((float)head_dim);
  const dim3 grid((unsigned)(batch * heads));
  if (head_dim <= 32)
    hipLaunchKernelGGL(attn_fwd_kernel<32>, grid, dim3(256), 0, st, qkv, out, T, heads,
                       head_dim, scale, offsets);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), 0, st, qkv, out, T, heads,
                       head_dim, scale, offsets);
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
    hipLaunchKernelGGL(attn_bwd_kernel<32>, grid, dim3(256), bwd_smem<32>(), st, qkv, dout,
                       dqkv, T, heads, head_dim, scale, offsets);
  else
    hipLaunchKernelGGL(attn_bwd_kernel<64>, grid, dim3(256), bwd_smem<64>(), st, qkv, dout,
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
