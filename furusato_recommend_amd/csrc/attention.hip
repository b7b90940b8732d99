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
// P never goes through LDS in the forward.  The contraction over head dims
// uses the dim order 4t + g (lane group g, step t), which with row strides
// ≡ 4 (mod 32) floats makes every strided operand read hit 64 distinct banks.
//
// Forward, wave w = query block w:   Sᵀ_kb = K_kb Q_wᵀ (kb <= w), scale,
//   causal mask, column softmax -> Pᵀ; Oᵀ = Σ_kb Vᵀ_kb Pᵀ_kb; store O rows.
// Backward, phase A (wave w = query block w): recompute Pᵀ; dPᵀ = V dOᵀ;
//   δ_q = Σ_k P dP; dSᵀ = Pᵀ ⊙ (dPᵀ − δ) / sqrt(dh); dQᵀ = Kᵀ dSᵀ -> store;
//   the softmax statistic (base-2 log-sum-exp) and δ of each query -> LDS, the
//   wave's own K / V block -> registers.  Phase B (wave w = key block w), per
//   query block qb >= w: S = Q_qb K_wᵀ and dP = dO_qb V_wᵀ (queries on the
//   accumulator rows, keys on the lanes — the layout in which P and dS are
//   the B operands of the next products), P and dS from the statistics;
//   dVᵀ += Σ_q dOᵀ P, dKᵀ += Σ_q Qᵀ dS -> store.  Recomputing P / dS in
//   phase B (twice its MFMAs) instead of keeping Pᵀ / dSᵀ tiles in LDS halves
//   the backward's LDS: more workgroups per CU hide the per-workgroup
//   memory latency that bounds these small problems.
// LDS (head dim padded to DPAD = 32 / 64): forward K, V (35 KB at DPAD 64,
// 16 rows per block); backward K, V, later reused for Q, dO, plus 2 floats
// per row of statistics (35 KB): 4 workgroups per CU either way.
// Softmax in base 2 (common.h exp2_hw): scores are scaled by scale·log2(e),
// every exponential is one v_exp_f32, and phase B's P = exp2(s·c − lse2)
// needs one statistic per query (read as float4 per lane group).
// q/k/v are read straight from the packed in-projection output (head h =
// columns h*dh .. of each third); O / dQKV are written in the same layout.
// Sequences come either as a uniform [B, T, 3d] batch or packed by offsets.
#include <algorithm>

#include "common.h"

namespace mirec {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kT = 64;  // longest sequence
constexpr int kB = 16;  // block edge = MFMA tile edge

// NB = number of 16-row blocks a workgroup holds (the bucket: sequences of
// at most 16*NB positions); one wave per block, so a workgroup is 64*NB
// threads and its LDS is sized for 16*NB rows.
template <int DPAD, int NB>
struct AttnShape {
  static constexpr int TR = NB * kB;      // rows held
  static constexpr int NT = 64 * NB;      // threads
  static constexpr int Q4 = DPAD / 4;     // head dims per lane in the S / dP products
  static constexpr int NCB = DPAD / kB;   // 16-dim output blocks
  static constexpr int LDK = DPAD + 4;    // K / V, then Q / dO row stride (≡ 4 mod 32)
  static constexpr int fwd_lds = (int)sizeof(float) * 2 * TR * LDK;
  static constexpr int bwd_region = 2 * TR * LDK;
  static constexpr int bwd_lds = (int)sizeof(float) * (bwd_region + 2 * TR);
};

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// Rows of sequence b: [row0, row0 + T) — uniform (b*T, T) or from offsets,
// at most `cap` rows.
__device__ __forceinline__ void seq_rows(const int32_t *offsets, int64_t b, int cap, int &T,
                                         int64_t &row0) {
  if (offsets == nullptr) {
    row0 = b * T;
  } else {
    row0 = offsets[b];
    T = min(offsets[b + 1] - offsets[b], cap);
  }
}

// Rows [0, R) of two head slices (row stride rs) into LDS tiles with row
// stride LD: rows >= T and columns >= dh are zero (padding must be finite:
// a masked score still multiplies a V row).  All loads are issued before
// the first LDS store.  float4 when dh % 4 == 0 (rows 16-byte aligned).
template <int DPAD, int LD, int TR, int NT>
__device__ __forceinline__ void load_pair(float *d0, float *d1, const float *s0, const float *s1,
                                          int64_t rs, int T, int R, int dh) {
  constexpr int C4 = DPAD / 4;
  if ((dh & 3) == 0) {
    constexpr int PER = TR * C4 / NT;
    float4 v0[PER], v1[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = threadIdx.x + q * NT, i = e / C4, c = e % C4;
      const bool ok = i < T && 4 * c < dh;
      v0[q] = ok ? ld4(s0 + (int64_t)i * rs + 4 * c) : f4_zero();
      v1[q] = ok ? ld4(s1 + (int64_t)i * rs + 4 * c) : f4_zero();
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = threadIdx.x + q * NT, i = e / C4, c = e % C4;
      if (i < R) {
        st4(d0 + i * LD + 4 * c, v0[q]);
        st4(d1 + i * LD + 4 * c, v1[q]);
      }
    }
  } else {
    constexpr int PS = TR * DPAD / NT;
    float v0[PS], v1[PS];
#pragma unroll
    for (int q = 0; q < PS; ++q) {
      const int e = threadIdx.x + q * NT, i = e / DPAD, c = e % DPAD;
      const bool ok = i < T && c < dh;
      v0[q] = ok ? s0[(int64_t)i * rs + c] : 0.f;
      v1[q] = ok ? s1[(int64_t)i * rs + c] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < PS; ++q) {
      const int e = threadIdx.x + q * NT, i = e / DPAD, c = e % DPAD;
      if (i < R) {
        d0[i * LD + c] = v0[q];
        d1[i * LD + c] = v1[q];
      }
    }
  }
}

// A lane's Q4 head dims of one row in the S / dP contraction order: lane
// group g holds dims 4t + g (t < Q4), zero if !valid or past dh.  With the
// K / V row stride ≡ 4 (mod 32) the matching LDS reads (row j, dim 4t + g)
// hit 64 distinct banks.
template <int Q4>
__device__ __forceinline__ void load_seg(const float *row, int g, int dh, bool valid,
                                         float (&v)[Q4]) {
#pragma unroll
  for (int t = 0; t < Q4; ++t) v[t] = (valid && 4 * t + g < dh) ? row[4 * t + g] : 0.f;
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
// P[query 16w + j][key 16kb + 4g + r] (j = lane & 15, g = lane >> 4), and the
// query's lse2 = log2 Σ_k exp2(s_k · scale · log2 e) (base-2 log-sum-exp).
template <int DPAD, int NB>
__device__ __forceinline__ void scores_softmax(const float *sK, const float (&q)[DPAD / 4], int w,
                                               int T, float scale, f32x4 (&s)[NB],
                                               float &lse2_out) {
  using S = AttnShape<DPAD, NB>;
  const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
#pragma unroll
  for (int kb = 0; kb < NB; ++kb) s[kb] = zero4();
#pragma unroll
  for (int t = 0; t < S::Q4; ++t) {
#pragma unroll
    for (int kb = 0; kb < NB; ++kb)
      if (kb <= w) s[kb] = mfma16(sK[(kB * kb + j) * S::LDK + 4 * t + g], q[t], s[kb]);
  }
  const int qi = kB * w + j;
  const float c2 = scale * kLog2e;
  float m = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < NB; ++kb) {
    if (kb > w) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = kB * kb + 4 * g + r;
      const float v = (key > qi || key >= T) ? -INFINITY : s[kb][r] * c2;
      s[kb][r] = v;
      m = fmaxf(m, v);
    }
  }
  m = fmaxf(m, __shfl_xor(m, 16));
  m = fmaxf(m, __shfl_xor(m, 32));
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < NB; ++kb) {
    if (kb > w) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = exp2_hw(s[kb][r] - m);
      s[kb][r] = e;
      sum += e;
    }
  }
  sum += __shfl_xor(sum, 16);
  sum += __shfl_xor(sum, 32);
  const float inv = 1.f / sum;
#pragma unroll
  for (int kb = 0; kb < NB; ++kb) {
    if (kb > w) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) s[kb][r] *= inv;
  }
  lse2_out = m + log2_hw(sum);
}

// Sequence seq0 + blockIdx.x / H (or order[seq0 + blockIdx.x / H]), head
// blockIdx.x % H.
template <int DPAD, int NB>
__global__ __launch_bounds__(64 * NB) void attn_fwd_kernel(const float *__restrict__ qkv,
                                                           float *__restrict__ out, int T, int H,
                                                           int dh, float scale,
                                                           const int32_t *__restrict__ offsets,
                                                           int64_t seq0,
                                                           const int32_t *__restrict__ order) {
  using S = AttnShape<DPAD, NB>;
  __shared__ __attribute__((aligned(16))) float sK[S::TR * S::LDK];
  __shared__ __attribute__((aligned(16))) float sV[S::TR * S::LDK];
  // the wave index, wave-uniform in an SGPR (the compiler cannot prove
  // threadIdx.x >> 6 uniform): every block loop and bound derived from it
  // becomes a scalar branch instead of an exec-masked one
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = lane & 15, g = lane >> 4;
  const int64_t b = order ? (int64_t)order[seq0 + blockIdx.x / H] : seq0 + blockIdx.x / H;
  const int h = blockIdx.x % H;
  const int d = H * dh;
  const int64_t rs = 3 * (int64_t)d;
  int64_t row0;
  seq_rows(offsets, b, S::TR, T, row0);
  const int nb = (T + kB - 1) / kB;
  const float *base = qkv + row0 * rs + h * dh;
  load_pair<DPAD, S::LDK, S::TR, S::NT>(sK, sV, base + d, base + 2 * d, rs, T, kB * nb, dh);
  const int qi = kB * w + j;
  float q[S::Q4];
  load_seg<S::Q4>(base + (int64_t)qi * rs, g, dh, w < nb && qi < T, q);
  __syncthreads();
  if (w >= nb) return;  // no barrier below
  f32x4 p[NB];
  float lse2_;
  scores_softmax<DPAD, NB>(sK, q, w, T, scale, p, lse2_);
  f32x4 o[S::NCB];
#pragma unroll
  for (int cb = 0; cb < S::NCB; ++cb) o[cb] = zero4();
#pragma unroll
  for (int kb = 0; kb < NB; ++kb) {
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

// waves_per_eu(4): at most 128 registers, so four workgroups (the LDS
// limit) fit per CU
template <int DPAD, int NB>
__global__ __launch_bounds__(64 * NB) __attribute__((amdgpu_waves_per_eu(4))) void attn_bwd_kernel(const float *__restrict__ qkv,
                                                           const float *__restrict__ dout,
                                                           float *__restrict__ dqkv, int T, int H,
                                                           int dh, float scale,
                                                           const int32_t *__restrict__ offsets,
                                                           int64_t seq0,
                                                           const int32_t *__restrict__ order) {
  using S = AttnShape<DPAD, NB>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float *sK = smem, *sV = smem + S::TR * S::LDK;   // phase A
  float *sQ = smem, *sDO = smem + S::TR * S::LDK;  // phase B (same region)
  float *sM = smem + S::bwd_region, *sD = sM + S::TR;  // per query: lse2, δ
  // the wave index, wave-uniform in an SGPR (the compiler cannot prove
  // threadIdx.x >> 6 uniform): every block loop and bound derived from it
  // becomes a scalar branch instead of an exec-masked one
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = lane & 15, g = lane >> 4;
  const int64_t b = order ? (int64_t)order[seq0 + blockIdx.x / H] : seq0 + blockIdx.x / H;
  const int h = blockIdx.x % H;
  const int d = H * dh;
  const int64_t rs = 3 * (int64_t)d;
  int64_t row0;
  seq_rows(offsets, b, S::TR, T, row0);
  const int nb = (T + kB - 1) / kB;
  const float *base = qkv + row0 * rs + h * dh;
  float *gbase = dqkv + row0 * rs + h * dh;
  load_pair<DPAD, S::LDK, S::TR, S::NT>(sK, sV, base + d, base + 2 * d, rs, T, kB * nb, dh);
  const int qi = kB * w + j;
  const bool qvalid = w < nb && qi < T;
  float q[S::Q4], dov[S::Q4];
  load_seg<S::Q4>(base + (int64_t)qi * rs, g, dh, qvalid, q);
  load_seg<S::Q4>(dout + (row0 + qi) * d + h * dh, g, dh, qvalid, dov);
  __syncthreads();
  // ---------------------------------------------------- phase A: query block w
  float kr[S::Q4], vr[S::Q4];  // K / V rows 16w + j, dims 4t + g (phase B operands)
  if (w < nb) {
    f32x4 p[NB], dp[NB];
    float lse2;
    scores_softmax<DPAD, NB>(sK, q, w, T, scale, p, lse2);
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) dp[kb] = zero4();
#pragma unroll
    for (int t = 0; t < S::Q4; ++t) {
#pragma unroll
      for (int kb = 0; kb < NB; ++kb)
        if (kb <= w) dp[kb] = mfma16(sV[(kB * kb + j) * S::LDK + 4 * t + g], dov[t], dp[kb]);
    }
    float delta = 0.f;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb > w) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) delta += p[kb][r] * dp[kb][r];
    }
    delta += __shfl_xor(delta, 16);
    delta += __shfl_xor(delta, 32);
    if (g == 0) {
      sM[qi] = lse2;
      sD[qi] = delta;
    }
    // dSᵀ (in dp), then dQᵀ = Kᵀ dSᵀ
    f32x4 dq[S::NCB];
#pragma unroll
    for (int cb = 0; cb < S::NCB; ++cb) dq[cb] = zero4();
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb > w) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dp[kb][r] = p[kb][r] * (dp[kb][r] - delta) * scale;
        const float *krow = sK + (kB * kb + 4 * g + r) * S::LDK + j;
#pragma unroll
        for (int cb = 0; cb < S::NCB; ++cb) dq[cb] = mfma16(krow[kB * cb], dp[kb][r], dq[cb]);
      }
    }
    if (qi < T) {
      float *row = gbase + (int64_t)qi * rs;
#pragma unroll
      for (int cb = 0; cb < S::NCB; ++cb) store4(row, kB * cb + 4 * g, dh, dq[cb]);
    }
#pragma unroll
    for (int t = 0; t < S::Q4; ++t) {
      kr[t] = sK[qi * S::LDK + 4 * t + g];
      vr[t] = sV[qi * S::LDK + 4 * t + g];
    }
  }
  __syncthreads();  // K / V no longer read from LDS; statistics complete
  if (w < nb) {
#pragma unroll
    for (int t = 0; t < S::Q4; ++t) {
      sQ[qi * S::LDK + 4 * t + g] = q[t];
      sDO[qi * S::LDK + 4 * t + g] = dov[t];
    }
  }
  __syncthreads();
  // ------------------------------------------------------ phase B: key block w
  if (w < nb) {
    const int key = kB * w + j;
    f32x4 dv[S::NCB], dk[S::NCB];
#pragma unroll
    for (int cb = 0; cb < S::NCB; ++cb) {
      dv[cb] = zero4();
      dk[cb] = zero4();
    }
    const float c2 = scale * kLog2e;
    for (int qb = w; qb < nb; ++qb) {
      // S[query 16qb + 4g + r][key 16w + j] and dP likewise; the four
      // queries' statistics as one float4 each
      const float4 l4 = ld4(sM + kB * qb + 4 * g), d4 = ld4(sD + kB * qb + 4 * g);
      const float lq[4] = {l4.x, l4.y, l4.z, l4.w}, dq4[4] = {d4.x, d4.y, d4.z, d4.w};
      f32x4 sc = zero4(), dpc = zero4();
      const float *qrow = sQ + (kB * qb + j) * S::LDK + g;
      const float *orow = sDO + (kB * qb + j) * S::LDK + g;
#pragma unroll
      for (int t = 0; t < S::Q4; ++t) {
        sc = mfma16(qrow[4 * t], kr[t], sc);
        dpc = mfma16(orow[4 * t], vr[t], dpc);
      }
      float pr[4], dsr[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = kB * qb + 4 * g + r;
        const bool ok = key <= qq && qq < T;
        const float pv = ok ? exp2_hw(fmaf(sc[r], c2, -lq[r])) : 0.f;
        pr[r] = pv;
        dsr[r] = pv * (dpc[r] - dq4[r]) * scale;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = kB * qb + 4 * g + r;
        const float *dorow = sDO + qq * S::LDK + j;
        const float *qr = sQ + qq * S::LDK + j;
#pragma unroll
        for (int cb = 0; cb < S::NCB; ++cb) {
          dv[cb] = mfma16(dorow[kB * cb], pr[r], dv[cb]);
          dk[cb] = mfma16(qr[kB * cb], dsr[r], dk[cb]);
        }
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

// ------------------------------------------------------------ packed backward
// The backward above with several short sequences in one workgroup: the
// sequences come in packs (mirec_attention_length_order: longest first,
// one pack = one sequence of 3-4 blocks, two of 2 blocks or four of 1
// block), so no wave idles on a short sequence and a 4-block workgroup's
// LDS serves up to four sequences.  Pack p, head h = workgroup p*H + h;
// wave w is block w of the pack's block list: sequence i = slot(w), local
// block w - lo (lo = the sequence's first block in the pack).  LDS row R
// holds local row 16 (R/16 - lo) + R%16 of its block's sequence.
// κ layout helpers of the packed backward: lane group g of a 16-row block
// holds dims 16 c + 4 g + e (e < 4) of its row at contraction step 4 c + e;
// dims >= dh (dh % 4 == 0) read as zero.
template <int Q4>
__device__ __forceinline__ void ld_kappa_dh(const float *row, int g, int dh, bool ok,
                                            float (&v)[Q4]) {
#pragma unroll
  for (int c = 0; c < Q4 / 4; ++c) {
    // unconditional load of a clamped dim, zero selected after (no
    // exec-masked branch around the load)
    const int dim = 16 * c + 4 * g;
    float4 x = ld4(row + min(dim, dh - 4));
    if (!(ok && dim < dh)) x = f4_zero();
    v[4 * c] = x.x;
    v[4 * c + 1] = x.y;
    v[4 * c + 2] = x.z;
    v[4 * c + 3] = x.w;
  }
}

// scores_softmax with the key operand read from LDS in the κ order (float4):
// key blocks 0..w of sK (the sequence's first block at sK), query row 16 w + j.
template <int DPAD, int NB>
__device__ __forceinline__ void scores_softmax_kappa(const float *sK, const float (&q)[DPAD / 4],
                                                     int w, int T, float scale, f32x4 (&s)[NB],
                                                     float &lse2_out) {
  using S = AttnShape<DPAD, NB>;
  const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
#pragma unroll
  for (int kb = 0; kb < NB; ++kb) s[kb] = zero4();
#pragma unroll
  for (int c = 0; c < S::Q4 / 4; ++c) {
#pragma unroll
    for (int kb = 0; kb < NB; ++kb)
      if (kb <= w) {
        const float4 k4 = ld4(sK + (kB * kb + j) * S::LDK + 16 * c + 4 * g);
        s[kb] = mfma16(k4.x, q[4 * c], s[kb]);
        s[kb] = mfma16(k4.y, q[4 * c + 1], s[kb]);
        s[kb] = mfma16(k4.z, q[4 * c + 2], s[kb]);
        s[kb] = mfma16(k4.w, q[4 * c + 3], s[kb]);
      }
  }
  const int qi = kB * w + j;
  const float c2 = scale * kLog2e;
  float m = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < NB; ++kb) {
    if (kb > w) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = kB * kb + 4 * g + r;
      const float v = (key > qi || key >= T) ? -INFINITY : s[kb][r] * c2;
      s[kb][r] = v;
      m = fmaxf(m, v);
    }
  }
  m = fmaxf(m, __shfl_xor(m, 16));
  m = fmaxf(m, __shfl_xor(m, 32));
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < NB; ++kb) {
    if (kb > w) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = exp2_hw(s[kb][r] - m);
      s[kb][r] = e;
      sum += e;
    }
  }
  sum += __shfl_xor(sum, 16);
  sum += __shfl_xor(sum, 32);
  const float inv = 1.f / sum;
#pragma unroll
  for (int kb = 0; kb < NB; ++kb) {
    if (kb > w) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) s[kb][r] *= inv;
  }
  lse2_out = m + log2_hw(sum);
}

struct PackSeqs {
  int64_t row0[4];
  int T[4], lo[4], n;  // n = the pack's block count
};

// The pack's descriptor: (first row, length) of its four slots, written by
// the ordering pass (mirec_attention_length_order) — two 16-byte loads, no
// dependent load of the offsets.
__device__ __forceinline__ void read_pack(const int32_t *packs, int64_t pk, PackSeqs &ps) {
  const int4 *d = reinterpret_cast<const int4 *>(packs + 4 + 8 * pk);
  const int4 a = d[0], b = d[1];
  const int r0[4] = {a.x, a.z, b.x, b.z}, len[4] = {a.y, a.w, b.y, b.w};
  int nb = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int T = min(len[i], kT);
    ps.row0[i] = r0[i];
    ps.T[i] = T;
    ps.lo[i] = nb;
    nb += (T + kB - 1) / kB;
  }
  ps.n = nb;
}

// (T, first block, first row) of the sequence holding block w (w < ps.n),
// by selects (no dynamic register indexing).
__device__ __forceinline__ void seq_of(const PackSeqs &ps, int w, int &T, int &lo,
                                       int64_t &row0) {
  T = ps.T[0];
  lo = ps.lo[0];
  row0 = ps.row0[0];
#pragma unroll
  for (int k = 1; k < 4; ++k)
    if (w >= ps.lo[k] && ps.T[k] > 0) {
      T = ps.T[k];
      lo = ps.lo[k];
      row0 = ps.row0[k];
    }
}

// K / V rows of every block of the pack (rows past a sequence's length and
// dims past dh zero): load_pack_regs issues the loads into registers,
// store_pack puts them into LDS — the caller issues its own row loads in
// between, so all of a workgroup's global loads share one round trip.
template <int DPAD>
struct PackRegs {
  static constexpr int PER = 4 * kB * (DPAD / 4) / 256;
  float4 v0[PER], v1[PER];
};

template <int DPAD>
__device__ __forceinline__ void load_pack_regs(PackRegs<DPAD> &pr, const float *qkv, int64_t rs,
                                               int coff, const PackSeqs &ps, int dh) {
  constexpr int C4 = DPAD / 4, PER = PackRegs<DPAD>::PER;
  float4 *v0 = pr.v0, *v1 = pr.v1;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    // thread t covers row R = t / C4 + q·(256 / C4) (16-row block w, row
    // R % 16 in it), dims 4c..; the block is the same for a whole wave
    // (DPAD 64: w = q; DPAD 32: t / 128 + 2q), so the sequence lookup runs
    // on scalars
    const int c = threadIdx.x % C4, rr = (threadIdx.x / C4) % kB;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / C4) / kB) +
                  q * (256 / C4 / kB);
    // unconditional loads: a row past its sequence's length loads the
    // sequence's last row (its score is masked to -inf, its P and dS are 0),
    // a block past the pack's blocks loads a row of the pack (never read);
    // only dims past dh must be zero (they would enter the contractions)
    int T, lo;
    int64_t r0;
    seq_of(ps, w, T, lo, r0);
    const int64_t row = r0 + min(kB * (w - lo) + rr, T - 1);
    const float *src = qkv + row * rs + coff + 4 * min(c, dh / 4 - 1);
    v0[q] = ld4(src);
    v1[q] = ld4(src + rs / 3);
  }
  if (dh < DPAD) {  // (wave-uniform) dims past dh read as zero
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const bool dim_ok = 4 * (int)(threadIdx.x % C4) < dh;
      v0[q] = dim_ok ? v0[q] : f4_zero();
      v1[q] = dim_ok ? v1[q] : f4_zero();
    }
  }
}

template <int DPAD, int LD>
__device__ __forceinline__ void store_pack(float *d0, float *d1, const PackRegs<DPAD> &pr) {
  constexpr int C4 = DPAD / 4, PER = PackRegs<DPAD>::PER;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int e = threadIdx.x + q * 256, R = e / C4, c = e % C4;
    st4(d0 + R * LD + 4 * c, pr.v0[q]);
    st4(d1 + R * LD + 4 * c, pr.v1[q]);
  }
}

// waves_per_eu(4): at most 128 registers, so four workgroups (the LDS
// limit) fit per CU.  dh % 4 == 0.
// FWD_STATS: the forward's lse2 [n_rows, H] (the wave forward's base-2
// log-sum-exp) is given, so phase A's P = exp2(S·c2 − lse2) directly: no
// max and sum reductions, no normalisation pass; δ = Σ_k P dP as before.
// (δ = rowsum(dO ⊙ O), FlashAttention-2's form, was measured slower here:
// it reads O, 29 MB more per C4 launch, for VALU this kernel is not bound by.)
template <int DPAD, bool FWD_STATS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void attn_bwd_packed_kernel(
    const float *__restrict__ qkv, const float *__restrict__ dout, float *__restrict__ dqkv,
    int H, int dh, float scale, const int32_t *__restrict__ offsets,
    const int32_t *__restrict__ packs, int64_t batch, int64_t n_rows,
    const float *__restrict__ fwd_lse2) {
  constexpr int NB = 4;
  using S = AttnShape<DPAD, NB>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float *sK = smem, *sV = smem + S::TR * S::LDK;   // phase A
  float *sQ = smem, *sDO = smem + S::TR * S::LDK;  // phase B (same region)
  float *sM = smem + S::bwd_region, *sD = sM + S::TR;  // per query: lse2, δ
  const int64_t pk = blockIdx.x / H;
  const int64_t busy = (int64_t)packs[0] * H;
  if ((int64_t)blockIdx.x >= busy) {
    // a spare workgroup: zero its share of the capacity padding rows
    const int64_t w4 = 3 * (int64_t)H * dh / 4;
    const int64_t e0 = (int64_t)offsets[batch] * w4, e1 = n_rows * w4;
    const int64_t stride = ((int64_t)gridDim.x - busy) * 256;
    for (int64_t e = e0 + ((int64_t)blockIdx.x - busy) * 256 + threadIdx.x; e < e1; e += stride)
      st4(dqkv + 4 * e, f4_zero());
    return;
  }
  const int h = blockIdx.x % H;
  // the wave index, wave-uniform in an SGPR (the compiler cannot prove
  // threadIdx.x >> 6 uniform): every block loop and bound derived from it
  // becomes a scalar branch instead of an exec-masked one
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = lane & 15, g = lane >> 4;
  const int d = H * dh;
  const int64_t rs = 3 * (int64_t)d;
  PackSeqs ps;
  read_pack(packs, pk, ps);
  PackRegs<DPAD> kv;
  load_pack_regs<DPAD>(kv, qkv, rs, d + h * dh, ps, dh);
  // this wave's sequence
  const bool act = w < ps.n;
  int T = 0, lo = 0;
  int64_t row0 = 0;
  if (act) seq_of(ps, w, T, lo, row0);
  lo &= 3;                                           // (0 <= lo <= w)
  const int hi = act ? lo + (T + kB - 1) / kB : 0;  // one past the sequence's last block
  const float *base = qkv + row0 * rs + h * dh;
  float *gbase = dqkv + row0 * rs + h * dh;
  const int ql = kB * (w - lo) + j;  // local query row of phase A
  const int qa = kB * w + j;         // its LDS row
  // q / dO rows in the κ layout: lane group g holds dims 16 c + 4 g + e
  // (float4 loads; the LDS operands are read the same way, as float4 —
  // conflict-free at the row stride ≡ 4 mod 32)
  // (a query row past T loads the sequence's last row: its dQ is not
  // stored, its P is 0 in phase B; an idle wave loads row 0, never used)
  float q[S::Q4], dov[S::Q4];
  const int qlc = act ? min(ql, T - 1) : 0;
  ld_kappa_dh<S::Q4>(base + (int64_t)qlc * rs, g, dh, true, q);
  ld_kappa_dh<S::Q4>(dout + (row0 + qlc) * d + h * dh, g, dh, true, dov);
  float lq = 0.f;
  if constexpr (FWD_STATS) lq = fwd_lse2[(row0 + qlc) * H + h];
  store_pack<DPAD, S::LDK>(sK, sV, kv);  // (waits for the K / V loads only)
  __syncthreads();
  // ---------------------------------------------------- phase A: query block w
  float kr[S::Q4], vr[S::Q4];
  if (FWD_STATS && act) {
    // P from the forward's lse2 (no max / sum passes); δ = Σ_k P dP
    const int lw = (w - lo) & 3;
    const float *sKl = sK + kB * lo * S::LDK, *sVl = sV + kB * lo * S::LDK;
    const float c2 = scale * kLog2e, nl = -lq;
    f32x4 p[NB], dp[NB];
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      p[kb] = zero4();
      dp[kb] = zero4();
    }
#pragma unroll
    for (int c = 0; c < S::Q4 / 4; ++c) {
#pragma unroll
      for (int kb = 0; kb < NB; ++kb)
        if (kb <= lw) {
          const float4 k4 = ld4(sKl + (kB * kb + j) * S::LDK + 16 * c + 4 * g);
          const float4 v4 = ld4(sVl + (kB * kb + j) * S::LDK + 16 * c + 4 * g);
          p[kb] = mfma16(k4.x, q[4 * c], p[kb]);
          dp[kb] = mfma16(v4.x, dov[4 * c], dp[kb]);
          p[kb] = mfma16(k4.y, q[4 * c + 1], p[kb]);
          dp[kb] = mfma16(v4.y, dov[4 * c + 1], dp[kb]);
          p[kb] = mfma16(k4.z, q[4 * c + 2], p[kb]);
          dp[kb] = mfma16(v4.z, dov[4 * c + 2], dp[kb]);
          p[kb] = mfma16(k4.w, q[4 * c + 3], p[kb]);
          dp[kb] = mfma16(v4.w, dov[4 * c + 3], dp[kb]);
        }
    }
    float delta = 0.f;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb > lw) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kB * kb + 4 * g + r;
        const float pv = (key <= ql && key < T) ? exp2_hw(fmaf(p[kb][r], c2, nl)) : 0.f;
        p[kb][r] = pv;
        delta = fmaf(pv, dp[kb][r], delta);
      }
    }
    delta += __shfl_xor(delta, 16);
    delta += __shfl_xor(delta, 32);
    if (g == 0) {
      sM[qa] = lq;
      sD[qa] = delta;
    }
    f32x4 dq[S::NCB];
#pragma unroll
    for (int cb = 0; cb < S::NCB; ++cb) dq[cb] = zero4();
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb > lw) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ds = p[kb][r] * (dp[kb][r] - delta) * scale;
        const float *krow = sKl + (kB * kb + 4 * g + r) * S::LDK + j;
#pragma unroll
        for (int cb = 0; cb < S::NCB; ++cb) dq[cb] = mfma16(krow[kB * cb], ds, dq[cb]);
      }
    }
    if (ql < T) {
      float *row = gbase + (int64_t)ql * rs;
#pragma unroll
      for (int cb = 0; cb < S::NCB; ++cb) store4(row, kB * cb + 4 * g, dh, dq[cb]);
    }
#pragma unroll
    for (int c = 0; c < S::Q4 / 4; ++c) {
      const float4 k4 = ld4(sK + qa * S::LDK + 16 * c + 4 * g);
      const float4 v4 = ld4(sV + qa * S::LDK + 16 * c + 4 * g);
      kr[4 * c] = k4.x;
      kr[4 * c + 1] = k4.y;
      kr[4 * c + 2] = k4.z;
      kr[4 * c + 3] = k4.w;
      vr[4 * c] = v4.x;
      vr[4 * c + 1] = v4.y;
      vr[4 * c + 2] = v4.z;
      vr[4 * c + 3] = v4.w;
    }
  } else if (!FWD_STATS && act) {
    f32x4 p[NB], dp[NB];
    float lse2;
    // local key blocks kb = 0..lw (LDS block lo + kb); the masks tell the
    // compiler lw, lo < 4 (as the plain kernel's w), which keeps the
    // unrolled block loops from holding every block's operands at once
    const int lw = (w - lo) & 3;
    const float *sKl = sK + kB * lo * S::LDK, *sVl = sV + kB * lo * S::LDK;  // lo < 4
    scores_softmax_kappa<DPAD, NB>(sKl, q, lw, T, scale, p, lse2);
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) dp[kb] = zero4();
#pragma unroll
    for (int c = 0; c < S::Q4 / 4; ++c) {
#pragma unroll
      for (int kb = 0; kb < NB; ++kb)
        if (kb <= lw) {
          const float4 v4 = ld4(sVl + (kB * kb + j) * S::LDK + 16 * c + 4 * g);
          dp[kb] = mfma16(v4.x, dov[4 * c], dp[kb]);
          dp[kb] = mfma16(v4.y, dov[4 * c + 1], dp[kb]);
          dp[kb] = mfma16(v4.z, dov[4 * c + 2], dp[kb]);
          dp[kb] = mfma16(v4.w, dov[4 * c + 3], dp[kb]);
        }
    }
    float delta = 0.f;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb > lw) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) delta += p[kb][r] * dp[kb][r];
    }
    delta += __shfl_xor(delta, 16);
    delta += __shfl_xor(delta, 32);
    if (g == 0) {
      sM[qa] = lse2;
      sD[qa] = delta;
    }
    f32x4 dq[S::NCB];
#pragma unroll
    for (int cb = 0; cb < S::NCB; ++cb) dq[cb] = zero4();
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      if (kb > lw) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dp[kb][r] = p[kb][r] * (dp[kb][r] - delta) * scale;
        const float *krow = sKl + (kB * kb + 4 * g + r) * S::LDK + j;
#pragma unroll
        for (int cb = 0; cb < S::NCB; ++cb) dq[cb] = mfma16(krow[kB * cb], dp[kb][r], dq[cb]);
      }
    }
    if (ql < T) {
      float *row = gbase + (int64_t)ql * rs;
#pragma unroll
      for (int cb = 0; cb < S::NCB; ++cb) store4(row, kB * cb + 4 * g, dh, dq[cb]);
    }
#pragma unroll
    for (int c = 0; c < S::Q4 / 4; ++c) {
      const float4 k4 = ld4(sK + qa * S::LDK + 16 * c + 4 * g);
      const float4 v4 = ld4(sV + qa * S::LDK + 16 * c + 4 * g);
      kr[4 * c] = k4.x;
      kr[4 * c + 1] = k4.y;
      kr[4 * c + 2] = k4.z;
      kr[4 * c + 3] = k4.w;
      vr[4 * c] = v4.x;
      vr[4 * c + 1] = v4.y;
      vr[4 * c + 2] = v4.z;
      vr[4 * c + 3] = v4.w;
    }
  }
  __syncthreads();  // K / V no longer read from LDS; statistics complete
  if (act) {
#pragma unroll
    for (int c = 0; c < S::Q4 / 4; ++c) {
      st4(sQ + qa * S::LDK + 16 * c + 4 * g,
          make_float4(q[4 * c], q[4 * c + 1], q[4 * c + 2], q[4 * c + 3]));
      st4(sDO + qa * S::LDK + 16 * c + 4 * g,
          make_float4(dov[4 * c], dov[4 * c + 1], dov[4 * c + 2], dov[4 * c + 3]));
    }
  }
  __syncthreads();
  // ------------------------------------------------------ phase B: key block w
  if (act) {
    const int key = kB * (w - lo) + j;  // local
    f32x4 dv[S::NCB], dk[S::NCB];
#pragma unroll
    for (int cb = 0; cb < S::NCB; ++cb) {
      dv[cb] = zero4();
      dk[cb] = zero4();
    }
    // local query blocks lw..nbs-1 of the sequence (LDS block lo + qb)
    const int lw = (w - lo) & 3, nbs = hi - lo, o = kB * (lo & 3);
    const float *sQl = sQ + o * S::LDK, *sDOl = sDO + o * S::LDK;
    const float *sMl = sM + o, *sDl = sD + o;
    const float c2 = scale * kLog2e;
    for (int qb = lw; qb < nbs; ++qb) {
      float pr[4], dsr[4];
      // the four queries' statistics of this lane group: one float4 each
      const float4 l4 = ld4(sMl + kB * qb + 4 * g), d4 = ld4(sDl + kB * qb + 4 * g);
      const float lq[4] = {l4.x, l4.y, l4.z, l4.w}, dq4[4] = {d4.x, d4.y, d4.z, d4.w};
      f32x4 sc = zero4(), dpc = zero4();
      const float *qrow = sQl + (kB * qb + j) * S::LDK + 4 * g;
      const float *orow = sDOl + (kB * qb + j) * S::LDK + 4 * g;
#pragma unroll
      for (int c = 0; c < S::Q4 / 4; ++c) {
        const float4 q4 = ld4(qrow + 16 * c), o4 = ld4(orow + 16 * c);
        sc = mfma16(q4.x, kr[4 * c], sc);
        dpc = mfma16(o4.x, vr[4 * c], dpc);
        sc = mfma16(q4.y, kr[4 * c + 1], sc);
        dpc = mfma16(o4.y, vr[4 * c + 1], dpc);
        sc = mfma16(q4.z, kr[4 * c + 2], sc);
        dpc = mfma16(o4.z, vr[4 * c + 2], dpc);
        sc = mfma16(q4.w, kr[4 * c + 3], sc);
        dpc = mfma16(o4.w, vr[4 * c + 3], dpc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = kB * qb + 4 * g + r;  // local query = its local LDS row
        const bool ok = key <= qq && qq < T;
        const float pv = ok ? exp2_hw(fmaf(sc[r], c2, -lq[r])) : 0.f;
        pr[r] = pv;
        dsr[r] = pv * (dpc[r] - dq4[r]) * scale;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = kB * qb + 4 * g + r;
        const float *dorow = sDOl + qq * S::LDK + j;
        const float *qrr = sQl + qq * S::LDK + j;
#pragma unroll
        for (int cb = 0; cb < S::NCB; ++cb) {
          dv[cb] = mfma16(dorow[kB * cb], pr[r], dv[cb]);
          dk[cb] = mfma16(qrr[kB * cb], dsr[r], dk[cb]);
        }
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

template <int DPAD, bool FWD_STATS>
static int launch_packed_bwd(const float *qkv, const float *dout, const int32_t *offsets,
                             const int32_t *packs, int64_t batch, int heads, int dh, float *dqkv,
                             int64_t n_rows, const float *fwd_lse2, hipStream_t st) {
  constexpr int lds = AttnShape<DPAD, 4>::bwd_lds;
  static int rc = -1;
  if (rc < 0)
    rc = hipFuncSetAttribute((const void *)attn_bwd_packed_kernel<DPAD, FWD_STATS>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess ? 0 : 1;
  if (rc != 0) return MIREC_ERR_HIP;
  // at most batch packs per head, plus spare workgroups for the padding rows
  hipLaunchKernelGGL((attn_bwd_packed_kernel<DPAD, FWD_STATS>),
                     dim3((unsigned)(batch * heads + 256)), dim3(256), lds, st, qkv, dout, dqkv,
                     heads, dh, 1.f / sqrtf((float)dh), offsets, packs, batch, n_rows, fwd_lse2);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

// Dynamic LDS above 64 KiB needs an explicit opt-in per kernel (once).
template <int DPAD, int NB>
static int allow_lds() {
  static int rc = -1;
  if (rc < 0)
    rc = hipFuncSetAttribute((const void *)attn_bwd_kernel<DPAD, NB>,
                             hipFuncAttributeMaxDynamicSharedMemorySize,
                             AttnShape<DPAD, NB>::bwd_lds) == hipSuccess ? 0 : 1;
  return rc;
}

// One launch over sequences [seq0, seq0 + n) of the bucket NB.
template <int DPAD, int NB>
static int launch_bucket(bool bwd, const float *qkv, const float *dout, const int32_t *offsets,
                         int64_t seq0, int64_t n, int T, int heads, int dh, float *outp,
                         hipStream_t st, const int32_t *order) {
  if (n <= 0) return MIREC_OK;
  const float scale = 1.f / sqrtf((float)dh);
  const dim3 grid((unsigned)(n * heads)), block(64 * NB);
  if (!bwd) {
    hipLaunchKernelGGL((attn_fwd_kernel<DPAD, NB>), grid, block, 0, st, qkv, outp, T, heads, dh,
                       scale, offsets, seq0, order);
  } else {
    if (allow_lds<DPAD, NB>() != 0) return MIREC_ERR_HIP;
    constexpr int lds = AttnShape<DPAD, NB>::bwd_lds;
    hipLaunchKernelGGL((attn_bwd_kernel<DPAD, NB>), grid, block, lds, st, qkv, dout, outp, T,
                       heads, dh, scale, offsets, seq0, order);
  }
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

template <int DPAD>
static int launch_nb(int nb, bool bwd, const float *qkv, const float *dout,
                     const int32_t *offsets, int64_t seq0, int64_t n, int T, int heads, int dh,
                     float *outp, hipStream_t st, const int32_t *order) {
  switch (nb) {
    case 1: return launch_bucket<DPAD, 1>(bwd, qkv, dout, offsets, seq0, n, T, heads, dh, outp, st, order);
    case 2: return launch_bucket<DPAD, 2>(bwd, qkv, dout, offsets, seq0, n, T, heads, dh, outp, st, order);
    case 3: return launch_bucket<DPAD, 3>(bwd, qkv, dout, offsets, seq0, n, T, heads, dh, outp, st, order);
    default: return launch_bucket<DPAD, 4>(bwd, qkv, dout, offsets, seq0, n, T, heads, dh, outp, st, order);
  }
}

// bucket_end[k] (k < 4): sequences [bucket_end[k-1], bucket_end[k]) run on
// the NB = k+1 kernel.  Uniform batches pass T and one bucket.
static int launch(bool bwd, const float *qkv, const float *dout, const int32_t *offsets,
                  const int64_t *bucket_end, int T, int heads, int dh, float *outp,
                  hipStream_t st, const int32_t *order = nullptr) {
  int64_t prev = 0;
  for (int k = 0; k < 4; ++k) {
    const int64_t end = bucket_end[k];
    const int rc = dh <= 32 ? launch_nb<32>(k + 1, bwd, qkv, dout, offsets, prev, end - prev, T,
                                            heads, dh, outp, st, order)
                            : launch_nb<64>(k + 1, bwd, qkv, dout, offsets, prev, end - prev, T,
                                            heads, dh, outp, st, order);
    if (rc != MIREC_OK) return rc;
    prev = end;
  }
  return MIREC_OK;
}

// Uniform batch: every sequence has T rows -> the NB = ceil(T/16) bucket.
static void uniform_buckets(int64_t batch, int T, int64_t (&be)[4]) {
  const int nb = (T + kB - 1) / kB;
  for (int k = 0; k < 4; ++k) be[k] = (k + 1 >= nb) ? batch : 0;
}

static bool valid_buckets(const int64_t *be) {
  if (be[0] < 0) return false;
  for (int k = 1; k < 4; ++k)
    if (be[k] < be[k - 1]) return false;
  return true;
}

}  // namespace mirec

extern "C" int mirec_attention_fwd(const float *qkv, int64_t batch, int32_t T, int32_t heads,
                                   int32_t head_dim, float *out, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(qkv && out && batch >= 0 && T >= 1 && T <= kT && heads >= 1);
  MIREC_CHECK_ARG(head_dim >= 1 && head_dim <= 64);
  int64_t be[4];
  uniform_buckets(batch, T, be);
  return launch(false, qkv, nullptr, nullptr, be, T, heads, head_dim, out,
                reinterpret_cast<hipStream_t>(stream));
}

extern "C" int mirec_attention_bwd(const float *qkv, const float *dout, int64_t batch, int32_t T,
                                   int32_t heads, int32_t head_dim, float *dqkv,
                                   mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(qkv && dout && dqkv && batch >= 0 && T >= 1 && T <= kT && heads >= 1);
  MIREC_CHECK_ARG(head_dim >= 1 && head_dim <= 64);
  int64_t be[4];
  uniform_buckets(batch, T, be);
  return launch(true, qkv, dout, nullptr, be, T, heads, head_dim, dqkv,
                reinterpret_cast<hipStream_t>(stream));
}

extern "C" int mirec_attention_varlen_fwd(const float *qkv, const int32_t *offsets,
                                          int64_t batch, int32_t heads, int32_t head_dim,
                                          float *out, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(qkv && offsets && out && batch >= 0 && heads >= 1);
  MIREC_CHECK_ARG(head_dim >= 1 && head_dim <= 64);
  const int64_t be[4] = {0, 0, 0, batch};
  return launch(false, qkv, nullptr, offsets, be, kT, heads, head_dim, out,
                reinterpret_cast<hipStream_t>(stream));
}

extern "C" int mirec_attention_varlen_bwd(const float *qkv, const float *dout,
                                          const int32_t *offsets, int64_t batch, int32_t heads,
                                          int32_t head_dim, float *dqkv, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(qkv && dout && offsets && dqkv && batch >= 0 && heads >= 1);
  MIREC_CHECK_ARG(head_dim >= 1 && head_dim <= 64);
  const int64_t be[4] = {0, 0, 0, batch};
  return launch(true, qkv, dout, offsets, be, kT, heads, head_dim, dqkv,
                reinterpret_cast<hipStream_t>(stream));
}

extern "C" int mirec_attention_bucketed_fwd(const float *qkv, const int32_t *offsets,
                                            const int64_t *bucket_end, int32_t heads,
                                            int32_t head_dim, float *out, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(qkv && offsets && bucket_end && out && heads >= 1);
  MIREC_CHECK_ARG(head_dim >= 1 && head_dim <= 64 && valid_buckets(bucket_end));
  return launch(false, qkv, nullptr, offsets, bucket_end, kT, heads, head_dim, out,
                reinterpret_cast<hipStream_t>(stream));
}

extern "C" int mirec_attention_bucketed_bwd(const float *qkv, const float *dout,
                                            const int32_t *offsets, const int64_t *bucket_end,
                                            int32_t heads, int32_t head_dim, float *dqkv,
                                            mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(qkv && dout && offsets && bucket_end && dqkv && heads >= 1);
  MIREC_CHECK_ARG(head_dim >= 1 && head_dim <= 64 && valid_buckets(bucket_end));
  return launch(true, qkv, dout, offsets, bucket_end, kT, heads, head_dim, dqkv,
                reinterpret_cast<hipStream_t>(stream));
}

extern "C" int mirec_attention_ordered_fwd(const float *qkv, const int32_t *offsets,
                                           const int32_t *order, int64_t batch, int32_t heads,
                                           int32_t head_dim, float *out, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(qkv && offsets && order && out && batch >= 0 && heads >= 1);
  MIREC_CHECK_ARG(head_dim >= 1 && head_dim <= 64);
  const int64_t be[4] = {0, 0, 0, batch};
  return launch(false, qkv, nullptr, offsets, be, kT, heads, head_dim, out,
                reinterpret_cast<hipStream_t>(stream), order);
}

extern "C" int mirec_attention_ordered_bwd(const float *qkv, const float *dout,
                                           const int32_t *offsets, const int32_t *order,
                                           int64_t batch, int32_t heads, int32_t head_dim,
                                           float *dqkv, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(qkv && dout && offsets && order && dqkv && batch >= 0 && heads >= 1);
  MIREC_CHECK_ARG(head_dim >= 1 && head_dim <= 64);
  const int64_t be[4] = {0, 0, 0, batch};
  return launch(true, qkv, dout, offsets, be, kT, heads, head_dim, dqkv,
                reinterpret_cast<hipStream_t>(stream), order);
}

extern "C" int mirec_attention_packed_bwd(const float *qkv, const float *dout,
                                          const int32_t *offsets, const int32_t *packs,
                                          int64_t batch, int32_t heads, int32_t head_dim,
                                          float *dqkv, int64_t n_rows, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(batch >= 0 && heads >= 1 && head_dim >= 4 && head_dim <= 64 &&
                  head_dim % 4 == 0 && n_rows >= 0);
  if (batch == 0) return MIREC_OK;
  MIREC_CHECK_ARG(qkv && dout && offsets && packs && dqkv && (uintptr_t)packs % 16 == 0);
  MIREC_CHECK_ARG(((uintptr_t)qkv | (uintptr_t)dout | (uintptr_t)dqkv) % 16 == 0);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  return head_dim <= 32
             ? launch_packed_bwd<32, false>(qkv, dout, offsets, packs, batch, heads, head_dim,
                                            dqkv, n_rows, nullptr, st)
             : launch_packed_bwd<64, false>(qkv, dout, offsets, packs, batch, heads, head_dim,
                                            dqkv, n_rows, nullptr, st);
}

extern "C" int mirec_attention_packed_bwd_lse(const float *qkv, const float *lse,
                                              const float *dout, const int32_t *offsets,
                                              const int32_t *packs, int64_t batch, int32_t heads,
                                              int32_t head_dim, float *dqkv, int64_t n_rows,
                                              mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(batch >= 0 && heads >= 1 && head_dim >= 4 && head_dim <= 64 &&
                  head_dim % 4 == 0 && n_rows >= 0);
  if (batch == 0) return MIREC_OK;
  MIREC_CHECK_ARG(qkv && lse && dout && offsets && packs && dqkv && (uintptr_t)packs % 16 == 0);
  MIREC_CHECK_ARG(((uintptr_t)qkv | (uintptr_t)dout | (uintptr_t)dqkv) % 16 == 0);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  return head_dim <= 32
             ? launch_packed_bwd<32, true>(qkv, dout, offsets, packs, batch, heads, head_dim,
                                           dqkv, n_rows, lse, st)
             : launch_packed_bwd<64, true>(qkv, dout, offsets, packs, batch, heads, head_dim,
                                           dqkv, n_rows, lse, st);
}
