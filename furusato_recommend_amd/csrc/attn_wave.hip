// SASRec causal self-attention core, one WAVE per (sequence, head)
// (model/sasrec.py:385-397: torch.nn.MultiheadAttention with a causal mask,
// sequences of at most 64 positions).  Head dims 16, 32 or 64.
//
// Why a wave, not a workgroup: at C4 a (sequence, head) is ~28 positions x
// 64 dims — a few µs of work that the workgroup form (csrc/attention.hip:
// K / V staged in LDS, one wave per 16-row query block, barriers between
// phases) spends mostly parked on its loads and barriers, with up to three
// of its four waves idle on short sequences and 36 KB of LDS capping a CU at
// four sequences in flight.  Here every operand goes global -> registers in
// the exact lane layout its MFMA takes, nothing touches LDS and nothing
// synchronises, so a CU holds as many (sequence, head) units as its register
// file allows (~100 VGPRs: 4-5 waves per SIMD) and their load latencies
// overlap one another.
//
// v_mfma_f32_16x16x4_f32 (exact f32 products).  Lane (j, g) = (lane & 15,
// lane >> 4).  A 16x16 accumulator holds C[4g + r][j] in element r; an A
// operand lane supplies A[j][g], a B operand lane B[g][j].  Two register
// layouts of a 16-row block X of a head slice are used:
//   κ ("contraction"): lane (j, g) holds Q4 = dh/4 dims of row j, dims
//     16c + 4g + e at step t = 4c + e (float4 loads; the t-th MFMA of a
//     product over dims contracts that dim).  Q, K, V, dO as A or B of S / dP.
//   π ("output"): lane (j, g) holds X[row 4g + r][NCB·σ(j) + cb] for r < 4,
//     cb < NCB = dh/16 (σ below), the A operand of a product that contracts
//     over rows and outputs dims: output dim block cb, row j of A is dim
//     NCB·σ(j) + cb, so the accumulator lane (j, g) ends up holding, per r,
//     the NCB contiguous dims from NCB·(4r + g) of one row.
//
// Forward (per query block w):  Sᵀ_kb = K_kb Q_wᵀ (A = K κ, B = Q κ; keys on
//   the accumulator rows, queries on the lanes), scale, causal mask, softmax
//   over keys (per lane + two shuffles) -> Pᵀ; Oᵀ = Σ_kb Vᵀ_kb Pᵀ_kb (A = V π,
//   B = Pᵀ as accumulated).  Also lse2 = max + log2 Σ per query (for backward).
// Softmax in base 2 (common.h exp2_hw): scores scaled by c2 = scale·log2(e),
// so each exponential is one v_exp_f32 and the backward's P = exp2(s·c2 −
// lse2) one fma + one v_exp_f32.
// Backward, two launches (FlashAttention-2's split, without its dQ atomics):
//   dq pass, per query block w:  δ = rowsum(dO ⊙ O); per kb <= w: Pᵀ =
//     exp2(Sᵀ·c2 − lse2), dPᵀ = V dOᵀ, dSᵀ = Pᵀ ⊙ (dPᵀ − δ)·scale, dQᵀ +=
//     Kᵀ dSᵀ (A = K π) -> store dQ rows and δ.
//   dkdv pass, per key block kb: per w >= kb: S = Q_w K_kbᵀ (queries on the
//     accumulator rows: A = Q κ, B = K κ), dP = dO V_kbᵀ, P and dS from lse /
//     δ; dVᵀ += dOᵀ P, dKᵀ += Qᵀ dS (A = dO π, Q π) -> store dK, dV rows.
// Every sum runs in a fixed order: results are bitwise reproducible.
#include "common.h"

namespace mirec {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kMaxT = 64;  // longest sequence
constexpr int kBlk = 16;   // block edge = MFMA tile edge
constexpr int kUnitsPerWG = 4;

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// N contiguous floats (N = 1, 2 or 4), zero when !ok.
template <int N>
__device__ __forceinline__ void ld_n(const float *p, bool ok, float *v) {
  if constexpr (N == 4) {
    const float4 x = ok ? ld4(p) : f4_zero();
    v[0] = x.x;
    v[1] = x.y;
    v[2] = x.z;
    v[3] = x.w;
  } else if constexpr (N == 2) {
    const float2 x = ok ? *reinterpret_cast<const float2 *>(p) : make_float2(0.f, 0.f);
    v[0] = x.x;
    v[1] = x.y;
  } else {
    v[0] = ok ? p[0] : 0.f;
  }
}

template <int N>
__device__ __forceinline__ void st_n(float *p, const float *v) {
  if constexpr (N == 4) {
    st4(p, make_float4(v[0], v[1], v[2], v[3]));
  } else if constexpr (N == 2) {
    *reinterpret_cast<float2 *>(p) = make_float2(v[0], v[1]);
  } else {
    p[0] = v[0];
  }
}

// κ layout of one row: step t = 4c + e contracts dim 16c + 4g + e, so the
// c-th float4 load of the 16 lanes of a row group covers 64 contiguous
// bytes of that row (one load instruction: 16 rows x 64 B).
template <int Q4>
__device__ __forceinline__ void ld_kappa(const float *row, int g, bool ok, float (&v)[Q4]) {
#pragma unroll
  for (int c = 0; c < Q4 / 4; ++c) ld_n<4>(row + 16 * c + 4 * g, ok, v + 4 * c);
}

// π layout: an A operand row j stands for dims NCB·σ(j) + cb (cb < NCB),
// σ(j) = 4 (j & 3) + (j >> 2), so a load of the 16 lanes covers the whole
// row and the accumulator lane (j, g) holds, for each r, the NCB contiguous
// dims from NCB·(4r + g): the 4 lane groups store 4·NCB contiguous floats.
__device__ __forceinline__ int sigma(int j) { return 4 * (j & 3) + (j >> 2); }

template <int NCB>
__device__ __forceinline__ void ld_pi(const float *row, int j, bool ok, float (&v)[NCB]) {
  ld_n<NCB>(row + NCB * sigma(j), ok, v);
}

template <int NCB>
__device__ __forceinline__ void st_out(float *row, int g, const f32x4 (&acc)[NCB]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) v[cb] = acc[cb][r];
    st_n<NCB>(row + NCB * (4 * r + g), v);
  }
}

// (sequence, head) of this wave; rows [row0, row0 + T) of the sequence.
struct Unit {
  int64_t row0;
  int T, h;
};

// order (optional): the sequence of every unit group, longest first
// (mirec_attention_length_order): a workgroup's four units have similar
// lengths and the longest units start first.
__device__ __forceinline__ bool unit_of(const int32_t *offsets, const int32_t *order,
                                        int T_uniform, int H, int64_t n_units, Unit &u) {
  const int64_t unit = (int64_t)blockIdx.x * kUnitsPerWG +
                       __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  if (unit >= n_units) return false;
  const int64_t b = order != nullptr ? (int64_t)order[unit / H] : unit / H;
  u.h = (int)(unit % H);
  if (offsets == nullptr) {
    u.row0 = b * T_uniform;
    u.T = T_uniform;
  } else {
    u.row0 = offsets[b];
    u.T = min(offsets[b + 1] - offsets[b], kMaxT);
  }
  return u.T > 0;
}

template <int DH>
// waves_per_eu(2): the preloaded unit (Q, K, V: 192 registers at dh = 64)
// still fits two waves per SIMD
__global__ __launch_bounds__(64 * kUnitsPerWG) __attribute__((amdgpu_waves_per_eu(2))) void attnw_fwd_kernel(
    const float *__restrict__ qkv, float *__restrict__ out, float *__restrict__ lse, int T_uniform,
    int H, float scale, const int32_t *__restrict__ offsets, const int32_t *__restrict__ order,
    int64_t n_units, int64_t batch, int64_t n_rows) {
  constexpr int Q4 = DH / 4, NCB = DH / 16;
  const int64_t unit_wgs = (n_units + kUnitsPerWG - 1) / kUnitsPerWG;
  if ((int64_t)blockIdx.x >= unit_wgs) {  // the padding rows [offsets[batch], n_rows) of out
    const int64_t w4 = (int64_t)H * DH / 4;
    const int64_t e0 = (int64_t)offsets[batch] * w4, e1 = n_rows * w4;
    const int64_t stride = ((int64_t)gridDim.x - unit_wgs) * blockDim.x;
    for (int64_t e = e0 + ((int64_t)blockIdx.x - unit_wgs) * blockDim.x + threadIdx.x; e < e1;
         e += stride)
      st4(out + 4 * e, f4_zero());
    return;
  }
  Unit u;
  if (!unit_of(offsets, order, T_uniform, H, n_units, u)) return;
  const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
  const int d = H * DH, T = u.T;
  const int64_t rs = 3 * (int64_t)d;
  const float *qb = qkv + u.row0 * rs + u.h * DH, *kb_ = qb + d, *vb = qb + 2 * d;
  const int nb = (T + kBlk - 1) / kBlk;
  // every operand of the unit in flight at once (one round trip): Q, K in
  // the κ layout, V in the π layout, for the sequence's nb blocks
  // rows past T load row T - 1 (unconditional loads, no exec-masked
  // branches): their scores are masked to -inf and their P is 0, and the
  // query rows past T are not stored; blocks past nb are not loaded
  // (wave-uniform) and never read
  float qa[4][Q4], k[4][Q4], v[4][4][NCB];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    if (b >= nb) break;
    const int r = min(kBlk * b + j, T - 1);
    ld_kappa<Q4>(qb + (int64_t)r * rs, g, true, qa[b]);
    ld_kappa<Q4>(kb_ + (int64_t)r * rs, g, true, k[b]);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int vr = min(kBlk * b + 4 * g + rr, T - 1);
      ld_pi<NCB>(vb + (int64_t)vr * rs, j, true, v[b][rr]);
    }
  }
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    if (w >= nb) break;
    const int qi = kBlk * w + j;
    const float c2 = scale * kLog2e;
    f32x4 s[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s[kb] = zero4();
      if (kb <= w) {
#pragma unroll
        for (int t = 0; t < Q4; ++t) s[kb] = mfma16(k[kb][t], qa[w][t], s[kb]);
      }
    }
    float m = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      if (kb > w) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kBlk * kb + 4 * g + r;
        const float x = (key > qi || key >= T) ? -INFINITY : s[kb][r] * c2;
        s[kb][r] = x;
        m = fmaxf(m, x);
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
        const float e = exp2_hw(s[kb][r] - m);
        s[kb][r] = e;
        sum += e;
      }
    }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    const float inv = 1.f / sum;
    f32x4 o[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) o[cb] = zero4();
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      if (kb > w) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = s[kb][r] * inv;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) o[cb] = mfma16(v[kb][r][cb], p, o[cb]);
      }
    }
    if (qi < T) {
      st_out<NCB>(out + (u.row0 + qi) * d + u.h * DH, g, o);
      if (g == 0 && lse != nullptr) lse[(u.row0 + qi) * H + u.h] = m + log2_hw(sum);
    }
  }
}

// dq pass: dQ rows and δ (= rowsum(dO ⊙ O)) of every query.
template <int DH>
__global__ __launch_bounds__(64 * kUnitsPerWG) void attnw_bwd_dq_kernel(
    const float *__restrict__ qkv, const float *__restrict__ out, const float *__restrict__ lse,
    const float *__restrict__ dout, float *__restrict__ dqkv, float *__restrict__ delta,
    int T_uniform, int H, float scale, const int32_t *__restrict__ offsets, const int32_t *__restrict__ order,
    int64_t n_units) {
  constexpr int Q4 = DH / 4, NCB = DH / 16;
  Unit u;
  if (!unit_of(offsets, order, T_uniform, H, n_units, u)) return;
  const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
  const int d = H * DH, T = u.T;
  const int64_t rs = 3 * (int64_t)d;
  const float *qb = qkv + u.row0 * rs + u.h * DH, *kb_ = qb + d, *vb = qb + 2 * d;
  const int nb = (T + kBlk - 1) / kBlk;
  for (int w = 0; w < nb; ++w) {
    const int qi = kBlk * w + j;
    const bool qok = qi < T;
    const int64_t qrow = u.row0 + qi;
    float q[Q4], dov[Q4], ov[Q4];
    ld_kappa<Q4>(qb + (int64_t)qi * rs, g, qok, q);
    ld_kappa<Q4>(dout + qrow * d + u.h * DH, g, qok, dov);
    ld_kappa<Q4>(out + qrow * d + u.h * DH, g, qok, ov);
    const float l = qok ? lse[qrow * H + u.h] : 0.f;
    float dl = 0.f;
#pragma unroll
    for (int t = 0; t < Q4; ++t) dl = fmaf(dov[t], ov[t], dl);
    dl += __shfl_xor(dl, 16);
    dl += __shfl_xor(dl, 32);
    f32x4 dq[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) dq[cb] = zero4();
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      if (kb > w) break;
      const int kr = kBlk * kb + j;
      float kk[Q4], vk[Q4], kp[4][NCB];
      ld_kappa<Q4>(kb_ + (int64_t)kr * rs, g, kr < T, kk);
      ld_kappa<Q4>(vb + (int64_t)kr * rs, g, kr < T, vk);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pr = kBlk * kb + 4 * g + r;
        ld_pi<NCB>(kb_ + (int64_t)pr * rs, j, pr < T, kp[r]);
      }
      f32x4 s = zero4(), dp = zero4();
#pragma unroll
      for (int t = 0; t < Q4; ++t) {
        s = mfma16(kk[t], q[t], s);
        dp = mfma16(vk[t], dov[t], dp);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kBlk * kb + 4 * g + r;
        const bool ok = key <= qi && qok;
        const float p = ok ? exp2_hw(fmaf(s[r], scale * kLog2e, -l)) : 0.f;
        const float ds = p * (dp[r] - dl) * scale;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) dq[cb] = mfma16(kp[r][cb], ds, dq[cb]);
      }
    }
    if (qok) {
      st_out<NCB>(dqkv + qrow * rs + u.h * DH, g, dq);
      if (g == 0) delta[qrow * H + u.h] = dl;
    }
  }
}

// dkdv pass: dK, dV rows of every key block.
template <int DH>
__global__ __launch_bounds__(64 * kUnitsPerWG) void attnw_bwd_dkdv_kernel(
    const float *__restrict__ qkv, const float *__restrict__ lse, const float *__restrict__ dout,
    const float *__restrict__ delta, float *__restrict__ dqkv, int T_uniform, int H, float scale,
    const int32_t *__restrict__ offsets, const int32_t *__restrict__ order, int64_t n_units) {
  constexpr int Q4 = DH / 4, NCB = DH / 16;
  Unit u;
  if (!unit_of(offsets, order, T_uniform, H, n_units, u)) return;
  const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
  const int d = H * DH, T = u.T;
  const int64_t rs = 3 * (int64_t)d;
  const float *qb = qkv + u.row0 * rs + u.h * DH, *kb_ = qb + d, *vb = qb + 2 * d;
  const float *dob = dout + u.row0 * d + u.h * DH;
  const int nb = (T + kBlk - 1) / kBlk;
  for (int kb = 0; kb < nb; ++kb) {
    const int key = kBlk * kb + j;
    float kk[Q4], vk[Q4];
    ld_kappa<Q4>(kb_ + (int64_t)key * rs, g, key < T, kk);
    ld_kappa<Q4>(vb + (int64_t)key * rs, g, key < T, vk);
    f32x4 dk[NCB], dv[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      dk[cb] = zero4();
      dv[cb] = zero4();
    }
    for (int w = kb; w < nb; ++w) {
      const int qj = kBlk * w + j;  // κ rows: query on the lane
      float qk[Q4], dok[Q4], qp[4][NCB], dp_[4][NCB], l[4], dl[4];
      ld_kappa<Q4>(qb + (int64_t)qj * rs, g, qj < T, qk);
      ld_kappa<Q4>(dob + (int64_t)qj * d, g, qj < T, dok);
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // π rows: query 16w + 4g + r
        const int qq = kBlk * w + 4 * g + r;
        const bool ok = qq < T;
        ld_pi<NCB>(qb + (int64_t)qq * rs, j, ok, qp[r]);
        ld_pi<NCB>(dob + (int64_t)qq * d, j, ok, dp_[r]);
        l[r] = ok ? lse[(u.row0 + qq) * H + u.h] : 0.f;
        dl[r] = ok ? delta[(u.row0 + qq) * H + u.h] : 0.f;
      }
      f32x4 s = zero4(), dp = zero4();
#pragma unroll
      for (int t = 0; t < Q4; ++t) {
        s = mfma16(qk[t], kk[t], s);
        dp = mfma16(dok[t], vk[t], dp);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = kBlk * w + 4 * g + r;
        const bool ok = key <= qq && qq < T;
        const float p = ok ? exp2_hw(fmaf(s[r], scale * kLog2e, -l[r])) : 0.f;
        const float ds = p * (dp[r] - dl[r]) * scale;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          dv[cb] = mfma16(dp_[r][cb], p, dv[cb]);
          dk[cb] = mfma16(qp[r][cb], ds, dk[cb]);
        }
      }
    }
    if (key < T) {
      float *row = dqkv + (u.row0 + key) * rs + u.h * DH;
      st_out<NCB>(row + d, g, dk);
      st_out<NCB>(row + 2 * d, g, dv);
    }
  }
}

// order = the sequences by length, longest first (counting sort over the 65
// clamped lengths; the order among equal lengths is arbitrary — it changes
// no result, every unit is independent).  packs (optional, int32 [4 + 8
// batch], 16-byte aligned): packs[0] = the pack count, packs[4 + 8p + 2s],
// packs[5 + 8p + 2s] = (first row, length) of the sequence in slot s of pack
// p, (0, 0) for an empty slot — the descriptor the backward workgroup reads
// with two 16-byte loads, no dependent load of the offsets.  Over the same
// order, each sequence of 49-64 positions (4 blocks of 16) is a pack of its
// own; each of 33-48 (3 blocks) takes a sequence of 1-16 (1 block) into its
// fourth wave while there are any (the longest of each); those of 17-32 go
// two to a pack and the remaining 1-16 four to a pack (empty sequences in
// none): mirec_attention_packed_bwd's workgroups, longest first.
__global__ __launch_bounds__(1024) void length_order_kernel(const int32_t *__restrict__ offsets,
                                                           int64_t batch,
                                                           int32_t *__restrict__ order,
                                                           int32_t *__restrict__ packs,
                                                           float *__restrict__ zero_buf,
                                                           int64_t zero_rows, int32_t zero_w4) {
  if (blockIdx.x > 0) {  // workgroups 1..: the capacity padding rows of the output
    const int64_t e0 = (int64_t)offsets[batch] * zero_w4, e1 = zero_rows * zero_w4;
    const int64_t stride = (int64_t)(gridDim.x - 1) * blockDim.x;
    for (int64_t e = e0 + (int64_t)(blockIdx.x - 1) * blockDim.x + threadIdx.x; e < e1;
         e += stride)
      st4(zero_buf + 4 * e, f4_zero());
    return;
  }
  __shared__ int cnt[kMaxT + 1], start[kMaxT + 1];
  __shared__ int cls_start[5], cls_count[5], pack_base[5], n31;
  for (int i = threadIdx.x; i <= kMaxT; i += blockDim.x) cnt[i] = 0;
  __syncthreads();
  for (int64_t b = threadIdx.x; b < batch; b += blockDim.x)
    atomicAdd(&cnt[min(offsets[b + 1] - offsets[b], kMaxT)], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int L = kMaxT; L >= 0; --L) {
      start[L] = acc;
      acc += cnt[L];
    }
    // classes by block count k = ceil(L / 16), contiguous in the order
    for (int k = 0; k <= 4; ++k) cls_count[k] = 0;
    for (int L = 0; L <= kMaxT; ++L) cls_count[(L + kBlk - 1) / kBlk] += cnt[L];
    // 3-block sequences carry a 1-block one in their idle fourth wave
    n31 = min(cls_count[3], cls_count[1]);
    int pos = 0, pb = 0;
    for (int k = 4; k >= 1; --k) {
      const int per = k >= 3 ? 1 : (k == 2 ? 2 : 4);
      const int alone = k == 1 ? cls_count[1] - n31 : cls_count[k];  // in packs of class k
      cls_start[k] = pos;
      pack_base[k] = pb;
      pos += cls_count[k];
      pb += (alone + per - 1) / per;
    }
    cls_start[0] = pos;
    pack_base[0] = pb;  // = the pack count
  }
  __syncthreads();
  if (packs != nullptr) {
    const int n_packs = pack_base[0];
    if (threadIdx.x < 4) packs[threadIdx.x] = threadIdx.x == 0 ? n_packs : 0;
    // slots no sequence fills: (0, 0) (written before, and disjoint from,
    // the sequence slots below)
    for (int p = threadIdx.x; p < n_packs; p += blockDim.x) {
      // class of pack p: the k with pack_base[k] <= p < pack_base[k - 1]
      int k = 4;
      while (k > 1 && p >= pack_base[k - 1]) --k;
      const int per = k >= 3 ? 1 : (k == 2 ? 2 : 4);
      const int i = p - pack_base[k];
      const int used = k == 3   ? 1 + (i < n31 ? 1 : 0)
                       : k == 1 ? min(per, cls_count[1] - n31 - i * per)
                                : min(per, cls_count[k] - i * per);
      for (int sl = used; sl < 4; ++sl) {
        packs[4 + 8 * (int64_t)p + 2 * sl] = 0;
        packs[5 + 8 * (int64_t)p + 2 * sl] = 0;
      }
    }
  }
  for (int64_t b = threadIdx.x; b < batch; b += blockDim.x) {
    const int L = min(offsets[b + 1] - offsets[b], kMaxT);
    const int pos = atomicAdd(&start[L], 1);
    order[pos] = (int32_t)b;
    const int k = (L + kBlk - 1) / kBlk;
    if (packs != nullptr && k > 0) {
      const int per = k >= 3 ? 1 : (k == 2 ? 2 : 4);
      const int i = pos - cls_start[k];
      int64_t slot;
      if (k == 1 && i < n31)  // slot 1 of the i-th 3-block pack (blocks 3)
        slot = 4 + 8 * (int64_t)(pack_base[3] + i) + 2;
      else {
        const int ia = k == 1 ? i - n31 : i;
        slot = 4 + 8 * (int64_t)(pack_base[k] + ia / per) + 2 * (ia % per);
      }
      packs[slot] = offsets[b];
      packs[slot + 1] = L;
    }
  }
}

template <int DH>
int launch_fwd(const float *qkv, const int32_t *offsets, const int32_t *order, int64_t units, int T,
               int H, float *out, float *lse, int64_t batch, int64_t n_rows, hipStream_t st) {
  // unit workgroups, plus 32 that zero the padding rows when asked
  const int64_t unit_wgs = (units + kUnitsPerWG - 1) / kUnitsPerWG;
  const dim3 grid((unsigned)(unit_wgs + (n_rows > 0 && offsets ? 32 : 0))),
      block(64 * kUnitsPerWG);
  hipLaunchKernelGGL((attnw_fwd_kernel<DH>), grid, block, 0, st, qkv, out, lse, T, H,
                     1.f / sqrtf((float)DH), offsets, order, units, batch, n_rows);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

template <int DH>
int launch_bwd(const float *qkv, const float *out, const float *lse, const float *dout,
               const int32_t *offsets, const int32_t *order, int64_t units, int T, int H,
               float *dqkv, float *delta, hipStream_t st) {
  const dim3 grid((unsigned)((units + kUnitsPerWG - 1) / kUnitsPerWG)), block(64 * kUnitsPerWG);
  const float scale = 1.f / sqrtf((float)DH);
  hipLaunchKernelGGL((attnw_bwd_dq_kernel<DH>), grid, block, 0, st, qkv, out, lse, dout, dqkv,
                     delta, T, H, scale, offsets, order, units);
  MIREC_LAUNCH_CHECK();
  hipLaunchKernelGGL((attnw_bwd_dkdv_kernel<DH>), grid, block, 0, st, qkv, lse, dout, delta,
                     dqkv, T, H, scale, offsets, order, units);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

}  // namespace
}  // namespace mirec

using namespace mirec;

static bool wave_dims_ok(int32_t head_dim) {
  return head_dim == 16 || head_dim == 32 || head_dim == 64;
}

extern "C" int mirec_attention_wave_supported(int32_t head_dim) {
  return wave_dims_ok(head_dim) ? 1 : 0;
}

extern "C" int mirec_attention_length_order(const int32_t *offsets, int64_t batch,
                                            int32_t *order, int32_t *packs, float *zero_buf,
                                            int64_t zero_rows, int32_t zero_width,
                                            mirec_stream_t stream) {
  MIREC_CHECK_ARG(batch >= 0 && batch <= INT32_MAX / 4);
  MIREC_CHECK_ARG(zero_buf == nullptr ||
                  (zero_rows >= 0 && zero_width > 0 && zero_width % 4 == 0 &&
                   (uintptr_t)zero_buf % 16 == 0));
  if (batch == 0) {
    if (packs != nullptr) return hipMemsetAsync(packs, 0, sizeof(int32_t),
                                                reinterpret_cast<hipStream_t>(stream)) ==
                                           hipSuccess ? MIREC_OK : MIREC_ERR_HIP;
    return MIREC_OK;
  }
  MIREC_CHECK_ARG(offsets && order && (uintptr_t)packs % 16 == 0);
  // workgroup 0 orders and packs; with zero_buf, 32 more zero the padding
  hipLaunchKernelGGL(length_order_kernel, dim3(zero_buf != nullptr ? 33 : 1), dim3(1024), 0,
                     reinterpret_cast<hipStream_t>(stream), offsets, batch, order, packs,
                     zero_buf, zero_rows, zero_width / 4);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_attention_wave_fwd(const float *qkv, const int32_t *offsets,
                                        const int32_t *order, int64_t batch, int32_t T,
                                        int32_t heads, int32_t head_dim, float *out, float *lse,
                                        int64_t n_rows, mirec_stream_t stream) {
  MIREC_CHECK_ARG(batch >= 0 && heads >= 1 && wave_dims_ok(head_dim));
  MIREC_CHECK_ARG(offsets != nullptr || (T >= 1 && T <= kMaxT));
  if (batch == 0) return MIREC_OK;
  MIREC_CHECK_ARG(qkv && out && lse && ((uintptr_t)qkv | (uintptr_t)out) % 16 == 0);
  const int64_t units = batch * heads;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (head_dim) {
    case 16: return launch_fwd<16>(qkv, offsets, order, units, T, heads, out, lse, batch, n_rows, st);
    case 32: return launch_fwd<32>(qkv, offsets, order, units, T, heads, out, lse, batch, n_rows, st);
    default: return launch_fwd<64>(qkv, offsets, order, units, T, heads, out, lse, batch, n_rows, st);
  }
}

extern "C" int mirec_attention_wave_bwd(const float *qkv, const float *out, const float *lse,
                                        const float *dout, const int32_t *offsets,
                                        const int32_t *order, int64_t batch, int32_t T,
                                        int32_t heads, int32_t head_dim, float *dqkv,
                                        float *delta, mirec_stream_t stream) {
  MIREC_CHECK_ARG(batch >= 0 && heads >= 1 && wave_dims_ok(head_dim));
  MIREC_CHECK_ARG(offsets != nullptr || (T >= 1 && T <= kMaxT));
  if (batch == 0) return MIREC_OK;
  MIREC_CHECK_ARG(qkv && out && lse && dout && dqkv && delta);
  MIREC_CHECK_ARG(((uintptr_t)qkv | (uintptr_t)out | (uintptr_t)dout | (uintptr_t)dqkv) % 16 ==
                  0);
  const int64_t units = batch * heads;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (head_dim) {
    case 16:
      return launch_bwd<16>(qkv, out, lse, dout, offsets, order, units, T, heads, dqkv, delta, st);
    case 32:
      return launch_bwd<32>(qkv, out, lse, dout, offsets, order, units, T, heads, dqkv, delta, st);
    default:
      return launch_bwd<64>(qkv, out, lse, dout, offsets, order, units, T, heads, dqkv, delta, st);
  }
}
