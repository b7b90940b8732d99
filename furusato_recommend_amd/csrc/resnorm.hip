// The row-wise tail of the SASRec block (model/sasrec.py:385-397) fused into
// one pass per stage:
//
//   pre = res + dropout(z + bias)        (res / bias / dropout optional)
//   out = relu ? max(pre, 0) : pre
//   y   = LayerNorm(out) * gamma + beta  (optional; torch's eps, biased var)
//
// The block is  y1 = LN_a(x);  a = attn(y1) W_oᵀ;  h, y2 = (x + drop(a + b_o),
// relu, LN_f);  f = y2 W_fᵀ;  x', y1' = (h + drop(f + b_f), LN_a of the next
// layer).  Unfused, every arrow is its own torch launch (add, dropout, relu,
// layer norm and their backwards: ~14 elementwise passes over the token
// rows per layer); here it is one forward and one backward pass per stage.
// The linear biases ride along so their gradients come out of the same
// backward pass (no separate column reduction).
//
// Layout: rows of d floats (d % 4 == 0, d <= 1024); LPR lanes own one row,
// NC float4 per lane, lane-group reductions by xor shuffles.  Dropout masks
// are the counter hash of common.h over (row * d + col), recomputed in the
// backward.  Parameter gradients are column sums over all rows: every block
// writes one [3, d] partial (dgamma, dbeta, dbias) and a second launch adds
// the partials in block order (deterministic).
#include "common.h"

namespace mirec {

namespace {

constexpr int kBlock = 256;
constexpr int kMaxFwdBlocks = 4096;
constexpr int kMaxBwdBlocks = 1024;

struct FwdArgs {
  const float *res, *z, *bias, *gamma, *beta;
  float *out, *y, *mean, *rstd;
  int64_t n;
  int32_t d, relu;
  uint64_t key;
  uint32_t thresh;
  float scale, eps;
  const uint64_t *key_base;  // device; mixed into key at run time (graph replays)
};

struct BwdArgs {
  const float *g_y, *g_out, *out, *mean, *rstd, *gamma;
  float *d_res, *d_z, *partial;
  int64_t n;
  int32_t d, relu;
  uint64_t key;
  uint32_t thresh;
  float scale;
  const uint64_t *key_base;
};


__device__ __forceinline__ float4 relu_mask(float4 g, float4 v) {
  return make_float4(v.x > 0.f ? g.x : 0.f, v.y > 0.f ? g.y : 0.f, v.z > 0.f ? g.z : 0.f,
                     v.w > 0.f ? g.w : 0.f);
}

__device__ __forceinline__ float4 f4_mul(float4 a, float4 b) {
  return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}

template <int LPR, int NC>
__global__ __launch_bounds__(kBlock) void resnorm_fwd_kernel(FwdArgs a) {
  constexpr int RPB = kBlock / LPR;
  const uint64_t key = a.thresh != 0u ? run_key(a.key, a.key_base) : 0ull;
  const int lane = threadIdx.x % LPR;
  const int64_t d = a.d;
  const float inv_d = 1.f / (float)a.d;
  float4 gam[NC], bet[NC], bia[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = 4 * (lane + k * LPR);
    const bool ok = c < a.d;
    gam[k] = ok && a.gamma ? ld4(a.gamma + c) : make_float4(1.f, 1.f, 1.f, 1.f);
    bet[k] = ok && a.beta ? ld4(a.beta + c) : f4_zero();
    bia[k] = ok && a.bias ? ld4(a.bias + c) : f4_zero();
  }
  for (int64_t r = (int64_t)blockIdx.x * RPB + threadIdx.x / LPR; r < a.n;
       r += (int64_t)gridDim.x * RPB) {
    float4 v[NC];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = 4 * (lane + k * LPR);
      v[k] = f4_zero();
      if (c < a.d) {
        const int64_t e = r * d + c;
        float4 x = f4_add(ld4(a.z + e), bia[k]);
        if (a.thresh != 0u) x = drop4(x, key, (uint64_t)e, a.thresh, a.scale);
        if (a.res) x = f4_add(x, ld4(a.res + e));
        if (a.relu)
          x = make_float4(fmaxf(x.x, 0.f), fmaxf(x.y, 0.f), fmaxf(x.z, 0.f), fmaxf(x.w, 0.f));
        if (a.out) st4(a.out + e, x);
        v[k] = x;
        s += (x.x + x.y) + (x.z + x.w);
      }
    }
    if (a.y == nullptr) continue;
    const float mu = group_sum<LPR>(s) * inv_d;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      if (4 * (lane + k * LPR) < a.d) {
        const float4 t = f4_sub(v[k], make_float4(mu, mu, mu, mu));
        q += f4_dot(t, t);
      }
    }
    const float rs = rsqrtf(group_sum<LPR>(q) * inv_d + a.eps);
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = 4 * (lane + k * LPR);
      if (c < a.d) {
        const float4 t = f4_scale(rs, f4_sub(v[k], make_float4(mu, mu, mu, mu)));
        st4(a.y + r * d + c, f4_add(f4_mul(t, gam[k]), bet[k]));
      }
    }
    if (lane == 0) {
      a.mean[r] = mu;
      a.rstd[r] = rs;
    }
  }
}

template <int LPR, int NC>
__global__ __launch_bounds__(kBlock) void resnorm_bwd_kernel(BwdArgs a) {
  constexpr int RPB = kBlock / LPR;
  const uint64_t key = a.thresh != 0u ? run_key(a.key, a.key_base) : 0ull;
  constexpr int DW = 4 * LPR * NC;  // padded row width
  __shared__ float red[RPB][3][DW];
  const int lane = threadIdx.x % LPR, grp = threadIdx.x / LPR;
  const int64_t d = a.d;
  const float inv_d = 1.f / (float)a.d;
  float4 gam[NC], pg[NC], pb[NC], pz[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = 4 * (lane + k * LPR);
    gam[k] = c < a.d && a.gamma ? ld4(a.gamma + c) : make_float4(1.f, 1.f, 1.f, 1.f);
    pg[k] = pb[k] = pz[k] = f4_zero();
  }
  for (int64_t r = (int64_t)blockIdx.x * RPB + grp; r < a.n; r += (int64_t)gridDim.x * RPB) {
    float4 v[NC], gy[NC], g[NC];
    float s1 = 0.f, s2 = 0.f;
    float mu = 0.f, rs = 0.f;
    if (a.g_y) {
      mu = a.mean[r];
      rs = a.rstd[r];
    }
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = 4 * (lane + k * LPR);
      v[k] = gy[k] = g[k] = f4_zero();
      if (c < a.d) {
        const int64_t e = r * d + c;
        v[k] = ld4(a.out + e);
        if (a.g_out) g[k] = ld4(a.g_out + e);
        if (a.g_y) {
          gy[k] = ld4(a.g_y + e);
          const float4 xh = f4_scale(rs, f4_sub(v[k], make_float4(mu, mu, mu, mu)));
          const float4 gx = f4_mul(gy[k], gam[k]);
          s1 += (gx.x + gx.y) + (gx.z + gx.w);
          s2 += f4_dot(gx, xh);
        }
      }
    }
    if (a.g_y) {
      const float m1 = group_sum<LPR>(s1) * inv_d;
      const float m2 = group_sum<LPR>(s2) * inv_d;
#pragma unroll
      for (int k = 0; k < NC; ++k) {
        if (4 * (lane + k * LPR) < a.d) {
          const float4 xh = f4_scale(rs, f4_sub(v[k], make_float4(mu, mu, mu, mu)));
          const float4 gx = f4_mul(gy[k], gam[k]);
          // dx = rstd * (gx - mean(gx) - xhat * mean(gx * xhat))
          const float4 t = f4_sub(f4_sub(gx, make_float4(m1, m1, m1, m1)), f4_scale(m2, xh));
          g[k] = f4_fma(rs, t, g[k]);
          pg[k] = f4_add(pg[k], f4_mul(gy[k], xh));
          pb[k] = f4_add(pb[k], gy[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = 4 * (lane + k * LPR);
      if (c < a.d) {
        const int64_t e = r * d + c;
        float4 x = a.relu ? relu_mask(g[k], v[k]) : g[k];
        if (a.d_res) st4(a.d_res + e, x);
        if (a.thresh != 0u) x = drop4(x, key, (uint64_t)e, a.thresh, a.scale);
        if (a.d_z) st4(a.d_z + e, x);
        pz[k] = f4_add(pz[k], x);
      }
    }
  }
  if (a.partial == nullptr) return;  // block-uniform
  // column partials of this block: lane groups -> LDS -> one [3, d] row
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = 4 * (lane + k * LPR);
    *reinterpret_cast<float4 *>(&red[grp][0][c]) = pg[k];
    *reinterpret_cast<float4 *>(&red[grp][1][c]) = pb[k];
    *reinterpret_cast<float4 *>(&red[grp][2][c]) = pz[k];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * a.d; i += kBlock) {
    const int t = i / a.d, c = i - t * a.d;
    float acc = 0.f;
#pragma unroll 8
    for (int q = 0; q < RPB; ++q) acc += red[q][t][c];
    a.partial[(int64_t)blockIdx.x * 3 * a.d + i] = acc;
  }
}

// out[j] = sum over parts of partial[p][j] for the 3*d columns; one
// workgroup of 1024 threads per 64 columns, 16 waves splitting the parts.
__global__ __launch_bounds__(1024) void resnorm_reduce_kernel(const float *__restrict__ partial,
                                                              int32_t parts, int32_t d,
                                                              float *d_gamma, float *d_beta,
                                                              float *d_bias) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  const int cols = 3 * d;
  float acc = 0.f;
  if (j < cols) {
    // 16 partials' loads in flight per round (sum order unchanged)
    for (int p0 = w; p0 < parts; p0 += 16 * 16) {
      float x[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int p = p0 + 16 * u;
        x[u] = p < parts ? partial[(int64_t)p * cols + j] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (p0 + 16 * u < parts) acc += x[u];
    }
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && j < cols) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) s += red[q][lane];
    const int t = j / d, c = j - t * d;
    float *dst = t == 0 ? d_gamma : (t == 1 ? d_beta : d_bias);
    if (dst) dst[c] = s;
  }
}

struct Shape {
  int lpr, nc;
};

inline bool pick_shape(int32_t d, Shape *s) {
  if (d < 4 || d % 4 || d > 1024) return false;
  const int d4 = d / 4;
  int lpr = 1;
  while (lpr < d4 && lpr < 64) lpr <<= 1;
  const int nc = (d4 + lpr - 1) / lpr;
  s->lpr = lpr;
  s->nc = nc <= 1 ? 1 : (nc <= 2 ? 2 : 4);
  return true;
}

#define MIREC_RESNORM_SWITCH(KERNEL, SH, GRID, ARGS, STREAM)                        \
  do {                                                                              \
    switch ((SH).nc == 1 ? (SH).lpr : 64 * (SH).nc) {                              \
      case 1: KERNEL<1, 1><<<GRID, kBlock, 0, STREAM>>>(ARGS); break;              \
      case 2: KERNEL<2, 1><<<GRID, kBlock, 0, STREAM>>>(ARGS); break;              \
      case 4: KERNEL<4, 1><<<GRID, kBlock, 0, STREAM>>>(ARGS); break;              \
      case 8: KERNEL<8, 1><<<GRID, kBlock, 0, STREAM>>>(ARGS); break;              \
      case 16: KERNEL<16, 1><<<GRID, kBlock, 0, STREAM>>>(ARGS); break;            \
      case 32: KERNEL<32, 1><<<GRID, kBlock, 0, STREAM>>>(ARGS); break;            \
      case 64: KERNEL<64, 1><<<GRID, kBlock, 0, STREAM>>>(ARGS); break;            \
      case 128: KERNEL<64, 2><<<GRID, kBlock, 0, STREAM>>>(ARGS); break;           \
      default: KERNEL<64, 4><<<GRID, kBlock, 0, STREAM>>>(ARGS); break;            \
    }                                                                               \
  } while (0)

inline int64_t blocks_for(int64_t n, const Shape &s, int64_t cap) {
  const int64_t rpb = kBlock / s.lpr;
  const int64_t b = (n + rpb - 1) / rpb;
  return b < 1 ? 1 : (b > cap ? cap : b);
}

}  // namespace

}  // namespace mirec

using namespace mirec;

extern "C" int mirec_resnorm_fwd(const float *res, const float *z, const float *bias,
                                 const float *gamma, const float *beta, int64_t n, int32_t d,
                                 int32_t relu, float dropout_p, uint64_t seed,
                                 const uint64_t *seed_base, float eps, float *out, float *y,
                                 float *mean, float *rstd, mirec_stream_t stream) {
  Shape sh;
  MIREC_CHECK_ARG(n >= 0 && pick_shape(d, &sh));
  FwdArgs a{res, z, bias, gamma, beta, out, y, mean, rstd, n, d, relu ? 1 : 0, 0, 0u, 1.f, eps,
            seed_base};
  MIREC_CHECK_ARG(dropout_params(dropout_p, seed, &a.key, &a.thresh, &a.scale));
  if (n == 0) return MIREC_OK;  // (empty tensors may carry null pointers)
  MIREC_CHECK_ARG(z != nullptr);
  // out may be omitted only when it equals z
  MIREC_CHECK_ARG(out != nullptr || (res == nullptr && bias == nullptr && !relu && a.thresh == 0u));
  MIREC_CHECK_ARG(y == nullptr || (mean != nullptr && rstd != nullptr));
  MIREC_CHECK_ARG(out != nullptr || y != nullptr);
  const int64_t grid = blocks_for(n, sh, kMaxFwdBlocks);
  hipStream_t s = (hipStream_t)stream;
  MIREC_RESNORM_SWITCH(resnorm_fwd_kernel, sh, (unsigned)grid, a, s);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int64_t mirec_resnorm_work_floats(int64_t n, int32_t d) {
  Shape sh;
  if (n < 0 || !pick_shape(d, &sh)) return -1;
  return blocks_for(n, sh, kMaxBwdBlocks) * 3 * (int64_t)d;
}

extern "C" int mirec_resnorm_bwd(const float *g_y, const float *g_out, const float *out,
                                 const float *mean, const float *rstd, const float *gamma,
                                 int64_t n, int32_t d, int32_t relu, float dropout_p,
                                 uint64_t seed, const uint64_t *seed_base, float *d_res,
                                 float *d_z, float *work,
                                 float *d_gamma, float *d_beta, float *d_bias,
                                 mirec_stream_t stream) {
  Shape sh;
  MIREC_CHECK_ARG(n >= 0 && pick_shape(d, &sh));
  BwdArgs a{g_y, g_out, out, mean, rstd, gamma, d_res, d_z, work, n, d, relu ? 1 : 0, 0, 0u, 1.f,
            seed_base};
  MIREC_CHECK_ARG(dropout_params(dropout_p, seed, &a.key, &a.thresh, &a.scale));
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {  // empty sums; empty tensors may carry null pointers
    if (d_gamma) MIREC_HIP(hipMemsetAsync(d_gamma, 0, sizeof(float) * d, s));
    if (d_beta) MIREC_HIP(hipMemsetAsync(d_beta, 0, sizeof(float) * d, s));
    if (d_bias) MIREC_HIP(hipMemsetAsync(d_bias, 0, sizeof(float) * d, s));
    return MIREC_OK;
  }
  MIREC_CHECK_ARG(g_y == nullptr || (mean != nullptr && rstd != nullptr));
  MIREC_CHECK_ARG(g_y != nullptr || (d_gamma == nullptr && d_beta == nullptr));
  const bool sums = d_gamma || d_beta || d_bias;
  MIREC_CHECK_ARG(out != nullptr && (!sums || work != nullptr));
  const int64_t grid = blocks_for(n, sh, kMaxBwdBlocks);
  if (!sums) a.partial = nullptr;
  MIREC_RESNORM_SWITCH(resnorm_bwd_kernel, sh, (unsigned)grid, a, s);
  MIREC_LAUNCH_CHECK();
  if (sums) {
    resnorm_reduce_kernel<<<(unsigned)((3 * d + 63) / 64), 1024, 0, s>>>(
        work, (int32_t)grid, d, d_gamma, d_beta, d_bias);
    MIREC_LAUNCH_CHECK();
  }
  return MIREC_OK;
}

// The fixed-order column reduce of [parts][3][d] partials (shared with the
// fused GEMM + row-tail backward, csrc/gemm.hip).
extern "C" int mirec_resnorm_reduce_partials(const float *work, int64_t parts, int32_t d,
                                             float *d_gamma, float *d_beta, float *d_bias,
                                             mirec_stream_t stream) {
  MIREC_CHECK_ARG(work && parts > 0 && parts <= INT32_MAX && d > 0);
  resnorm_reduce_kernel<<<(unsigned)((3 * d + 63) / 64), 1024, 0, (hipStream_t)stream>>>(
      work, (int32_t)parts, d, d_gamma, d_beta, d_bias);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}
