// Fused BPR loss / gradient seeds for LightGCN (model/lgcn.py:98-133).
//
// Forward (one LPR-lane group per triple, float4 row reads):
//   pos = <out_u, out_p>, neg = <out_u, out_n>, sp = softplus(neg - pos)
//   reg = 1/2 (|e_u|^2 + |e_p|^2 + |e_n|^2)          (ego rows, lgcn.py:103-112)
//   coef = d mean(sp)/d(neg-pos) = (1/B) * sigmoid(neg-pos)  (threshold 20)
// Loss: a single-workgroup fixed-order reduction (deterministic).
// Seeds: the 3B (node, occurrence) pairs are radix-sorted (stable, rocPRIM via
// hipCUB); the head position q of every distinct node owns the node's
// gradient row and sums the node's occurrences in occurrence order:
//   user occurrence:  coef * out_n - coef * out_p
//   pos  occurrence: -coef * out_u
//   neg  occurrence:  coef * out_u
// seed_p[q] = that / (L+1)  (the d/dx_l of the layer mean, lgcn.py:85)
// seed_e[q] = decay * sum_occ e_node / B  (d decay*reg / d e)
// slot[node] = q publishes the row to the propagation epilogues.
#include <hipcub/hipcub.hpp>

#include "common.h"
#include "smallsort.h"

namespace mirec {

constexpr int kWaves = 4;

template <int D>
__global__ __launch_bounds__(256) MIREC_NO_PK_F32 void bpr_forward_kernel(
    const float *__restrict__ out, const float *__restrict__ emb, int64_t n_users,
    int64_t batch, const int32_t *__restrict__ users, const int32_t *__restrict__ pos,
    const int32_t *__restrict__ neg, float grad_scale, float *coef, float *softplus, float *reg,
    int32_t *keys, int32_t *vals) {
  constexpr int LPR = D / 4;
  constexpr int G = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int sub = lane % LPR;
  const int64_t t = ((int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * G + lane / LPR;
  const bool live = t < batch;
  const int64_t tt = live ? t : 0;
  const int64_t u = users[tt];
  const int64_t p = n_users + pos[tt];
  const int64_t n = n_users + neg[tt];
  const float4 ou = ld4(out + u * D + sub * 4);
  const float4 op = ld4(out + p * D + sub * 4);
  const float4 on = ld4(out + n * D + sub * 4);
  const float4 eu = ld4(emb + u * D + sub * 4);
  const float4 ep = ld4(emb + p * D + sub * 4);
  const float4 en = ld4(emb + n * D + sub * 4);
  const float ps = group_sum<LPR>(f4_dot(ou, op));
  const float ns = group_sum<LPR>(f4_dot(ou, on));
  const float r = group_sum<LPR>(f4_dot(eu, eu) + f4_dot(ep, ep) + f4_dot(en, en));
  if (live && sub == 0) {
    const float x = ns - ps;
    const float invb = 1.f / (float)batch;
    float sp, c;
    if (x > 20.f) {  // torch softplus(beta=1, threshold=20)
      sp = x;
      c = invb;
    } else {
      const float z = expf(x);
      sp = log1pf(z);
      c = invb * z / (z + 1.f);
    }
    if (grad_scale != 1.f) c *= grad_scale;
    softplus[t] = sp;
    coef[t] = c;
    reg[t] = 0.5f * r;
    keys[t] = (int32_t)u;
    keys[batch + t] = (int32_t)p;
    keys[2 * batch + t] = (int32_t)n;
    vals[t] = (int32_t)t;
    vals[batch + t] = (int32_t)(batch + t);
    vals[2 * batch + t] = (int32_t)(2 * batch + t);
  }
}

// Single workgroup, fixed partition and tree: deterministic loss.
__global__ __launch_bounds__(1024) void bpr_loss_kernel(const float *softplus, const float *reg,
                                                        int64_t batch, float decay,
                                                        float *loss_out, float *loss_accum) {
  __shared__ float s_sp[1024];
  __shared__ float s_rg[1024];
  float a = 0.f, b = 0.f;
  for (int64_t i = threadIdx.x; i < batch; i += 1024) {
    a += softplus[i];
    b += reg[i];
  }
  s_sp[threadIdx.x] = a;
  s_rg[threadIdx.x] = b;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      s_sp[threadIdx.x] += s_sp[threadIdx.x + s];
      s_rg[threadIdx.x] += s_rg[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float fb = (float)batch;
    const float loss = s_sp[0] / fb + decay * (s_rg[0] / fb);
    loss_out[0] = loss;
    if (loss_accum != nullptr) loss_accum[0] += loss;
  }
}

__global__ void seed_heads_kernel(const int32_t *keys_sorted, int64_t n, int32_t *slot) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  const int32_t k = keys_sorted[q];
  if (q == 0 || keys_sorted[q - 1] != k) slot[k] = (int32_t)q;
}

template <int D>
__global__ __launch_bounds__(256) void seed_accum_kernel(
    const float *__restrict__ out, const float *__restrict__ emb, int64_t n_users,
    int64_t batch, const int32_t *__restrict__ users, const int32_t *__restrict__ pos,
    const int32_t *__restrict__ neg, const float *__restrict__ coef,
    const int32_t *__restrict__ keys_sorted, const int32_t *__restrict__ vals_sorted,
    float decay, float grad_scale, float layer_div, float *seed_p, float *seed_e) {
  constexpr int LPR = D / 4;
  constexpr int G = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int sub = lane % LPR;
  const int64_t n = 3 * batch;
  const int64_t q = ((int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * G + lane / LPR;
  if (q >= n) return;
  const int32_t node = keys_sorted[q];
  if (q > 0 && keys_sorted[q - 1] == node) return;  // not the head of its run
  // The run is walked LPR entries per round: lane j decodes entry q0 + j
  // (source rows and coefficients), then the group loads the rows 8 at a
  // time and adds them in entry order — the serial walk's exact sequence of
  // fmas (bitwise equal) without one dependent index chain per entry (a
  // Zipf-popular item is hundreds of entries of a batch).
  const int base = lane - sub;
  const unsigned long long low = LPR == 64 ? ~0ull : ((1ull << LPR) - 1ull);
  const unsigned long long gmask = low << base;
  float4 gp = f4_zero();
  int cnt = 0;
  for (int64_t q0 = q;; q0 += LPR) {
    const int64_t qj = q0 + sub;
    const bool in = qj < n && keys_sorted[qj] == node;
    int32_t ra = -1, rb = -1;
    float ca = 0.f, cb = 0.f;
    if (in) {
      const int64_t occ = vals_sorted[qj];
      const int64_t role = occ / batch;
      const int64_t t = occ - role * batch;
      const float c = coef[t];
      if (role == 0) {  // the negative's row, then the positive's
        ra = (int32_t)(n_users + neg[t]);
        ca = c;
        rb = (int32_t)(n_users + pos[t]);
        cb = -c;
      } else {
        ra = users[t];
        ca = role == 1 ? -c : c;
      }
    }
    const unsigned long long bal = (__ballot(in) & gmask) >> base;
    const int m = bal == low ? LPR : (int)__builtin_ctzll(~bal);
    for (int u0 = 0; u0 < m; u0 += 8) {
      float4 xa[8], xb[8];
      float wa[8], wb[8];
      bool hb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int src = base + ((u0 + u) & (LPR - 1));
        const int32_t a_row = __shfl(ra, src), b_row = __shfl(rb, src);
        wa[u] = __shfl(ca, src);
        wb[u] = __shfl(cb, src);
        const bool ok = u0 + u < m;
        xa[u] = ok ? ld4(out + (int64_t)a_row * D + sub * 4) : f4_zero();
        hb[u] = ok && b_row >= 0;
        xb[u] = hb[u] ? ld4(out + (int64_t)b_row * D + sub * 4) : f4_zero();
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (u0 + u >= m) break;
        gp = f4_fma(wa[u], xa[u], gp);
        if (hb[u]) gp = f4_fma(wb[u], xb[u], gp);
      }
    }
    cnt += m;
    if (m < LPR) break;
  }
  const float4 e = ld4(emb + (int64_t)node * D + sub * 4);
  float re = decay * ((float)cnt / (float)batch);
  if (grad_scale != 1.f) re *= grad_scale;
  st4(seed_p + q * D + sub * 4, f4_div(gp, layer_div));
  st4(seed_e + q * D + sub * 4, f4_scale(re, e));
}

__global__ void seed_reset_kernel(int32_t *slot, const int32_t *keys_sorted, int64_t n) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n) {
    const int32_t k = keys_sorted[q];
    if (k >= 0) slot[k] = -1;
  }
}

// Data-parallel seed exchange.  pack: head positions keep their node id,
// the others get the sentinel n_nodes (sorted last by the merge).
__global__ void seed_pack_kernel(const int32_t *keys_sorted, int64_t n, int32_t sentinel,
                                 int32_t *keys_packed) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  const int32_t k = keys_sorted[q];
  keys_packed[q] = (q == 0 || keys_sorted[q - 1] != k) ? k : sentinel;
}

// merge heads: slot[node] = q for the first position of each node's run;
// sentinel positions become -1 (ignored by reset / accumulate).
__global__ void merge_heads_kernel(int32_t *keys_sorted, int64_t n, int32_t sentinel,
                                   int32_t *slot) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  // Sentinels sort last, so a real key's predecessor is never rewritten
  // concurrently (the sentinel -> -1 rewrite only touches sentinel runs).
  const int32_t k = keys_sorted[q];
  const int32_t prev = q > 0 ? keys_sorted[q - 1] : -2;
  if (k == sentinel) {
    keys_sorted[q] = -1;
    return;
  }
  if (prev != k) slot[k] = (int32_t)q;
}

// merged seed row of a node = sum of its gathered rows in gathered order
// (rank-major: identical on every rank).
template <int D>
__global__ __launch_bounds__(256) void merge_accum_kernel(const int32_t *__restrict__ keys_sorted,
                                                          const int32_t *__restrict__ idx_sorted,
                                                          int64_t n, const float *__restrict__ rows_p,
                                                          const float *__restrict__ rows_e,
                                                          float *seed_p, float *seed_e) {
  constexpr int LPR = D / 4;
  constexpr int G = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int sub = lane % LPR;
  const int64_t q = ((int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * G + lane / LPR;
  if (q >= n) return;
  const int32_t node = keys_sorted[q];
  if (node < 0) return;
  if (q > 0 && keys_sorted[q - 1] == node) return;
  float4 ap = f4_zero(), ae = f4_zero();
  for (int64_t q2 = q; q2 < n && keys_sorted[q2] == node; ++q2) {
    const int64_t r = idx_sorted[q2];
    ap = f4_add(ap, ld4(rows_p + r * D + sub * 4));
    ae = f4_add(ae, ld4(rows_e + r * D + sub * 4));
  }
  st4(seed_p + q * D + sub * 4, ap);
  st4(seed_e + q * D + sub * 4, ae);
}

__global__ void iota_kernel(int32_t *v, int64_t n) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n) v[q] = (int32_t)q;
}

static int end_bit_for(int64_t n_nodes) {
  int b = 1;
  while (b < 31 && ((int64_t)1 << b) < n_nodes) ++b;
  return b;
}

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// The (node, occurrence) sorts: up to kSmallSortMax pairs the library's own
// one / two-launch sort (smallsort.hip: the C2 step's 6 144 seeds in one
// launch instead of the radix sort's six), above it the device library's
// radix sort; both return the stable order.
static int sort_temp_bytes(int64_t n3, int64_t n_nodes, size_t *bytes) {
  if (n3 <= kSmallSortMax) {
    *bytes = small_sort_workspace(n3);
    return MIREC_OK;
  }
  size_t tb = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(
      nullptr, tb, (const int32_t *)nullptr, (int32_t *)nullptr, (const int32_t *)nullptr,
      (int32_t *)nullptr, (int)n3, 0, end_bit_for(n_nodes), (hipStream_t)0);
  if (e != hipSuccess) {
    g_last_hip_error = (int)e;
    return MIREC_ERR_HIP;
  }
  *bytes = tb;
  return MIREC_OK;
}

static hipError_t sort_pairs(void *ws, size_t tb, const int32_t *keys, int32_t *keys_sorted,
                             const int32_t *vals, int32_t *vals_sorted, int64_t n,
                             int64_t n_nodes, hipStream_t st) {
  if (n <= kSmallSortMax)
    return small_sort_pairs(ws, tb, keys, keys_sorted, vals, vals_sorted, n, st);
  return hipcub::DeviceRadixSort::SortPairs(ws, tb, keys, keys_sorted, vals, vals_sorted, (int)n,
                                            0, end_bit_for(n_nodes), st);
}

template <int D>
static int launch_bpr_forward(const float *out, const float *emb, int64_t n_users, int64_t batch,
                              const int32_t *users, const int32_t *pos, const int32_t *neg,
                              float grad_scale, float *coef, float *sp, float *reg,
                              int32_t *keys, int32_t *vals, hipStream_t st) {
  constexpr int G = 64 / (D / 4);
  const int64_t per_block = (int64_t)kWaves * G;
  const int64_t blocks = (batch + per_block - 1) / per_block;
  hipLaunchKernelGGL((bpr_forward_kernel<D>), dim3(blocks), dim3(256), 0, st, out, emb, n_users,
                     batch, users, pos, neg, grad_scale, coef, sp, reg, keys, vals);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

template <int D>
static int launch_seed_accum(const float *out, const float *emb, int64_t n_users, int64_t batch,
                             const int32_t *users, const int32_t *pos, const int32_t *neg,
                             const float *coef, const int32_t *ks, const int32_t *vs, float decay,
                             float grad_scale, float layer_div, float *seed_p, float *seed_e,
                             hipStream_t st) {
  constexpr int G = 64 / (D / 4);
  const int64_t per_block = (int64_t)kWaves * G;
  const int64_t blocks = (3 * batch + per_block - 1) / per_block;
  hipLaunchKernelGGL((seed_accum_kernel<D>), dim3(blocks), dim3(256), 0, st, out, emb, n_users,
                     batch, users, pos, neg, coef, ks, vs, decay, grad_scale, layer_div, seed_p,
                     seed_e);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

}  // namespace mirec

extern "C" int mirec_bpr_forward(const float *out, const float *emb, int64_t n_nodes,
                                 int64_t n_users, int32_t dim, int64_t batch,
                                 const int32_t *users, const int32_t *pos, const int32_t *neg,
                                 float grad_scale, float *coef, float *softplus, float *reg,
                                 int32_t *keys, int32_t *vals, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(out && emb && users && pos && neg && coef && softplus && reg && keys && vals);
  MIREC_CHECK_ARG(batch > 0 && n_users > 0 && n_nodes > n_users);
  MIREC_CHECK_ARG(3 * batch < INT32_MAX && n_nodes < INT32_MAX);
  if (!dim_supported(dim)) return MIREC_ERR_DIM;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (dim) {
#define C(DD) \
  case DD:    \
    return launch_bpr_forward<DD>(out, emb, n_users, batch, users, pos, neg, grad_scale, coef, softplus, reg, keys, vals, st);
    C(4) C(8) C(16) C(32) C(64) C(128) C(256)
#undef C
  }
  return MIREC_ERR_DIM;
}

extern "C" int mirec_bpr_loss(const float *softplus, const float *reg, int64_t batch,
                              float decay, float *loss_out, float *loss_accum,
                              mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(softplus && reg && loss_out && batch > 0);
  hipLaunchKernelGGL(bpr_loss_kernel, dim3(1), dim3(1024), 0,
                     reinterpret_cast<hipStream_t>(stream), softplus, reg, batch, decay, loss_out,
                     loss_accum);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_bpr_seed_workspace(int64_t batch, int64_t n_nodes, size_t *bytes) {
  using namespace mirec;
  MIREC_CHECK_ARG(bytes != nullptr && batch > 0 && n_nodes > 0);
  size_t tb = 0;
  int rc = sort_temp_bytes(3 * batch, n_nodes, &tb);
  if (rc != MIREC_OK) return rc;
  *bytes = align_up(tb) + align_up((size_t)3 * batch * sizeof(int32_t));
  return MIREC_OK;
}

extern "C" int mirec_bpr_seed(const float *out, const float *emb, int64_t n_nodes, int64_t n_users,
                              int32_t dim, int64_t batch, const int32_t *users,
                              const int32_t *pos, const int32_t *neg, const float *coef,
                              const int32_t *keys, const int32_t *vals, float decay,
                              float grad_scale, int32_t n_layers, int32_t *slot, float *seed_p,
                              float *seed_e,
                              int32_t *keys_sorted, void *workspace, size_t workspace_bytes,
                              mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(out && emb && users && pos && neg && coef && keys && vals && slot && seed_p &&
                  seed_e && keys_sorted && workspace);
  MIREC_CHECK_ARG(batch > 0 && n_layers >= 0 && n_nodes > n_users);
  if (!dim_supported(dim)) return MIREC_ERR_DIM;
  const int64_t n3 = 3 * batch;
  size_t tb = 0;
  int rc = sort_temp_bytes(n3, n_nodes, &tb);
  if (rc != MIREC_OK) return rc;
  const size_t need = align_up(tb) + align_up((size_t)n3 * sizeof(int32_t));
  if (workspace_bytes < need) return MIREC_ERR_WORKSPACE;
  char *ws = static_cast<char *>(workspace);
  int32_t *vals_sorted = reinterpret_cast<int32_t *>(ws + align_up(tb));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  size_t tb2 = tb;
  MIREC_HIP(sort_pairs(ws, tb2, keys, keys_sorted, vals, vals_sorted, n3, n_nodes, st));
  hipLaunchKernelGGL(seed_heads_kernel, dim3((n3 + 255) / 256), dim3(256), 0, st, keys_sorted, n3,
                     slot);
  MIREC_LAUNCH_CHECK();
  const float layer_div = (float)(n_layers + 1);
  switch (dim) {
#define C(DD) \
  case DD:    \
    return launch_seed_accum<DD>(out, emb, n_users, batch, users, pos, neg, coef, keys_sorted, vals_sorted, decay, grad_scale, layer_div, seed_p, seed_e, st);
    C(4) C(8) C(16) C(32) C(64) C(128) C(256)
#undef C
  }
  return MIREC_ERR_DIM;
}

extern "C" int mirec_bpr_seed_reset(int32_t *slot, const int32_t *keys_sorted, int64_t n,
                                    mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(slot && keys_sorted && n >= 0);
  if (n == 0) return MIREC_OK;
  hipLaunchKernelGGL(seed_reset_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), slot, keys_sorted, n);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_seed_pack(const int32_t *keys_sorted, int64_t n, int64_t n_nodes,
                               int32_t *keys_packed, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(keys_sorted && keys_packed && n >= 0 && n_nodes > 0 && n_nodes < INT32_MAX);
  if (n == 0) return MIREC_OK;
  hipLaunchKernelGGL(seed_pack_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), keys_sorted, n, (int32_t)n_nodes,
                     keys_packed);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_seed_merge_workspace(int64_t n, int64_t n_nodes, size_t *bytes) {
  using namespace mirec;
  MIREC_CHECK_ARG(bytes && n > 0 && n_nodes > 0 && n < INT32_MAX);
  size_t tb = 0;
  int rc = sort_temp_bytes(n, n_nodes + 1, &tb);
  if (rc != MIREC_OK) return rc;
  *bytes = align_up(tb) + 2 * align_up((size_t)n * sizeof(int32_t));
  return MIREC_OK;
}

template <int D>
static int launch_merge_accum(const int32_t *ks, const int32_t *is, int64_t n, const float *rp,
                              const float *re, float *sp, float *se, hipStream_t st) {
  using namespace mirec;
  constexpr int G = 64 / (D / 4);
  const int64_t per_block = (int64_t)kWaves * G;
  hipLaunchKernelGGL((merge_accum_kernel<D>), dim3((n + per_block - 1) / per_block), dim3(256), 0,
                     st, ks, is, n, rp, re, sp, se);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_seed_merge(const int32_t *keys_packed, const float *rows_p,
                                const float *rows_e, int64_t n, int32_t dim, int64_t n_nodes,
                                int32_t *slot, float *seed_p, float *seed_e,
                                int32_t *keys_sorted, void *workspace, size_t workspace_bytes,
                                mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(keys_packed && rows_p && rows_e && slot && seed_p && seed_e && keys_sorted &&
                  workspace && n > 0 && n < INT32_MAX && n_nodes > 0 && n_nodes < INT32_MAX);
  if (!dim_supported(dim)) return MIREC_ERR_DIM;
  size_t tb = 0;
  int rc = sort_temp_bytes(n, n_nodes + 1, &tb);
  if (rc != MIREC_OK) return rc;
  const size_t need = align_up(tb) + 2 * align_up((size_t)n * sizeof(int32_t));
  if (workspace_bytes < need) return MIREC_ERR_WORKSPACE;
  char *ws = static_cast<char *>(workspace);
  int32_t *idx_in = reinterpret_cast<int32_t *>(ws + align_up(tb));
  int32_t *idx_sorted = reinterpret_cast<int32_t *>(ws + align_up(tb) + align_up(n * 4));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(iota_kernel, dim3((n + 255) / 256), dim3(256), 0, st, idx_in, n);
  MIREC_LAUNCH_CHECK();
  size_t tb2 = tb;
  MIREC_HIP(sort_pairs(ws, tb2, keys_packed, keys_sorted, idx_in, idx_sorted, n, n_nodes + 1, st));
  hipLaunchKernelGGL(merge_heads_kernel, dim3((n + 255) / 256), dim3(256), 0, st, keys_sorted, n,
                     (int32_t)n_nodes, slot);
  MIREC_LAUNCH_CHECK();
  switch (dim) {
#define C(DD) \
  case DD:    \
    return launch_merge_accum<DD>(keys_sorted, idx_sorted, n, rows_p, rows_e, seed_p, seed_e, st);
    C(4) C(8) C(16) C(32) C(64) C(128) C(256)
#undef C
  }
  return MIREC_ERR_DIM;
}

namespace mirec {
// dense[v] = dinv[v] * seed[slot[v]] (or 0 when clearing) for the listed
// nodes v = list[i], i < *count: one LPR-lane group per node, float4.
__global__ __launch_bounds__(256) void seed_dense_kernel(const int32_t *__restrict__ list,
                                                         const int32_t *__restrict__ count,
                                                         const int32_t *__restrict__ slot,
                                                         const float *__restrict__ dinv,
                                                         const float *__restrict__ seed,
                                                         int32_t d4, float *__restrict__ dense,
                                                         int clear) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e = i / d4, c = i - e * d4;
  if (e >= *count) return;
  const int32_t v = list[e];
  float4 x = f4_zero();
  if (!clear) {
    const int32_t r = slot[v];
    if (r >= 0) x = f4_scale(dinv[v], ld4(seed + ((int64_t)r * d4 + c) * 4));
  }
  st4(dense + ((int64_t)v * d4 + c) * 4, x);
}
}  // namespace mirec

extern "C" int mirec_seed_dense(const int32_t *list, const int32_t *count, int64_t cap,
                                const int32_t *slot, const float *dinv, const float *seed,
                                int32_t dim, float *dense, int32_t clear,
                                mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(list && count && dense && cap >= 0 && dim > 0 && dim % 4 == 0);
  MIREC_CHECK_ARG(clear || (slot && dinv && seed));
  if (cap == 0) return MIREC_OK;
  const int64_t tot = cap * (dim / 4);
  hipLaunchKernelGGL(seed_dense_kernel, dim3((tot + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), list, count, slot, dinv, seed,
                     dim / 4, dense, clear);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}
