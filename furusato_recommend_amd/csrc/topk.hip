// Evaluation top-k (Trainer.test, trainer.py:130-138): for each evaluated
// user b, the train positives of rating row b are set to -1024 (the user's
// CSR row, trainer.py:132-137) and the k best items are selected
// (torch.topk, :138).  The rating rows come from a library GEMM
// (users_emb · items_embᵀ, model/lgcn.py:124).
//
// One wave per user: the 64 lanes scan the row with coalesced loads, each
// keeping a sorted register top-k (static indexing, branch-free bubble
// insert, taken only when a score beats the lane's current k-th); the 64
// lane lists are then merged pairwise in LDS (6 rounds).  Order: score
// descending, ties to the lower item id (deterministic).
#include "common.h"

namespace mirec {

// Bubble (v, j) into the sorted list; (thr, thr_i) track entry k-1 (the
// current k-th best) so no register array is ever indexed dynamically.
template <int KMAX>
__device__ __forceinline__ void insert_sorted(float (&vals)[KMAX], int (&idxs)[KMAX], int k,
                                              float v, int j, float &thr, int &thr_i) {
  float cv = v;
  int ci = j;
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    if (i < k) {
      const bool sw = cv > vals[i] || (cv == vals[i] && ci < idxs[i]);
      const float tv = vals[i];
      const int ti = idxs[i];
      vals[i] = sw ? cv : tv;
      idxs[i] = sw ? ci : ti;
      cv = sw ? tv : cv;
      ci = sw ? ti : ci;
    }
    if (i == k - 1) {
      thr = vals[i];
      thr_i = idxs[i];
    }
  }
}

__device__ __forceinline__ bool better(float a, int ia, float b, int ib) {
  return a > b || (a == b && ia < ib);
}

template <int KMAX>
__global__ __launch_bounds__(64) void topk_masked_kernel(
    float *__restrict__ scores, int64_t n_eval, int64_t m_items, const int32_t *__restrict__ users,
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col, int64_t n_users, int k,
    int32_t *__restrict__ topk_idx, float *__restrict__ topk_val) {
  __shared__ float s_val[64 * KMAX];
  __shared__ int s_idx[64 * KMAX];
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  if (b >= n_eval) return;
  float *row = scores + b * m_items;
  // 1. mask the train positives (rating[exclude] = -(1 << 10))
  if (rowptr != nullptr) {
    const int64_t u = users[b];
    for (int64_t e = rowptr[u] + lane; e < rowptr[u + 1]; e += 64) {
      const int64_t it = (int64_t)col[e] - n_users;
      if (it >= 0 && it < m_items) row[it] = -1024.f;
    }
    __threadfence_block();
    __syncthreads();
  }
  // 2. per-lane top-k over a strided scan
  float vals[KMAX];
  int idxs[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    vals[i] = -INFINITY;
    idxs[i] = INT_MAX;
  }
  float thr = -INFINITY;
  int thr_i = INT_MAX;
  // Coalesced 4-B loads, 4 per lane in flight; one insertion site.
  for (int64_t j0 = lane; j0 < m_items; j0 += 256) {
    float v[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int64_t j = j0 + 64 * t;
      v[t] = j < m_items ? row[j] : -INFINITY;
    }
    if (v[0] >= thr || v[1] >= thr || v[2] >= thr || v[3] >= thr) {
#pragma unroll 1
      for (int t = 0; t < 4; ++t) {
        const float x = t == 0 ? v[0] : (t == 1 ? v[1] : (t == 2 ? v[2] : v[3]));
        const int j = (int)(j0 + 64 * t);
        if (j < m_items && better(x, j, thr, thr_i))
          insert_sorted<KMAX>(vals, idxs, k, x, j, thr, thr_i);
      }
    }
  }
  // 3. pairwise merges in LDS: 64 -> 32 -> ... -> 1 lists
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    s_val[lane * KMAX + i] = vals[i];
    s_idx[lane * KMAX + i] = idxs[i];
  }
  __syncthreads();
#pragma unroll 1
  for (int active = 32; active >= 1; active >>= 1) {
    float ov[KMAX];
    int oi[KMAX];
    if (lane < active) {
      const float *av = s_val + lane * KMAX, *bv = s_val + (lane + active) * KMAX;
      const int *ai = s_idx + lane * KMAX, *bi = s_idx + (lane + active) * KMAX;
      int pa = 0, pb = 0;
#pragma unroll
      for (int i = 0; i < KMAX; ++i) {
        if (i < k) {
          const bool ta = better(av[pa], ai[pa], bv[pb], bi[pb]);
          ov[i] = ta ? av[pa] : bv[pb];
          oi[i] = ta ? ai[pa] : bi[pb];
          pa += ta ? 1 : 0;
          pb += ta ? 0 : 1;
        }
      }
    }
    __syncthreads();
    if (lane < active) {
#pragma unroll
      for (int i = 0; i < KMAX; ++i)
        if (i < k) {
          s_val[lane * KMAX + i] = ov[i];
          s_idx[lane * KMAX + i] = oi[i];
        }
    }
    __syncthreads();
  }
  for (int i = lane; i < k; i += 64) {
    topk_idx[b * k + i] = s_idx[i];
    if (topk_val != nullptr) topk_val[b * k + i] = s_val[i];
  }
}

}  // namespace mirec

extern "C" int mirec_topk_masked(float *scores, int64_t n_eval, int64_t m_items,
                                 const int32_t *users, const mirec_csr_t *csr, int64_t n_users,
                                 int32_t k, int32_t *topk_idx, float *topk_val,
                                 mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(scores && topk_idx && n_eval >= 0 && m_items > 0 && k >= 1 && k <= 64);
  MIREC_CHECK_ARG(k <= m_items && m_items < INT32_MAX);
  MIREC_CHECK_ARG(csr == nullptr || (users && csr->rowptr && csr->col));
  if (n_eval == 0) return MIREC_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t *rp = csr ? csr->rowptr : nullptr;
  const int32_t *cl = csr ? csr->col : nullptr;
  // (a KMAX=32 instantiation spills on ROCm 7.2; 64 fits in 145 VGPRs)
  hipLaunchKernelGGL((topk_masked_kernel<64>), dim3(n_eval), dim3(64), 0, st, scores, n_eval,
                     m_items, users, rp, cl, n_users, (int)k, topk_idx, topk_val);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}
