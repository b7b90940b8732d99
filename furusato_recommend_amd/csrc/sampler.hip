// On-device BPR triple sampler: UniformSample (negative_sample.py:98-134)
// without the host round-trip.  One lane per triple, counter-based RNG
// (splitmix64-seeded xorshift64*: triple t of a call draws from the stream
// (seed, offset + t), so results do not depend on the launch shape).
//
//   u ~ U(users of this shard)       negative_sample.py:107  (redrawn if no positives,
//                                    the reference skips them: :116-117)
//   p = allPos[u][U(0, deg u)]       :119-120  (allPos order = CSR row order)
//     or, with per-user positive probabilities (the sample_pow option,
//     negative_sample.py:53-56: np.random.choice(len(allPos[u]), p=probs[u])),
//     the inverse CDF of the user's row: the first entry whose cumulative
//     probability exceeds a uniform draw (numpy's searchsorted 'right')
//   n ~ U[0, m_items) until n not in allPos[u]   :121-126
#include <algorithm>
#include <thread>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "common.h"

namespace mirec {

// (The RNG and the per-triple draw are __host__ __device__: the host sampler
// mirec_cpu_bpr_sample runs the same streams on CPU threads and returns the
// device sampler's triples bit for bit.)
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct XorShift64Star {
  uint64_t s;
  __host__ __device__ __forceinline__ uint64_t next() {
    s ^= s >> 12;
    s ^= s << 25;
    s ^= s >> 27;
    return s * 0x2545F4914F6CDD1Dull;
  }
  // Uniform integer in [0, n) by 64x64 -> high-64 multiply (Lemire).
  __host__ __device__ __forceinline__ int64_t below(int64_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (int64_t)__umul64hi(next(), (uint64_t)n);
#else
    return (int64_t)(uint64_t)(((unsigned __int128)next() * (uint64_t)n) >> 64);
#endif
  }
  // Uniform double in [0, 1) on the 2^-53 grid (exactly representable).
  __host__ __device__ __forceinline__ double unit() {
    return (double)(next() >> 11) * 0x1p-53;
  }
};

// The positive's entry offset in a user row [beg, beg + deg): uniform, or
// (cdf given: cdf[e - base] is the inclusive cumulative probability of entry
// e within its row, the row's last entry 1) the first entry whose cumulative
// probability exceeds a uniform draw in [0, 1) — an entry of zero
// probability is never chosen.
__host__ __device__ __forceinline__ int64_t draw_positive(XorShift64Star &rng, const double *__restrict__ cdf,
                                                 int64_t base, int64_t beg, int64_t deg) {
  if (cdf == nullptr) return rng.below(deg);
  const double r = rng.unit();
  const double *c = cdf + (beg - base);
  int64_t lo = 0, hi = deg - 1;  // the last entry (cdf 1 > r) always qualifies
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (c[mid] > r) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// Is `node` among the entries [beg, beg + deg) of a user row?  Binary search
// in the sorted copy of the row when the CSR carries one (csr.col_sorted),
// else a scan of the row in edge order.
__host__ __device__ __forceinline__ bool row_has(const int32_t *__restrict__ col,
                                        const int32_t *__restrict__ sorted, int64_t base,
                                        int64_t beg, int64_t deg, int32_t node) {
  if (sorted != nullptr) {
    const int32_t *a = sorted + (beg - base);
    int64_t lo = 0, hi = deg;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (a[mid] < node) lo = mid + 1;
      else hi = mid;
    }
    return lo < deg && a[lo] == node;
  }
  for (int64_t e = 0; e < deg; ++e)
    if (col[beg + e] == node) return true;
  return false;
}

constexpr int kMaxUserTries = 1 << 12;
constexpr int kMaxNegTries = 1 << 16;

// Triple t of a call (its own stream): writes users / pos / neg [t]; false
// if a draw exhausted its retry budget.
__host__ __device__ __forceinline__ bool bpr_sample_one(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const int32_t *__restrict__ sorted, const double *__restrict__ pos_cdf, int64_t n_users,
    int64_t m_items, int64_t t, uint64_t seed, uint64_t offset, int32_t shard, int32_t n_shards,
    int32_t *users, int32_t *pos, int32_t *neg) {
  XorShift64Star rng;
  // Shards get independent streams: (seed, shard) -> key, then (key, offset + t).
  const uint64_t key = splitmix64(seed + 0xD1B54A32D192ED03ull * (uint64_t)shard);
  rng.s = splitmix64(key ^ (offset + (uint64_t)t));
  if (rng.s == 0) rng.s = 0x853C49E6748FEA9Bull;
  const int64_t n_local = (n_users - shard + n_shards - 1) / n_shards;
  int64_t u = 0, beg = 0, deg = 0;
  int tries = 0;
  do {
    u = shard + (int64_t)n_shards * rng.below(n_local);
    beg = rowptr[u];
    deg = rowptr[u + 1] - beg;
  } while (deg == 0 && ++tries < kMaxUserTries);
  if (deg == 0) {
    users[t] = (int32_t)u;
    pos[t] = 0;
    neg[t] = 0;
    return false;
  }
  const int64_t base = rowptr[0];
  const int64_t p = (int64_t)col[beg + draw_positive(rng, pos_cdf, base, beg, deg)] - n_users;
  int64_t n = 0;
  bool ok = false;
  for (int k = 0; k < kMaxNegTries && !ok; ++k) {
    n = rng.below(m_items);
    ok = !row_has(col, sorted, base, beg, deg, (int32_t)(n_users + n));
  }
  users[t] = (int32_t)u;
  pos[t] = (int32_t)p;
  neg[t] = (int32_t)n;
  return ok;
}

__global__ __launch_bounds__(256) void bpr_sample_kernel(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const int32_t *__restrict__ sorted, const double *__restrict__ pos_cdf, int64_t n_users,
    int64_t m_items, int64_t batch, uint64_t seed, uint64_t offset, int32_t shard,
    int32_t n_shards, int32_t *users, int32_t *pos, int32_t *neg, int32_t *err) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= batch) return;
  if (!bpr_sample_one(rowptr, col, sorted, pos_cdf, n_users, m_items, t, seed, offset, shard,
                      n_shards, users, pos, neg))
    err[0] = 1;
}

// ---------------------------------------------------------------------------
// The ddp_lgcn.py epoch sampler (ddp_lgcn.py:33-35, 541-582): n_cand =
// TRAIN_ITERATIVE x trainDataSize candidate users drawn uniformly (users
// without positives are skipped, not redrawn: :567-568), a uniform positive
// each, and a candidate is kept only while its positive item has been kept
// fewer than POSITIVE_NUM_LIMIT times before it in draw order (:571-572) —
// i.e. iff its rank among the earlier candidates with the same item is below
// the cap.  In parallel: candidates are radix-sorted by item (stable, so draw
// order within an item), the rank is the distance to the item run's head
// (a max-scan of head positions), the kept flags are compacted in draw order
// (exclusive sum) and only the kept candidates draw their negative.
struct CandRng {
  XorShift64Star rng;
  __host__ __device__ CandRng(uint64_t seed, uint64_t offset, int32_t shard, int64_t t) {
    const uint64_t key = splitmix64(seed + 0xD1B54A32D192ED03ull * (uint64_t)shard);
    rng.s = splitmix64(key ^ (offset + (uint64_t)t));
    if (rng.s == 0) rng.s = 0x853C49E6748FEA9Bull;
  }
};

// candidate t: user u (its shard), positive item p or -1 (no positives)
__host__ __device__ __forceinline__ void draw_candidate(CandRng &c, const int64_t *__restrict__ rowptr,
                                               const int32_t *__restrict__ col,
                                               const double *__restrict__ pos_cdf, int64_t n_users,
                                               int32_t shard, int32_t n_shards, int64_t &u,
                                               int64_t &p, int64_t &beg, int64_t &deg) {
  const int64_t n_local = (n_users - shard + n_shards - 1) / n_shards;
  u = shard + (int64_t)n_shards * c.rng.below(n_local);
  beg = rowptr[u];
  deg = rowptr[u + 1] - beg;
  p = deg > 0 ? (int64_t)col[beg + draw_positive(c.rng, pos_cdf, rowptr[0], beg, deg)] - n_users
              : -1;
}

__global__ __launch_bounds__(256) void cand_kernel(const int64_t *__restrict__ rowptr,
                                                   const int32_t *__restrict__ col,
                                                   const double *__restrict__ pos_cdf,
                                                   int64_t n_users, int64_t m_items, int64_t n,
                                                   uint64_t seed, uint64_t offset, int32_t shard,
                                                   int32_t n_shards, int32_t *__restrict__ keys,
                                                   int32_t *__restrict__ vals,
                                                   int32_t *__restrict__ cand_u,
                                                   int32_t *__restrict__ cand_p) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  CandRng c(seed, offset, shard, t);
  int64_t u, p, beg, deg;
  draw_candidate(c, rowptr, col, pos_cdf, n_users, shard, n_shards, u, p, beg, deg);
  keys[t] = p >= 0 ? (int32_t)p : (int32_t)m_items;  // skipped users sort last
  vals[t] = (int32_t)t;
  if (cand_u) cand_u[t] = (int32_t)u;
  if (cand_p) cand_p[t] = (int32_t)p;
}

// head position of the item run at each sorted position (max-scan input)
__global__ __launch_bounds__(256) void cand_head_kernel(const int32_t *__restrict__ keys, int64_t n,
                                                        int32_t *__restrict__ head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  head[i] = (i == 0 || keys[i] != keys[i - 1]) ? (int32_t)i : 0;
}

__global__ __launch_bounds__(256) void cand_keep_kernel(const int32_t *__restrict__ keys,
                                                        const int32_t *__restrict__ vals,
                                                        const int32_t *__restrict__ run, int64_t n,
                                                        int32_t m_items, int32_t cap,
                                                        int32_t *__restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flag[vals[i]] = (keys[i] < m_items && i - run[i] < cap) ? 1 : 0;
}

// A kept candidate t redraws its stream (same u, p), then draws its negative,
// and writes the triple at output position o; false if the negative draw
// exhausted its retry budget.
__host__ __device__ __forceinline__ bool emit_candidate(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const int32_t *__restrict__ sorted, const double *__restrict__ pos_cdf, int64_t n_users,
    int64_t m_items, int64_t t, uint64_t seed, uint64_t offset, int32_t shard, int32_t n_shards,
    int64_t o, int32_t *users, int32_t *pos, int32_t *neg) {
  CandRng c(seed, offset, shard, t);  // the same stream: same u, p, then n
  int64_t u, p, beg, deg;
  draw_candidate(c, rowptr, col, pos_cdf, n_users, shard, n_shards, u, p, beg, deg);
  int64_t ng = 0;
  bool ok = false;
  const int64_t base = rowptr[0];
  for (int k = 0; k < kMaxNegTries && !ok; ++k) {
    ng = c.rng.below(m_items);
    ok = !row_has(col, sorted, base, beg, deg, (int32_t)(n_users + ng));
  }
  users[o] = (int32_t)u;
  pos[o] = (int32_t)p;
  neg[o] = (int32_t)ng;
  return ok;
}

__global__ __launch_bounds__(256) void cand_emit_kernel(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const int32_t *__restrict__ sorted, const double *__restrict__ pos_cdf, int64_t n_users,
    int64_t m_items, int64_t n, uint64_t seed, uint64_t offset, int32_t shard, int32_t n_shards,
    const int32_t *__restrict__ flag, const int32_t *__restrict__ at, int32_t *__restrict__ users,
    int32_t *__restrict__ pos, int32_t *__restrict__ neg, int32_t *__restrict__ count,
    int32_t *__restrict__ err) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  if (t == n - 1) count[0] = at[t] + flag[t];
  if (!flag[t]) return;
  if (!emit_candidate(rowptr, col, sorted, pos_cdf, n_users, m_items, t, seed, offset, shard,
                      n_shards, at[t], users, pos, neg))
    err[0] = 1;
}

struct MaxOp {
  __device__ __forceinline__ int32_t operator()(int32_t a, int32_t b) const {
    return a > b ? a : b;
  }
};

struct CapLayout {
  size_t keys_in, keys_out, vals_in, vals_out, run, flag, at, tmp, tmp_bytes, total;
  int end_bit;
};

static int cap_layout(int64_t n, int64_t m_items, CapLayout *L) {
  MIREC_CHECK_ARG(n >= 0 && n < ((int64_t)1 << 31) && m_items > 0 && m_items < ((int64_t)1 << 30));
  const auto up = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t seg = up(sizeof(int32_t) * std::max<int64_t>(n, 1));
  L->keys_in = 0;
  L->keys_out = seg;
  L->vals_in = 2 * seg;
  L->vals_out = 3 * seg;
  L->run = 4 * seg;
  L->flag = 5 * seg;
  L->at = 6 * seg;
  L->tmp = 7 * seg;
  int bits = 1;
  while (bits < 31 && ((int64_t)1 << bits) <= m_items) ++bits;
  L->end_bit = bits;
  const int nn = (int)std::max<int64_t>(n, 1);
  size_t a = 0, b = 0, c = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (int32_t *)nullptr, (int32_t *)nullptr,
                                           (int32_t *)nullptr, (int32_t *)nullptr, nn, 0, bits);
  (void)hipcub::DeviceScan::InclusiveScan(nullptr, b, (int32_t *)nullptr, (int32_t *)nullptr,
                                          MaxOp(), nn);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (int32_t *)nullptr, (int32_t *)nullptr, nn);
  L->tmp_bytes = std::max(a, std::max(b, c));
  L->total = L->tmp + up(L->tmp_bytes);
  return MIREC_OK;
}

}  // namespace mirec

extern "C" int mirec_bpr_sample_capped_workspace(int64_t n_candidates, int64_t m_items,
                                                 size_t *bytes) {
  using namespace mirec;
  MIREC_CHECK_ARG(bytes);
  CapLayout L;
  const int rc = cap_layout(n_candidates, m_items, &L);
  if (rc != MIREC_OK) return rc;
  *bytes = L.total;
  return MIREC_OK;
}

extern "C" int mirec_bpr_sample_capped_ex(const mirec_csr_t *csr, const double *pos_cdf,
                                          int64_t n_users, int64_t m_items,
                                       int64_t n_candidates, int32_t cap, uint64_t seed,
                                       uint64_t offset, int32_t shard, int32_t n_shards,
                                       int32_t *users, int32_t *pos, int32_t *neg,
                                       int32_t *count, int32_t *err, int32_t *cand_u,
                                       int32_t *cand_p, void *workspace, size_t workspace_bytes,
                                       mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(csr && csr->rowptr && csr->col && users && pos && neg && count && err);
  MIREC_CHECK_ARG(n_users > 0 && m_items > 0 && cap >= 0);
  MIREC_CHECK_ARG(n_shards >= 1 && shard >= 0 && shard < n_shards && shard < n_users);
  MIREC_CHECK_ARG(csr->n_rows >= n_users + m_items);
  CapLayout L;
  const int rc = cap_layout(n_candidates, m_items, &L);
  if (rc != MIREC_OK) return rc;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n_candidates == 0) {
    MIREC_HIP(hipMemsetAsync(count, 0, sizeof(int32_t), st));
    return MIREC_OK;
  }
  MIREC_CHECK_ARG(workspace);
  if (workspace_bytes < L.total) return MIREC_ERR_WORKSPACE;
  char *ws = static_cast<char *>(workspace);
  int32_t *keys_in = reinterpret_cast<int32_t *>(ws + L.keys_in);
  int32_t *keys_out = reinterpret_cast<int32_t *>(ws + L.keys_out);
  int32_t *vals_in = reinterpret_cast<int32_t *>(ws + L.vals_in);
  int32_t *vals_out = reinterpret_cast<int32_t *>(ws + L.vals_out);
  int32_t *run = reinterpret_cast<int32_t *>(ws + L.run);
  int32_t *flag = reinterpret_cast<int32_t *>(ws + L.flag);
  int32_t *at = reinterpret_cast<int32_t *>(ws + L.at);
  void *tmp = ws + L.tmp;
  size_t tb = L.tmp_bytes;
  const int n = (int)n_candidates;
  const dim3 grid((unsigned)((n_candidates + 255) / 256));
  const int32_t *sorted = csr->n_sorted >= n_users ? csr->col_sorted : nullptr;
  hipLaunchKernelGGL(cand_kernel, grid, dim3(256), 0, st, csr->rowptr, csr->col, pos_cdf, n_users,
                     m_items,
                     n_candidates, seed, offset, shard, n_shards, keys_in, vals_in, cand_u,
                     cand_p);
  MIREC_LAUNCH_CHECK();
  MIREC_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys_in, keys_out, vals_in, vals_out, n,
                                               0, L.end_bit, st));
  hipLaunchKernelGGL(cand_head_kernel, grid, dim3(256), 0, st, keys_out, n_candidates, keys_in);
  MIREC_LAUNCH_CHECK();
  tb = L.tmp_bytes;
  MIREC_HIP(hipcub::DeviceScan::InclusiveScan(tmp, tb, keys_in, run, MaxOp(), n, st));
  hipLaunchKernelGGL(cand_keep_kernel, grid, dim3(256), 0, st, keys_out, vals_out, run,
                     n_candidates, (int32_t)m_items, cap, flag);
  MIREC_LAUNCH_CHECK();
  tb = L.tmp_bytes;
  MIREC_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, flag, at, n, st));
  hipLaunchKernelGGL(cand_emit_kernel, grid, dim3(256), 0, st, csr->rowptr, csr->col, sorted,
                     pos_cdf, n_users, m_items, n_candidates, seed, offset, shard, n_shards, flag, at,
                     users, pos, neg, count, err);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_bpr_sample_capped(const mirec_csr_t *csr, int64_t n_users, int64_t m_items,
                                       int64_t n_candidates, int32_t cap, uint64_t seed,
                                       uint64_t offset, int32_t shard, int32_t n_shards,
                                       int32_t *users, int32_t *pos, int32_t *neg,
                                       int32_t *count, int32_t *err, int32_t *cand_u,
                                       int32_t *cand_p, void *workspace, size_t workspace_bytes,
                                       mirec_stream_t stream) {
  return mirec_bpr_sample_capped_ex(csr, nullptr, n_users, m_items, n_candidates, cap, seed,
                                    offset, shard, n_shards, users, pos, neg, count, err, cand_u,
                                    cand_p, workspace, workspace_bytes, stream);
}

extern "C" int mirec_bpr_sample_ex(const mirec_csr_t *csr, const double *pos_cdf, int64_t n_users,
                                   int64_t m_items, int64_t batch, uint64_t seed, uint64_t offset,
                                   int32_t shard, int32_t n_shards, int32_t *users, int32_t *pos,
                                   int32_t *neg, int32_t *err, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(csr && csr->rowptr && csr->col && users && pos && neg && err);
  MIREC_CHECK_ARG(n_users > 0 && m_items > 0 && batch >= 0);
  MIREC_CHECK_ARG(n_shards >= 1 && shard >= 0 && shard < n_shards && shard < n_users);
  MIREC_CHECK_ARG(csr->n_rows >= n_users + m_items);
  if (batch == 0) return MIREC_OK;
  hipLaunchKernelGGL(bpr_sample_kernel, dim3((batch + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), csr->rowptr, csr->col,
                     csr->n_sorted >= n_users ? csr->col_sorted : nullptr, pos_cdf, n_users,
                     m_items, batch, seed, offset, shard, n_shards, users, pos, neg, err);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_bpr_sample(const mirec_csr_t *csr, int64_t n_users, int64_t m_items,
                                int64_t batch, uint64_t seed, uint64_t offset, int32_t shard,
                                int32_t n_shards, int32_t *users, int32_t *pos, int32_t *neg,
                                int32_t *err, mirec_stream_t stream) {
  return mirec_bpr_sample_ex(csr, nullptr, n_users, m_items, batch, seed, offset, shard, n_shards,
                             users, pos, neg, err, stream);
}

// The same sampler on the host (configuration C1, "CPU single-process":
// BASELINE configs[0]; model/MF.py on a CPU device): host arrays, the same
// streams, so the triples equal mirec_bpr_sample's bit for bit.  Threads
// take contiguous blocks of triples.
extern "C" int mirec_cpu_bpr_sample(const int64_t *rowptr, const int32_t *col,
                                    const int32_t *col_sorted, const double *pos_cdf,
                                    int64_t n_users, int64_t m_items, int64_t batch,
                                    uint64_t seed, uint64_t offset, int32_t shard,
                                    int32_t n_shards, int32_t *users, int32_t *pos, int32_t *neg,
                                    int32_t *err, int32_t n_threads) {
  using namespace mirec;
  MIREC_CHECK_ARG(rowptr && col && users && pos && neg && err);
  MIREC_CHECK_ARG(n_users > 0 && m_items > 0 && batch >= 0);
  MIREC_CHECK_ARG(n_shards >= 1 && shard >= 0 && shard < n_shards && shard < n_users);
  if (batch == 0) return MIREC_OK;
  const int nt = (int)std::max<int64_t>(
      1, std::min<int64_t>(std::min<int64_t>(n_threads > 0 ? n_threads : 1, 64),
                           (batch + 4095) / 4096));
  std::vector<int> bad(nt, 0);
  auto work = [&](int w) {
    const int64_t a = batch * w / nt, b = batch * (w + 1) / nt;
    for (int64_t t = a; t < b; ++t)
      if (!bpr_sample_one(rowptr, col, col_sorted, pos_cdf, n_users, m_items, t, seed, offset,
                          shard, n_shards, users, pos, neg))
        bad[w] = 1;
  };
  std::vector<std::thread> th;
  for (int w = 1; w < nt; ++w) th.emplace_back(work, w);
  work(0);
  for (auto &x : th) x.join();
  for (int w = 0; w < nt; ++w)
    if (bad[w]) err[0] = 1;
  return MIREC_OK;
}

// The capped epoch sampler on the host (a CPU model under train_dp /
// Trainer(sampler="ddp_capped")): the device sampler's candidate streams, so
// the kept triples equal mirec_bpr_sample_capped_ex's bit for bit.  The
// candidates are drawn on n_threads threads, the keep decision is the
// reference's own sequential count per item (ddp_lgcn.py:571-572), and the
// kept candidates draw their negatives on the threads again.
extern "C" int mirec_cpu_bpr_sample_capped(const int64_t *rowptr, const int32_t *col,
                                           const int32_t *col_sorted, const double *pos_cdf,
                                           int64_t n_users, int64_t m_items,
                                           int64_t n_candidates, int32_t cap, uint64_t seed,
                                           uint64_t offset, int32_t shard, int32_t n_shards,
                                           int32_t *users, int32_t *pos, int32_t *neg,
                                           int32_t *count, int32_t *err, int32_t *cand_u,
                                           int32_t *cand_p, int32_t n_threads) {
  using namespace mirec;
  MIREC_CHECK_ARG(rowptr && col && users && pos && neg && count && err);
  MIREC_CHECK_ARG(n_users > 0 && m_items > 0 && cap >= 0 && n_candidates >= 0);
  MIREC_CHECK_ARG(n_candidates < ((int64_t)1 << 31));
  MIREC_CHECK_ARG(n_shards >= 1 && shard >= 0 && shard < n_shards && shard < n_users);
  const int64_t n = n_candidates;
  const int nt = (int)std::max<int64_t>(
      1, std::min<int64_t>(std::min<int64_t>(n_threads > 0 ? n_threads : 1, 64), (n + 4095) / 4096));
  auto parallel = [&](auto &&f) {
    std::vector<std::thread> th;
    for (int w = 1; w < nt; ++w) th.emplace_back([&, w] { f(n * w / nt, n * (w + 1) / nt, w); });
    f(0, n / nt, 0);
    for (auto &x : th) x.join();
  };
  std::vector<int32_t> item(n);
  parallel([&](int64_t a, int64_t b, int) {
    for (int64_t t = a; t < b; ++t) {
      CandRng c(seed, offset, shard, t);
      int64_t u, p, beg, deg;
      draw_candidate(c, rowptr, col, pos_cdf, n_users, shard, n_shards, u, p, beg, deg);
      item[t] = (int32_t)p;
      if (cand_u) cand_u[t] = (int32_t)u;
      if (cand_p) cand_p[t] = (int32_t)p;
    }
  });
  // kept iff fewer than cap earlier candidates with the same item were kept;
  // at[t] = the output position of a kept candidate, -1 otherwise
  std::vector<int32_t> seen(m_items, 0);
  std::vector<int64_t> at(n);
  int64_t k = 0;
  for (int64_t t = 0; t < n; ++t) {
    const int32_t p = item[t];
    at[t] = (p >= 0 && seen[p] < cap) ? k++ : -1;
    if (p >= 0 && seen[p] < cap) ++seen[p];
  }
  std::vector<int> bad(nt, 0);
  parallel([&](int64_t a, int64_t b, int w) {
    for (int64_t t = a; t < b; ++t)
      if (at[t] >= 0 && !emit_candidate(rowptr, col, col_sorted, pos_cdf, n_users, m_items, t,
                                        seed, offset, shard, n_shards, at[t], users, pos, neg))
        bad[w] = 1;
  });
  count[0] = (int32_t)k;
  for (int w = 0; w < nt; ++w)
    if (bad[w]) err[0] = 1;
  return MIREC_OK;
}
