// On-device BPR triple sampler: UniformSample (negative_sample.py:98-134)
// without the host round-trip.  One lane per triple, counter-based RNG
// (splitmix64-seeded xorshift64*: triple t of a call draws from the stream
// (seed, offset + t), so results do not depend on the launch shape).
//
//   u ~ U(users of this shard)       negative_sample.py:107  (redrawn if no positives,
//                                    the reference skips them: :116-117)
//   p = allPos[u][U(0, deg u)]       :119-120  (allPos order = CSR row order)
//   n ~ U[0, m_items) until n not in allPos[u]   :121-126
#include "common.h"

namespace mirec {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct XorShift64Star {
  uint64_t s;
  __device__ __forceinline__ uint64_t next() {
    s ^= s >> 12;
    s ^= s << 25;
    s ^= s >> 27;
    return s * 0x2545F4914F6CDD1Dull;
  }
  // Uniform integer in [0, n) by 64x64 -> high-64 multiply (Lemire).
  __device__ __forceinline__ int64_t below(int64_t n) {
    return (int64_t)__umul64hi(next(), (uint64_t)n);
  }
};

constexpr int kMaxUserTries = 1 << 12;
constexpr int kMaxNegTries = 1 << 16;

__global__ __launch_bounds__(256) void bpr_sample_kernel(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col, int64_t n_users,
    int64_t m_items, int64_t batch, uint64_t seed, uint64_t offset, int32_t shard,
    int32_t n_shards, int32_t *users, int32_t *pos, int32_t *neg, int32_t *err) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= batch) return;
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
    err[0] = 1;
    users[t] = (int32_t)u;
    pos[t] = 0;
    neg[t] = 0;
    return;
  }
  const int64_t p = (int64_t)col[beg + rng.below(deg)] - n_users;
  int64_t n = 0;
  bool ok = false;
  for (int k = 0; k < kMaxNegTries && !ok; ++k) {
    n = rng.below(m_items);
    const int32_t node = (int32_t)(n_users + n);
    ok = true;
    for (int64_t e = 0; e < deg; ++e) {
      if (col[beg + e] == node) {
        ok = false;
        break;
      }
    }
  }
  if (!ok) err[0] = 1;
  users[t] = (int32_t)u;
  pos[t] = (int32_t)p;
  neg[t] = (int32_t)n;
}

}  // namespace mirec

extern "C" int mirec_bpr_sample(const mirec_csr_t *csr, int64_t n_users, int64_t m_items,
                                int64_t batch, uint64_t seed, uint64_t offset, int32_t shard,
                                int32_t n_shards, int32_t *users, int32_t *pos, int32_t *neg,
                                int32_t *err, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(csr && csr->rowptr && csr->col && users && pos && neg && err);
  MIREC_CHECK_ARG(n_users > 0 && m_items > 0 && batch >= 0);
  MIREC_CHECK_ARG(n_shards >= 1 && shard >= 0 && shard < n_shards && shard < n_users);
  MIREC_CHECK_ARG(csr->n_rows >= n_users + m_items);
  if (batch == 0) return MIREC_OK;
  hipLaunchKernelGGL(bpr_sample_kernel, dim3((batch + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), csr->rowptr, csr->col, n_users,
                     m_items, batch, seed, offset, shard, n_shards, users, pos, neg, err);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}
