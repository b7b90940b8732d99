// Stable counting sort of (int32 key, int32 value) pairs whose keys are dense
// ids in [0, nk): the key sort of the table-gradient sums (tablegrad.hip) —
// GraphSAGE's id table at C3 (1.7 M entries over 1.1 M rows) and SASRec's item
// table at C4 (63 K entries over 100 K items); reference step:
// graphsage.py:311-324 / sasrec.py:437-474 (the embedding gradients those
// sums form).  It replaces the device library's radix sort there: the keys
// are row ids, so one counting pass and one scatter place every entry, and a
// radix sort's per-digit passes over all 21 key bits are not needed.
//
// Order.  The result is the stable order: equal keys in input order, bit for
// bit what a stable radix sort returns (so every sum downstream keeps its
// entry order and its bits).  The scatter's slot within a bucket comes from
// an atomic and is NOT deterministic; the order is restored per bucket class:
//   small  (c <= 32 entries): each entry counts the bucket's entry indices
//          below its own (<= 32 reads) — its rank;
//   mid    (32 < c <= mid_max, mid_max >= 1024): one workgroup per bucket
//          stages the indices in LDS and ranks them the same way;
//   big    (c > mid_max; at most n / mid_max buckets): no atomics at all.
//          Each tile of the input counts its big entries per bucket
//          (order-free LDS counts), a wave per bucket scans the counts over
//          the tiles, and each tile places its big entries in input order
//          (ballots per 64 entries, running per-bucket counters in LDS).
// Same-address contention is bounded: the counting pass sums each tile's
// keys in an LDS hash table first (one global atomic per distinct key per
// 4096 entries, so a hub id of 10^5 entries costs ~25 atomics), and the
// scatter's returning atomics touch small / mid buckets only (<= mid_max per
// address).
//
// Launches: zero, count, scan-reduce, scan-apply, scatter, big-scan, finish
// (small + mid), big-place — plain kernels on the caller's stream: no host
// synchronisation and no memset / memcpy nodes, so a captured HIP graph
// replays it (the table-gradient sums of the captured SASRec step).
#include "common.h"
#include "keysort.h"

namespace mirec {
namespace {

constexpr int kT = 256;                 // threads per workgroup (4 waves)
constexpr int kCountPer = 16;           // entries per thread in the count pass
constexpr int kCountTile = kT * kCountPer;
constexpr int kHashBits = 13;           // LDS hash slots = 2 x the tile
constexpr int kHash = 1 << kHashBits;
constexpr int kScanPer = 32;            // keys per thread in the scans
constexpr int kScanBlock = kT * kScanPer;
constexpr int kSmall = 32;              // small-bucket bound
constexpr int kMaxBigTiles = 1024;
constexpr int kStage = 2048;            // big-place staging chunk (entries)

struct KsLayout {
  int64_t n;
  int32_t nk, nk_pad, nblk, mid_max, mid_cap, big_cap, big_tile, n_big_tiles;
  size_t cnt, off, part, ctr, mid, tmp, mat, total;
};

size_t up256(size_t b) { return (b + 255) / 256 * 256; }

void ks_layout(int64_t n, int32_t nk, KsLayout *L) {
  L->n = n;
  L->nk = nk;
  L->nblk = (int32_t)(((int64_t)nk + kScanBlock - 1) / kScanBlock);
  L->nk_pad = L->nblk * kScanBlock;
  // mid_max >= n / 16000 keeps the big buckets (<= n / (mid_max + 1) + 1) and
  // a mid bucket (<= mid_max) inside one 64 KB LDS table each
  L->mid_max = (int32_t)std::max<int64_t>(1024, (n + 15999) / 16000);
  L->mid_cap = (int32_t)(n / (kSmall + 1) + 1);
  L->big_cap = (int32_t)(n / ((int64_t)L->mid_max + 1) + 1);
  const int64_t bt = std::max<int64_t>(4096, ((n + kMaxBigTiles - 1) / kMaxBigTiles + 255) / 256 * 256);
  L->big_tile = (int32_t)bt;
  L->n_big_tiles = (int32_t)std::max<int64_t>(1, (n + bt - 1) / bt);
  size_t o = 0;
  L->cnt = o;
  o += up256(4 * (size_t)L->nk_pad);
  L->off = o;
  o += up256(4 * ((size_t)L->nk_pad + 1));
  L->part = o;
  o += up256(4 * 3 * (size_t)L->nblk);
  L->ctr = o;
  o += 256;
  L->mid = o;
  o += up256(4 * (size_t)L->mid_cap);
  L->tmp = o;
  o += up256(4 * (size_t)std::max<int64_t>(n, 1));
  L->mat = o;
  o += up256(4 * (size_t)L->big_cap * L->n_big_tiles);
  L->total = o;
}

__device__ __forceinline__ int32_t clamp_key(int32_t k, int32_t nk) {
  return (uint32_t)k < (uint32_t)nk ? k : nk - 1;
}

// ---- block reductions / scans over 256 threads (3 components) ----
__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int u = __shfl_up(v, d);
    if (lane >= d) v += u;
  }
  return v;
}

// exclusive scan of (x, y, z) over the block; *tot = the block totals
__device__ __forceinline__ int3 block_excl_scan3(int3 v, int3 *tot) {
  __shared__ int3 wsum[kT / 64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int3 inc = make_int3(wave_incl_scan(v.x), wave_incl_scan(v.y), wave_incl_scan(v.z));
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int3 pre = make_int3(0, 0, 0), all = make_int3(0, 0, 0);
#pragma unroll
  for (int q = 0; q < kT / 64; ++q) {
    const int3 s = wsum[q];
    if (q < w) pre = make_int3(pre.x + s.x, pre.y + s.y, pre.z + s.z);
    all = make_int3(all.x + s.x, all.y + s.y, all.z + s.z);
  }
  __syncthreads();
  *tot = all;
  return make_int3(pre.x + inc.x - v.x, pre.y + inc.y - v.y, pre.z + inc.z - v.z);
}

__device__ __forceinline__ int3 block_sum3(int3 v) {
  int3 t;
  (void)block_excl_scan3(v, &t);
  return t;
}

// ---- 0: zero the counts (every call: the workspace may be fresh) ----
__global__ __launch_bounds__(kT) void ks_zero_kernel(int4 *__restrict__ cnt4, int64_t n4,
                                                     int32_t *__restrict__ ctr) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  for (int64_t j = i; j < n4; j += (int64_t)gridDim.x * kT) cnt4[j] = make_int4(0, 0, 0, 0);
  if (i < 4) ctr[i] = 0;
}

// ---- 1: bucket counts; a tile's keys summed in an LDS hash table first ----
__global__ __launch_bounds__(kT) void ks_count_kernel(const int32_t *__restrict__ keys, int64_t n,
                                                      int32_t nk, int32_t *__restrict__ cnt) {
  __shared__ int32_t hk[kHash];
  __shared__ int32_t hc[kHash];
  for (int s = threadIdx.x; s < kHash; s += kT) {
    hk[s] = -1;
    hc[s] = 0;
  }
  const int64_t base = (int64_t)blockIdx.x * kCountTile + threadIdx.x;
  int32_t k[kCountPer];
#pragma unroll
  for (int u = 0; u < kCountPer; ++u) {
    const int64_t i = base + (int64_t)u * kT;
    k[u] = i < n ? clamp_key(keys[i], nk) : -1;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kCountPer; ++u) {
    if (k[u] < 0) continue;
    uint32_t h = ((uint32_t)k[u] * 2654435761u) >> (32 - kHashBits);
    while (true) {  // at most kCountTile keys in kHash slots: a free slot exists
      const int32_t old = atomicCAS(&hk[h], -1, k[u]);
      if (old == -1 || old == k[u]) {
        atomicAdd(&hc[h], 1);
        break;
      }
      h = (h + 1) & (kHash - 1);
    }
  }
  __syncthreads();
  for (int s = threadIdx.x; s < kHash; s += kT) {
    const int32_t key = hk[s];
    if (key >= 0) atomicAdd(&cnt[key], hc[s]);
  }
}

// (entries, mid buckets, big buckets) of one bucket count
__device__ __forceinline__ int3 classify(int32_t c, int32_t mid_max) {
  return make_int3(c, (c > kSmall && c <= mid_max) ? 1 : 0, c > mid_max ? 1 : 0);
}

// ---- 2a: per scan block (8192 buckets) totals ----
__global__ __launch_bounds__(kT) void ks_scan_reduce_kernel(const int32_t *__restrict__ cnt,
                                                            int32_t mid_max,
                                                            int3 *__restrict__ part) {
  const int32_t *c = cnt + (int64_t)blockIdx.x * kScanBlock;
  int3 s = make_int3(0, 0, 0);
#pragma unroll 8
  for (int u = 0; u < kScanPer; ++u) {
    const int3 q = classify(c[u * kT + threadIdx.x], mid_max);
    s = make_int3(s.x + q.x, s.y + q.y, s.z + q.z);
  }
  const int3 t = block_sum3(s);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// ---- 2b: bucket starts, the mid-bucket list, big-bucket slots ----
// off[k] = entries in buckets < k; mid buckets listed in key order; a big
// bucket's count becomes -(slot + 1) (the scatter leaves those alone).
__global__ __launch_bounds__(kT) void ks_scan_apply_kernel(
    int32_t *__restrict__ cnt, int32_t mid_max, const int3 *__restrict__ part, int32_t nblk,
    int32_t *__restrict__ off, int32_t *__restrict__ mid, int32_t *__restrict__ ctr) {
  const int b = blockIdx.x;
  int3 p = make_int3(0, 0, 0);
  for (int j = threadIdx.x; j < b; j += kT) {
    const int3 q = part[j];
    p = make_int3(p.x + q.x, p.y + q.y, p.z + q.z);
  }
  const int3 pre = block_sum3(p);
  const int64_t k0 = (int64_t)b * kScanBlock + (int64_t)threadIdx.x * kScanPer;
  int32_t c[kScanPer];
#pragma unroll
  for (int u = 0; u < kScanPer / 4; ++u) {
    const int4 q = reinterpret_cast<const int4 *>(cnt + k0)[u];
    c[4 * u] = q.x;
    c[4 * u + 1] = q.y;
    c[4 * u + 2] = q.z;
    c[4 * u + 3] = q.w;
  }
  int3 s = make_int3(0, 0, 0);
#pragma unroll
  for (int u = 0; u < kScanPer; ++u) {
    const int3 q = classify(c[u], mid_max);
    s = make_int3(s.x + q.x, s.y + q.y, s.z + q.z);
  }
  int3 tot;
  const int3 ex = block_excl_scan3(s, &tot);
  int run = pre.x + ex.x, nm = pre.y + ex.y, nb = pre.z + ex.z;
#pragma unroll
  for (int u = 0; u < kScanPer / 4; ++u) {
    int4 o;
    o.x = run;
    run += c[4 * u];
    o.y = run;
    run += c[4 * u + 1];
    o.z = run;
    run += c[4 * u + 2];
    o.w = run;
    run += c[4 * u + 3];
    reinterpret_cast<int4 *>(off + k0)[u] = o;
  }
#pragma unroll
  for (int u = 0; u < kScanPer; ++u) {
    const int3 q = classify(c[u], mid_max);
    if (q.y) mid[nm++] = (int32_t)(k0 + u);
    if (q.z) cnt[k0 + u] = -(nb++) - 1;
  }
  if (b == nblk - 1 && threadIdx.x == kT - 1) {
    off[k0 + kScanPer] = run;  // = n: the padded buckets past nk are empty
    ctr[0] = pre.y + tot.y;
    ctr[1] = pre.z + tot.z;
  }
}

// ---- 3: scatter small / mid entries (slot from a returning atomic, order
// fixed in 5), count big ones per tile ----
__global__ __launch_bounds__(kT) void ks_scatter_kernel(
    const int32_t *__restrict__ keys, int64_t n, int32_t nk, int32_t *__restrict__ cnt,
    const int32_t *__restrict__ off, int32_t *__restrict__ tmp, int32_t big_tile,
    int32_t n_big_tiles, const int32_t *__restrict__ ctr, int32_t *__restrict__ mat) {
  extern __shared__ int32_t lds[];
  const int nbig = ctr[1];
  for (int s = threadIdx.x; s < nbig; s += kT) lds[s] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * big_tile;
  const int64_t t1 = std::min<int64_t>(n, t0 + big_tile);
  constexpr int U = 16;
  for (int64_t j0 = t0 + threadIdx.x; j0 < t1; j0 += (int64_t)U * kT) {
    int32_t k[U], v[U], o[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = j0 + (int64_t)u * kT;
      k[u] = i < t1 ? clamp_key(keys[i], nk) : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = k[u] >= 0 ? cnt[k[u]] : -1;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // a non-big bucket's count stays >= 1 until its last entry takes a slot
      o[u] = (k[u] >= 0 && v[u] >= 0) ? atomicSub(&cnt[k[u]], 1) : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (k[u] < 0) continue;
      if (v[u] >= 0) tmp[off[k[u]] + o[u] - 1] = (int32_t)(j0 + (int64_t)u * kT);
      else atomicAdd(&lds[-v[u] - 1], 1);
    }
  }
  __syncthreads();
  for (int s = threadIdx.x; s < nbig; s += kT)
    mat[(int64_t)s * n_big_tiles + blockIdx.x] = lds[s];
}

// ---- 4: per big bucket, exclusive scan of its tile counts (a wave each) ----
__global__ __launch_bounds__(kT) void ks_big_scan_kernel(int32_t *__restrict__ mat,
                                                         int32_t n_big_tiles,
                                                         const int32_t *__restrict__ ctr) {
  const int s = blockIdx.x * (kT / 64) + (threadIdx.x >> 6);
  if (s >= ctr[1]) return;
  const int lane = threadIdx.x & 63;
  int32_t *row = mat + (int64_t)s * n_big_tiles;
  const int per = (n_big_tiles + 63) / 64;
  const int a = std::min(n_big_tiles, lane * per), e = std::min(n_big_tiles, a + per);
  int loc = 0;
  for (int t = a; t < e; ++t) loc += row[t];
  int run = wave_incl_scan(loc) - loc;
  for (int t = a; t < e; ++t) {
    const int c = row[t];
    row[t] = run;
    run += c;
  }
}

__device__ __forceinline__ int32_t val_of(const int32_t *__restrict__ vals, int64_t i) {
  return vals ? vals[i] : (int32_t)i;
}

// ---- 5: small buckets (a thread per entry) and mid buckets (a workgroup
// per bucket, indices staged in LDS): rank = entries of the bucket with a
// lower input index ----
__global__ __launch_bounds__(kT) void ks_finish_kernel(
    const int32_t *__restrict__ keys, const int32_t *__restrict__ vals, int64_t n, int32_t nk,
    const int32_t *__restrict__ off, const int32_t *__restrict__ tmp,
    const int32_t *__restrict__ mid, const int32_t *__restrict__ ctr, int32_t n_small_blocks,
    int32_t n_mid_blocks, int32_t *__restrict__ keys_out, int32_t *__restrict__ vals_out) {
  extern __shared__ int32_t lds[];
  const int b = blockIdx.x;
  if (b < n_small_blocks) {
    const int64_t i = (int64_t)b * kT + threadIdx.x;
    if (i >= n) return;
    const int32_t k = clamp_key(keys[i], nk);
    const int32_t o = off[k], c = off[k + 1] - o;
    if (c > kSmall) return;
    int r = 0;
#pragma unroll 4
    for (int q = 0; q < c; ++q) r += tmp[o + q] < (int32_t)i ? 1 : 0;
    if (r >= c) return;  // (only if the scatter were inconsistent: no write past the bucket)
    keys_out[o + r] = k;
    vals_out[o + r] = val_of(vals, i);
    return;
  }
  const int nmid = ctr[0];
  for (int m = b - n_small_blocks; m < nmid; m += n_mid_blocks) {
    const int32_t k = mid[m];
    const int32_t o = off[k], c = off[k + 1] - o;
    for (int e = threadIdx.x; e < c; e += kT) lds[e] = tmp[o + e];
    __syncthreads();
    for (int e = threadIdx.x; e < c; e += kT) {
      const int32_t x = lds[e];
      int r = 0;
#pragma unroll 8
      for (int q = 0; q < c; ++q) r += lds[q] < x ? 1 : 0;
      if (r >= c) continue;
      keys_out[o + r] = k;
      vals_out[o + r] = val_of(vals, x);
    }
    __syncthreads();
  }
}

// ---- 6: big buckets, a workgroup per tile: its entries staged in input
// order (compacted in LDS with their bucket start and value), then one wave
// places them — per 64 entries, the lanes of one bucket found by ballot, each
// lane's rank among them by popcount, the bucket's running tile offset in LDS
__global__ __launch_bounds__(kT) void ks_big_place_kernel(
    const int32_t *__restrict__ keys, const int32_t *__restrict__ vals, int64_t n, int32_t nk,
    const int32_t *__restrict__ cnt, const int32_t *__restrict__ off,
    const int32_t *__restrict__ mat, int32_t big_tile, int32_t n_big_tiles,
    const int32_t *__restrict__ ctr, int32_t *__restrict__ keys_out,
    int32_t *__restrict__ vals_out) {
  extern __shared__ int32_t lds[];
  const int nbig = ctr[1];
  if (nbig == 0) return;
  int32_t *runs = lds;                 // [nbig]
  int32_t *st_slot = lds + nbig;       // [kStage] staged big entries:
  int32_t *st_base = st_slot + kStage; //   bucket slot, bucket start,
  int32_t *st_key = st_base + kStage;  //   key, value
  int32_t *st_val = st_key + kStage;
  __shared__ int32_t st_n;
  const int t = blockIdx.x;
  for (int s = threadIdx.x; s < nbig; s += kT) runs[s] = mat[(int64_t)s * n_big_tiles + t];
  const int64_t t0 = (int64_t)t * big_tile;
  const int64_t t1 = std::min<int64_t>(n, t0 + big_tile);
  constexpr int P = kStage / kT;  // consecutive entries per thread
  const int lane = threadIdx.x & 63;
  for (int64_t c0 = t0; c0 < t1; c0 += kStage) {
    int32_t k[P], v[P];
    int nb = 0;
#pragma unroll
    for (int u = 0; u < P; ++u) {
      const int64_t i = c0 + (int64_t)threadIdx.x * P + u;
      k[u] = i < t1 ? clamp_key(keys[i], nk) : -1;
    }
#pragma unroll
    for (int u = 0; u < P; ++u) {
      v[u] = k[u] >= 0 ? cnt[k[u]] : 0;
      nb += v[u] < 0 ? 1 : 0;
    }
    int3 tot;
    int w = block_excl_scan3(make_int3(nb, 0, 0), &tot).x;
#pragma unroll
    for (int u = 0; u < P; ++u) {
      if (v[u] >= 0) continue;
      const int64_t i = c0 + (int64_t)threadIdx.x * P + u;
      st_slot[w] = -v[u] - 1;
      st_base[w] = off[k[u]];
      st_key[w] = k[u];
      st_val[w] = val_of(vals, i);
      ++w;
    }
    if (threadIdx.x == 0) st_n = tot.x;
    __syncthreads();
    if (threadIdx.x < 64) {
      const int m = st_n;
      for (int g = 0; g < m; g += 64) {
        const int e = g + lane;
        const bool on = e < m;
        const int slot = on ? st_slot[e] : -1;
        uint64_t rem = __ballot(on);
        while (rem) {
          const int lead = __ffsll((unsigned long long)rem) - 1;
          const int ls = __shfl(slot, lead);
          const uint64_t mask = __ballot(on && slot == ls);
          const int base = runs[ls];
          if (on && slot == ls) {
            const int r = __popcll(mask & ((1ull << lane) - 1ull));
            const int32_t pos = st_base[e] + base + r;
            if (pos < n) keys_out[pos] = st_key[e];
            if (pos < n) vals_out[pos] = st_val[e];
          }
          if (lane == lead) runs[ls] = base + __popcll(mask);
          rem &= ~mask;
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace

size_t key_sort_workspace(int64_t n, int32_t nk) {
  if (n <= 0 || nk <= 0) return 256;
  KsLayout L;
  ks_layout(n, nk, &L);
  return L.total;
}

hipError_t key_sort_pairs(void *ws, size_t ws_bytes, const int32_t *keys_in, int32_t *keys_out,
                          const int32_t *vals_in, int32_t *vals_out, int64_t n, int32_t nk,
                          const int32_t **offsets, hipStream_t st) {
  if (n < 0 || n > kKeySortMaxN || nk <= 0) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  KsLayout L;
  ks_layout(n, nk, &L);
  if (ws == nullptr || ws_bytes < L.total || keys_in == nullptr || keys_out == nullptr ||
      vals_out == nullptr)
    return hipErrorInvalidValue;
  char *w = static_cast<char *>(ws);
  int32_t *cnt = reinterpret_cast<int32_t *>(w + L.cnt);
  int32_t *off = reinterpret_cast<int32_t *>(w + L.off);
  int3 *part = reinterpret_cast<int3 *>(w + L.part);
  int32_t *ctr = reinterpret_cast<int32_t *>(w + L.ctr);
  int32_t *mid = reinterpret_cast<int32_t *>(w + L.mid);
  int32_t *tmp = reinterpret_cast<int32_t *>(w + L.tmp);
  int32_t *mat = reinterpret_cast<int32_t *>(w + L.mat);
  const int64_t n4 = L.nk_pad / 4;
  hipLaunchKernelGGL(ks_zero_kernel, dim3((unsigned)std::min<int64_t>((n4 + kT - 1) / kT, 2048)),
                     dim3(kT), 0, st, reinterpret_cast<int4 *>(cnt), n4, ctr);
  hipLaunchKernelGGL(ks_count_kernel, dim3((unsigned)((n + kCountTile - 1) / kCountTile)), dim3(kT),
                     0, st, keys_in, n, nk, cnt);
  hipLaunchKernelGGL(ks_scan_reduce_kernel, dim3((unsigned)L.nblk), dim3(kT), 0, st, cnt,
                     L.mid_max, part);
  hipLaunchKernelGGL(ks_scan_apply_kernel, dim3((unsigned)L.nblk), dim3(kT), 0, st, cnt, L.mid_max,
                     part, L.nblk, off, mid, ctr);
  hipLaunchKernelGGL(ks_scatter_kernel, dim3((unsigned)L.n_big_tiles), dim3(kT),
                     4 * (size_t)L.big_cap, st, keys_in, n, nk, cnt, off, tmp, L.big_tile,
                     L.n_big_tiles, ctr, mat);
  hipLaunchKernelGGL(ks_big_scan_kernel, dim3((unsigned)((L.big_cap + 3) / 4)), dim3(kT), 0, st,
                     mat, L.n_big_tiles, ctr);
  const int32_t n_small_blocks = (int32_t)((n + kT - 1) / kT);
  const int32_t n_mid_blocks = std::min<int32_t>(L.mid_cap, 1024);
  hipLaunchKernelGGL(ks_finish_kernel, dim3((unsigned)(n_small_blocks + n_mid_blocks)), dim3(kT),
                     4 * (size_t)L.mid_max, st, keys_in, vals_in, n, nk, off, tmp, mid, ctr,
                     n_small_blocks, n_mid_blocks, keys_out, vals_out);
  hipLaunchKernelGGL(ks_big_place_kernel, dim3((unsigned)L.n_big_tiles), dim3(kT),
                     4 * ((size_t)L.big_cap + 4 * kStage), st, keys_in, vals_in, n, nk, cnt, off,
                     mat, L.big_tile, L.n_big_tiles, ctr, keys_out, vals_out);
  if (offsets) *offsets = off;
  return hipGetLastError();
}

}  // namespace mirec

extern "C" int mirec_key_sort_workspace(int64_t n, int32_t nk, size_t *bytes) {
  using namespace mirec;
  MIREC_CHECK_ARG(bytes && n >= 0 && n <= kKeySortMaxN && nk > 0);
  *bytes = key_sort_workspace(n, nk);
  return MIREC_OK;
}

extern "C" int mirec_key_sort_pairs(const int32_t *keys_in, const int32_t *vals_in,
                                    int32_t *keys_out, int32_t *vals_out, int32_t *offsets,
                                    int64_t n, int32_t nk, void *workspace, size_t workspace_bytes,
                                    mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(n >= 0 && n <= kKeySortMaxN && nk > 0);
  if (n == 0) return MIREC_OK;
  MIREC_CHECK_ARG(keys_in && keys_out && vals_out && workspace);
  if (workspace_bytes < key_sort_workspace(n, nk)) return MIREC_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int32_t *off = nullptr;
  MIREC_HIP(key_sort_pairs(workspace, workspace_bytes, keys_in, keys_out, vals_in, vals_out, n, nk,
                           &off, st));
  if (offsets) MIREC_HIP(hipMemcpyAsync(offsets, off, 4 * ((size_t)nk + 1), hipMemcpyDeviceToDevice, st));
  return MIREC_OK;
}
