// Deterministic id-table gradient of the GraphSAGE hop path and the Adam
// step that consumes it without a dense gradient tensor
// (model/graphsage.py:311-337: the table rows gathered for the sampled tree,
// the leaf hop's dropout-mean, and the parameter-norm term of the loss; the
// optimizer step of graphsage.py:388-397).
//
// The table gradient of one step is
//     G[r] = c_slice(r) * W[r]  +  S[r]
// where c_user / c_item = dL/d|slice| / |slice| come from the norm term
// (dense: every row) and S is the sum of the row contributions of the tree:
// the gradient rows of the gathered inner rows, and mask * g_out[t] / cnt_t
// for every leaf entry (sparse: the rows the tree touched).
//
//   mirec_table_grad_sorted  S for every touched row: the entries of all
//       groups are radix-sorted by row id (stable: each id keeps entry
//       order) and every run of equal ids is summed in that order — no
//       float atomics, bitwise repeatable.  The sums are STORED (not added)
//       into acc[r] and stamp[r] = gen marks the row as touched this step,
//       so neither buffer is ever cleared.  Pass 1: a group of LPR lanes
//       takes a chunk of kCh sorted entries, kCh rows in flight, and owns
//       the runs that start in it; a run that leaves the chunk but ends
//       within the next kCh entries (short: nearly every run) is summed whole
//       by its owner, one more batch.  Only a long run (a hub id) is cut at
//       chunk boundaries into partial slots.  Pass 2: the chunk holding a
//       long run's head adds the partials of the chunks the run covers, in
//       chunk order, with every aligned block of 256 chunks inside the run
//       pre-summed by its own group (pass 2a): a hub id in 1.5 M entries is
//       ~730 block sums on the head's path, read LPR at a time.
//   mirec_adam_table   Adam over the whole table with G formed on the fly
//       (W, m, v read once, written once; S read for stamped rows only) —
//       the dense gradient is never written.  Optionally the sums of squares
//       of the updated user / item slices (next step's norm term) per block.
//   mirec_table_grad_dense   G materialised (the data-parallel path, which
//       all-reduces it before the dense Adam).
#include <algorithm>

#include <hipcub/hipcub.hpp>

#include "common.h"
#include "smallsort.h"

namespace mirec {

constexpr int kMaxGroups = MIREC_TABLE_GRAD_MAX_GROUPS;
constexpr int kCh = 8;       // sorted entries per chunk (pass 1 loads them at once)
constexpr int kBatch = 8;            // partial rows in flight per lane in pass 2
constexpr int32_t kEnd = 0x7fffffff;

struct GroupArgs {
  int64_t ent_off[kMaxGroups + 1];  // entry offsets of the groups
  int64_t tgt_off[kMaxGroups + 1];  // target offsets (weight table)
  const int32_t *ids[kMaxGroups];
  const float *grad[kMaxGroups];
  uint64_t key[kMaxGroups];
  uint32_t thresh[kMaxGroups];
  float scale[kMaxGroups];
  int32_t k[kMaxGroups];
  int32_t mean[kMaxGroups];
  int32_t n_groups;
};

// Where the summed rows go.  Dense (slot == nullptr): acc[r] and stamp[r] =
// gen for row r.  Compact (slot != nullptr, mirec_table_grad_sorted_rows):
// the row of the run whose head is sorted entry h goes to vals[slot[h]] and
// its id to rows[slot[h]], slot = the exclusive prefix count of run heads —
// the touched rows ascending, packed, with no dense array and no export
// gather behind them.
struct TgOut {
  float *acc;
  int32_t *stamp;
  int32_t gen;
  const int32_t *slot;
  float *vals;
  int32_t *rows;
};

// Group of a global entry / target index (unrolled selects: the argument
// struct is never indexed dynamically, which would spill it to scratch).
__device__ __forceinline__ int group_of(const int64_t (&off)[kMaxGroups + 1], int n_groups,
                                        int64_t x) {
  int g = 0;
#pragma unroll
  for (int q = 1; q < kMaxGroups; ++q) g += (q < n_groups && x >= off[q]) ? 1 : 0;
  return g;
}

template <typename T, int N>
__device__ __forceinline__ T pick(const T (&a)[N], int g) {
  T r = a[0];
#pragma unroll
  for (int q = 1; q < N; ++q) r = (g == q) ? a[q] : r;
  return r;
}

// The LPR low bits (all 64 for LPR = 64).
template <int LPR>
__device__ __forceinline__ unsigned long long low_bits() {
  if constexpr (LPR == 64) return ~0ull;
  else return (1ull << LPR) - 1ull;
}

// keys[c] = row id of entry c (n_rows for an invalid child: sorts last),
// vals[c] = c; wt[t] = the weight of target t (1/cnt over its valid children
// for a mean group, else 1).
__global__ __launch_bounds__(256) void tg_prep_kernel(GroupArgs ga, int64_t n_ent, int64_t n_tgt,
                                                      int32_t n_rows, int32_t *__restrict__ keys,
                                                      int32_t *__restrict__ vals,
                                                      float *__restrict__ wt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_ent) {
    const int g = group_of(ga.ent_off, ga.n_groups, i);
    const int32_t id = pick(ga.ids, g)[i - pick(ga.ent_off, g)];
    keys[i] = (id >= 0 && id < n_rows) ? id : n_rows;
    vals[i] = (int32_t)i;
  }
  if (i < n_tgt) {
    const int g = group_of(ga.tgt_off, ga.n_groups, i);
    const int64_t t = i - pick(ga.tgt_off, g);
    const int k = pick(ga.k, g);
    const int32_t *ids = pick(ga.ids, g) + t * k;
    int cnt = 0;
    for (int c = 0; c < k; ++c) cnt += ids[c] >= 0 ? 1 : 0;
    wt[i] = pick(ga.mean, g) ? (cnt > 0 ? 1.f / (float)cnt : 0.f) : 1.f;
  }
}

// The plan of sorted entry i (tg_plan_kernel, after the sort): its index v
// in the groups' concatenation and its weight (1/cnt of its target for a
// mean group, else 1; x the dropout scale when its group drops out) — the
// one lookup of an entry that depends on another load, taken here in bulk
// so that pass 1's first round of loads carries everything but the rows.
__global__ __launch_bounds__(256) void tg_plan_kernel(GroupArgs ga, const int32_t *__restrict__ vals,
                                                      const float *__restrict__ wt, int64_t n,
                                                      int2 *__restrict__ plan) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t v = vals[i];
  const int g = group_of(ga.ent_off, ga.n_groups, v);
  const int32_t t = (v - (int32_t)pick(ga.ent_off, g)) / pick(ga.k, g);
  const float w = wt[pick(ga.tgt_off, g) + t];
  plan[i] = make_int2(v, __float_as_int(pick(ga.thresh, g) ? w * pick(ga.scale, g) : w));
}

// Plan entry (v, w) of the sorted order: gradient row address, hash base of
// its dropout quads (key + first quad), threshold, weight.
__device__ __forceinline__ void tg_decode(const GroupArgs &ga, int2 pl, int32_t d, uint64_t &am,
                                          uint64_t &hm, uint32_t &thm, float &wm) {
  const int32_t v = pl.x;
  const int g = group_of(ga.ent_off, ga.n_groups, v);
  const int32_t e = v - (int32_t)pick(ga.ent_off, g);
  const int32_t t = e / pick(ga.k, g);
  thm = pick(ga.thresh, g);
  wm = __int_as_float(pl.y);
  am = (uint64_t)(pick(ga.grad, g) + (int64_t)t * d);
  hm = pick(ga.key, g) + (uint64_t)((int64_t)e * (d / 4));
}

// A float4 through a pointer rebuilt from integers (e.g. broadcast by a lane
// shuffle): named as global memory, so it compiles to global_load_dwordx4.
// (A generic pointer makes it flat_load, which also counts on LGKM_CNT: every
// later `s_waitcnt lgkmcnt(0)` of a shuffle then waits for the row too,
// serialising the gathers.)
__device__ __forceinline__ float4 ldg4(const float *p) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const v4f v = *(const __attribute__((address_space(1))) v4f *)p;
  return make_float4(v.x, v.y, v.z, v.w);
}

// Lane base + u's x for every lane of a group of LPR lanes (u uniform, a
// constant after unrolling): __shfl (ds_bpermute).  (v_readlane for 32 /
// 64-lane groups measured slower at C3: 208 readlanes whose SGPR results
// serialise the wave, accumulate 0.379 vs 0.367 ms.)
template <int LPR>
__device__ __forceinline__ int grp_bcast(int x, int base, int u) {
  return __shfl(x, base + u);
}

// The kCh rows of one batch of entries (lane u of the group decoded entry u)
// in flight at once, then weighted and masked (their inputs re-broadcast, so
// only the rows stay live during the loads).  Only entries lo <= u < hi load
// (the others were not decoded: their addresses are null).
template <int LPR>
__device__ __forceinline__ void tg_rows(int base, int col, bool act, int lo, int hi, uint64_t am,
                                        uint64_t hm, uint32_t thm, float wm,
                                        float4 (&x)[kCh]) {
  const uint32_t am_lo = (uint32_t)am, am_hi = (uint32_t)(am >> 32);
  const uint32_t hm_lo = (uint32_t)hm, hm_hi = (uint32_t)(hm >> 32);
#pragma unroll
  for (int u = 0; u < kCh; ++u) {
    const uint64_t a = (uint64_t)(uint32_t)grp_bcast<LPR>((int)am_lo, base, u) |
                       ((uint64_t)(uint32_t)grp_bcast<LPR>((int)am_hi, base, u) << 32);
    x[u] = (act && u >= lo && u < hi) ? ldg4(reinterpret_cast<const float *>(a) + col) : f4_zero();
  }
#pragma unroll
  for (int u = 0; u < kCh; ++u) {
    const uint32_t th = (uint32_t)grp_bcast<LPR>((int)thm, base, u);
    const float w = __int_as_float(grp_bcast<LPR>(__float_as_int(wm), base, u));
    if (th != 0u) {
      const uint64_t hq = ((uint64_t)(uint32_t)grp_bcast<LPR>((int)hm_lo, base, u) |
                           ((uint64_t)(uint32_t)grp_bcast<LPR>((int)hm_hi, base, u) << 32)) +
                          (uint64_t)(col >> 2);
      x[u] = drop4_hq(x[u], hq, th, w);
    } else {
      x[u] = f4_scale(w, x[u]);
    }
  }
}

// Pass 1.  A group of LPR lanes (LPR >= kCh; d <= 4 LPR, or LPR = 64 with a
// column loop) takes chunk c = sorted entries [c kCh, (c + 1) kCh) and owns
// the RUNS (entries of one row id) that start in it.  Lane j < kCh loads and
// decodes entry j; the group fetches all kCh rows at once (ids broadcast by
// shuffle), weights and masks them while they are in flight, and adds them
// in entry order.  A run that leaves the chunk is SHORT when it ends within
// the next kCh entries (strictly before the next chunk's end, or the array
// ends inside that window): the owner then sums it whole — one more batch
// of at most kCh rows — and the next chunk skips those entries (the same
// test from its side: the run entering it started in the previous chunk and
// ends inside it).  Only LONG runs (hub rows) go through the partial slots
// and pass 2: their head chunk's segment to slot 1, every later chunk's
// first segment to slot 0.  Short runs — nearly all of them — are summed in
// one place without partial rows.
// The loads a chunk starts from: the keys before and around it, its
// entries' keys and indices and those of the window after it.
struct TgRaw {
  int32_t kprev, kpp, km, kx, sl;
  int2 pm, px;
};

__device__ __forceinline__ void tg_load_raw(const int32_t *__restrict__ keys,
                                            const int2 *__restrict__ plan,
                                            const int32_t *__restrict__ slot, int64_t n,
                                            int64_t chunk, int sub, TgRaw &r) {
  const int64_t beg = chunk * kCh;
  const int64_t end = beg + kCh < n ? beg + kCh : n;
  const int64_t xend = end + kCh < n ? end + kCh : n;
  const int64_t pe = beg + sub, px = end + sub;
  const bool in_chunk = sub < kCh && pe < end;
  const bool in_win = sub < kCh && px < xend;
  r.kprev = beg > 0 ? keys[beg - 1] : -1;
  r.kpp = beg > kCh ? keys[beg - kCh - 1] : -1;
  r.km = in_chunk ? keys[pe] : kEnd;
  r.kx = in_win ? keys[px] : kEnd;
  // the entries' plans load beside their keys (not behind them)
  r.pm = in_chunk ? plan[pe] : make_int2(0, 0);
  r.px = in_win ? plan[px] : make_int2(0, 0);
  r.sl = (slot != nullptr && in_chunk) ? slot[pe] : 0;  // compact output: the entries' slots
}

// One chunk of pass 1 from its loaded keys / indices (see below).
template <int LPR>
__device__ __forceinline__ void tg_chunk(const GroupArgs &ga, int64_t n, int32_t d, int32_t n_rows,
                                         const TgOut &o, float *__restrict__ part,
                                         int64_t chunk, int sub,
                                         int base, const TgRaw &r) {
  const int64_t beg = chunk * kCh;
  const int64_t end = beg + kCh < n ? beg + kCh : n;
  const int64_t xend = end + kCh < n ? end + kCh : n;  // the window after the chunk
  const int nin = (int)(end - beg);
  const int64_t pe = beg + sub, px = end + sub;
  const bool in_chunk = sub < kCh && pe < end;
  const bool in_win = sub < kCh && px < xend;
  const int32_t kprev = r.kprev, kpp = r.kpp, km = r.km, kx = r.kx;
  const int32_t first = __shfl(km, base);
  if (first >= n_rows) return;  // only invalid entries from here on
  const unsigned long long kmask = (1ull << kCh) - 1ull;
  // the run entering the chunk: short (owned by the previous chunk's group)
  // iff it started there and ends inside this chunk
  const bool cont_in = beg > 0 && first == kprev;
  const unsigned long long diff_in = (__ballot(in_chunk && km != kprev) >> base) & kmask;
  const bool in_short =
      cont_in && (beg <= kCh || kpp != kprev) && (diff_in != 0 || end < beg + kCh);
  const int skip = in_short ? (diff_in != 0 ? (int)__builtin_ctzll(diff_in) : nin) : 0;
  if (skip >= nin) return;
  // the run leaving the chunk: short iff it started here and ends inside
  // the window after the chunk
  const int32_t klast = __shfl(km, base + nin - 1);
  const int32_t knext = end < n ? __shfl(kx, base) : -1;
  const bool cont_out = end < n && klast == knext && klast < n_rows;
  const bool last_from_before = cont_in && klast == kprev;  // the run covers the chunk
  const unsigned long long diff_out = (__ballot(in_win && kx != klast) >> base) & kmask;
  const bool out_short = cont_out && !last_from_before && (diff_out != 0 || xend < end + kCh);
  const int n_ext =
      out_short ? (diff_out != 0 ? (int)__builtin_ctzll(diff_out) : (int)(xend - end)) : 0;
  uint64_t am = 0, hm = 0, am2 = 0, hm2 = 0;
  uint32_t thm = 0, thm2 = 0;
  float wm = 0.f, wm2 = 0.f;
  if (in_chunk && sub >= skip && km < n_rows) tg_decode(ga, r.pm, d, am, hm, thm, wm);
  if (sub < n_ext) tg_decode(ga, r.px, d, am2, hm2, thm2, wm2);
  // valid entries of the chunk: up to the first invalid id (they sort last)
  const unsigned long long bad = (__ballot(in_chunk && km >= n_rows) >> base) & kmask;
  const int nval = bad != 0 ? (int)__builtin_ctzll(bad) : nin;
  for (int c0 = 0; c0 < d; c0 += 4 * LPR) {
    const int col = c0 + 4 * sub;
    const bool act = col < d;
    // (the owned run's rows past the chunk follow in a second batch: loading
    // both at once measured slower — 127 VGPRs, four waves per SIMD instead
    // of five: pass 1 263 vs 226 us at C3, profiles/round4_tg_bench.jsonl)
    float4 x[kCh];
    tg_rows<LPR>(base, col, act, skip, nval, am, hm, thm, wm, x);
    int32_t cur = -1;
    int64_t seg_beg = 0;
    float4 acc = f4_zero();
    // segment [seg_beg, pos) of id cur ends: a final row sum, or (long runs
    // only) a partial slot
    auto close = [&](int64_t pos) {
      const bool cont_prev = seg_beg == beg && cont_in && !in_short;
      const bool cont_next = pos == end && cont_out && !out_short;
      float *dst;
      if (!cont_prev && !cont_next) {
        if (o.slot != nullptr) {  // a final row starts at its run's head: seg_beg
          const int q = __shfl(r.sl, base + (int)(seg_beg - beg));
          dst = o.vals + (int64_t)q * d;
          if (sub == 0 && c0 == 0) o.rows[q] = cur;
        } else {
          dst = o.acc + (int64_t)cur * d;
          if (sub == 0 && c0 == 0) o.stamp[cur] = o.gen;
        }
      } else {
        dst = part + (2 * chunk + (cont_prev ? 0 : 1)) * (int64_t)d;
      }
      if (act) st4(dst + col, acc);
    };
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      const int32_t ku = grp_bcast<LPR>(km, base, u);
      if (u >= skip && u < nval) {
        if (cur < 0) {
          cur = ku;
          seg_beg = beg + u;
        } else if (ku != cur) {
          close(beg + u);
          cur = ku;
          seg_beg = beg + u;
          acc = f4_zero();
        }
        acc = f4_add(acc, x[u]);
      }
    }
    if (n_ext > 0) {  // the rest of the last run (id klast == cur), in order
      tg_rows<LPR>(base, col, act, 0, n_ext, am2, hm2, thm2, wm2, x);
#pragma unroll
      for (int u = 0; u < kCh; ++u)
        if (u < n_ext) acc = f4_add(acc, x[u]);
    }
    if (cur >= 0) close(beg + nval);
  }
}

// Pass 1 driver: one chunk per lane group.  (A persistent form whose groups
// carry the next chunk's keys measured slower at C3, 259 vs 231 us: 109
// VGPRs, and the gathers, not the key loads, are what each wave waits on.)
template <int LPR>
__global__ __launch_bounds__(256) void tg_sum_kernel(GroupArgs ga, const int32_t *__restrict__ keys,
                                                     const int2 *__restrict__ plan, int64_t n,
                                                     int32_t d, int32_t n_rows, TgOut o,
                                                     float *__restrict__ part) {
  static_assert(LPR >= kCh, "chunk layout: one entry per lane");
  const int lane = threadIdx.x & 63;
  const int sub = lane & (LPR - 1);
  const int base = lane - sub;
  const int64_t group = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
  const int64_t n_chunks = (n + kCh - 1) / kCh;
  if (group >= n_chunks) return;  // the whole group leaves together
  TgRaw r;
  tg_load_raw(keys, plan, o.slot, n, group, sub, r);
  tg_chunk<LPR>(ga, n, d, n_rows, o, part, group, sub, base, r);
}

// Pass 2a: block sums of long runs.  Block b = chunks [G b, G b + G) lies
// wholly inside one run (and the run enters it from before: entries
// G b kCh - 1 .. G (b+1) kCh - 1 share one row id) -> bsum[b] = the head
// slots of its G chunks added in chunk order.  Pass 2b then adds one block
// sum instead of G partial rows, so a hub run of 10^6 entries is ~500 rows
// on the head group's path, not 10^5 (fixed positions -> fixed order).
constexpr int kBlockChunks = 256;  // G

__device__ __forceinline__ bool block_in_run(const int32_t *__restrict__ keys, int64_t n, int64_t b,
                                             int32_t id) {
  const int64_t e0 = b * kBlockChunks * kCh, e1 = (b + 1) * kBlockChunks * kCh;
  return e0 >= 1 && e1 <= n && keys[e0 - 1] == id && keys[e1 - 1] == id;
}

template <int LPR>
__global__ __launch_bounds__(256) void tg_block_kernel(const int32_t *__restrict__ keys, int64_t n,
                                                       int32_t d, int32_t n_rows,
                                                       const float *__restrict__ part,
                                                       float *__restrict__ bsum) {
  const int lane = threadIdx.x & 63;
  const int sub = lane & (LPR - 1);
  const int64_t b = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
  if ((b + 1) * kBlockChunks * kCh > n) return;
  const int64_t e0 = b * kBlockChunks * kCh;
  if (e0 < 1) return;
  const int32_t id = keys[e0 - 1];
  if (id >= n_rows || keys[(b + 1) * kBlockChunks * kCh - 1] != id) return;
  for (int c0 = 0; c0 < d; c0 += 4 * LPR) {
    const int col = c0 + 4 * sub;
    if (col >= d) continue;
    float4 sum = f4_zero();
    for (int j0 = 0; j0 < kBlockChunks; j0 += kBatch) {
      float4 x[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; ++u)
        x[u] = ld4(part + 2 * (b * kBlockChunks + j0 + u) * (int64_t)d + col);
#pragma unroll
      for (int u = 0; u < kBatch; ++u) sum = f4_add(sum, x[u]);
    }
    st4(bsum + b * (int64_t)d + col, sum);
  }
}

// Pass 2b: the group of the chunk holding a LONG run's head adds, in
// chunk order, its tail slot and the head slots of the chunks the run
// covers — a whole aligned block of G chunks inside the run as its block sum
// — and stores the sum.  Lanes test LPR chunks (or blocks) per round.
template <int LPR>
__global__ __launch_bounds__(256) void tg_fixup_kernel(const int32_t *__restrict__ keys, int64_t n,
                                                       int32_t d, int32_t n_rows,
                                                       const float *__restrict__ part,
                                                       const float *__restrict__ bsum, TgOut o) {
  const int lane = threadIdx.x & 63;
  const int sub = lane & (LPR - 1);
  const int base = lane - sub;
  const int64_t chunk = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
  const int64_t beg = chunk * kCh;
  if (beg >= n) return;
  const int64_t end = beg + kCh;
  if (end >= n) return;  // no next chunk
  // one round of key loads decides the common cases
  const int32_t klast = keys[end - 1];
  const int32_t kn = keys[end];
  const int32_t kp = beg > 0 ? keys[beg - 1] : -1;
  if (klast >= n_rows || kn != klast) return;  // last segment stays inside
  if (kp == klast) return;                      // the run's head is earlier
  // a short run (it ends within the next kCh entries) was summed whole by
  // its owner in pass 1: only long runs are left here
  const int64_t xend = end + kCh < n ? end + kCh : n;
  const bool differs = sub < kCh && end + sub < xend && keys[end + sub] != klast;
  if (((__ballot(differs) >> base) & ((1ull << kCh) - 1ull)) != 0 || xend < end + kCh) return;
  const unsigned long long gmask = low_bits<LPR>() << base;
  const unsigned long long low = low_bits<LPR>();
  // compact output: the run's head — its first entry in this chunk — and slot
  int q = 0;
  if (o.slot != nullptr) {
    const bool hd = sub < kCh && keys[beg + sub] == klast;
    const int h = (int)__builtin_ctzll((__ballot(hd) >> base) & ((1ull << kCh) - 1ull));
    q = o.slot[beg + h];
  }
  float *dst = o.slot != nullptr ? o.vals + (int64_t)q * d : o.acc + (int64_t)klast * d;
  for (int c0 = 0; c0 < d; c0 += 4 * LPR) {
    const int col = c0 + 4 * sub;
    const bool act = col < d;
    float4 sum = act ? ld4(part + (2 * chunk + 1) * (int64_t)d + col) : f4_zero();
    int64_t cc = chunk + 1;  // the run continues into chunk cc
    while (true) {
      if (cc % kBlockChunks == 0) {
        // block level: lane j tests block cc / G + j (inside the run, and
        // does the run go on past it?)
        const int64_t bj = cc / kBlockChunks + sub;
        const bool in = block_in_run(keys, n, bj, klast);
        const int64_t ej = (bj + 1) * kBlockChunks * kCh;
        const bool on = in && ej < n && keys[ej] == klast;
        const unsigned long long bal = (__ballot(on) & gmask) >> base;
        const int nfull = bal == low ? LPR : (int)__builtin_ctzll(~bal);
        const bool in_last = nfull < LPR && __shfl(in ? 1 : 0, base + nfull) != 0;
        const int take = nfull + (in_last ? 1 : 0);  // + a block the run ends with
        for (int j0 = 0; j0 < take; j0 += kBatch) {
          float4 x[kBatch];
#pragma unroll
          for (int u = 0; u < kBatch; ++u)
            x[u] = (act && j0 + u < take)
                       ? ld4(bsum + (cc / kBlockChunks + j0 + u) * (int64_t)d + col)
                       : f4_zero();
#pragma unroll
          for (int u = 0; u < kBatch; ++u)
            if (j0 + u < take) sum = f4_add(sum, x[u]);
        }
        if (nfull == LPR) {
          cc += (int64_t)LPR * kBlockChunks;
          continue;
        }
        if (in_last) break;  // the run ends with that block
        cc += (int64_t)nfull * kBlockChunks;  // the run ends inside block cc / G
      }
      // chunk level, up to the next block boundary: lane j: does the run
      // cover all of chunk cc + j and continue past it?
      const int64_t to_bound = kBlockChunks - cc % kBlockChunks;
      const int lim = to_bound < LPR ? (int)to_bound : LPR;
      const int64_t cj = cc + sub;
      const int64_t ej = (cj + 1) * kCh;
      const bool full = sub < lim && ej < n && keys[ej] == klast;
      const unsigned long long bal = (__ballot(full) & gmask) >> base;
      const unsigned long long lmask = lim == 64 ? ~0ull : ((1ull << lim) - 1ull);
      const int nfull = (bal & lmask) == lmask ? lim : (int)__builtin_ctzll(~bal);
      const int take = nfull < lim ? nfull + 1 : lim;  // + the chunk holding the tail
      for (int j0 = 0; j0 < take; j0 += kBatch) {
        float4 x[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; ++u)
          x[u] = (act && j0 + u < take) ? ld4(part + (2 * (cc + j0 + u)) * (int64_t)d + col)
                                        : f4_zero();
#pragma unroll
        for (int u = 0; u < kBatch; ++u)
          if (j0 + u < take) sum = f4_add(sum, x[u]);
      }
      if (nfull < lim) break;
      cc += lim;
    }
    if (act) st4(dst + col, sum);
  }
  if (sub == 0) {
    if (o.slot != nullptr) o.rows[q] = klast;
    else o.stamp[klast] = o.gen;
  }
}

// Compact output: slot = exclusive prefix count of the run heads (sorted
// entry i heads a run when its id is valid and differs from entry i - 1's).
struct TgHeadFlag {
  const int32_t *keys;
  int32_t n_rows;
  __host__ __device__ int operator()(int i) const {
    return (keys[i] < n_rows && (i == 0 || keys[i] != keys[i - 1])) ? 1 : 0;
  }
};

__device__ __forceinline__ int64_t tg_lower_bound(const int32_t *__restrict__ a, int64_t n,
                                                  int64_t x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// counts[0] = the rows written, counts[1 + p] = those in owner block p (rows
// [p N/P, (p + 1) N/P), the last block to N), from the packed ascending ids.
__global__ __launch_bounds__(256) void tg_rows_count_kernel(const int32_t *__restrict__ keys,
                                                            const int32_t *__restrict__ slot,
                                                            int64_t n, int32_t n_rows,
                                                            int32_t parts,
                                                            const int32_t *__restrict__ rows,
                                                            int32_t *__restrict__ counts) {
  const TgHeadFlag f{keys, n_rows};
  const int64_t tot = n > 0 ? (int64_t)slot[n - 1] + f((int)(n - 1)) : 0;
  if (threadIdx.x == 0) counts[0] = (int32_t)tot;
  const int64_t per = n_rows / parts;
  for (int p = threadIdx.x; p < parts; p += blockDim.x) {
    const int64_t lo = p * per, hi = p == parts - 1 ? n_rows : (p + 1) * per;
    counts[1 + p] = (int32_t)(tg_lower_bound(rows, tot, hi) - tg_lower_bound(rows, tot, lo));
  }
}

// ------------------------------------------------------------ consumers
// G = c * W[r] + (S[r] if row r was touched this step, else 0), float4 at
// offset off: one explicit fma per element, so the fused Adam and the
// materialised gradient round identically.
__device__ __forceinline__ float4 table_grad4(float4 w, const float *__restrict__ acc,
                                              const int32_t *__restrict__ stamp, int32_t gen,
                                              int64_t r, int64_t off, float c) {
  const float4 s = stamp[r] == gen ? ld4(acc + off) : f4_zero();
  return make_float4(fmaf(c, w.x, s.x), fmaf(c, w.y, s.y), fmaf(c, w.z, s.z), fmaf(c, w.w, s.w));
}

// Row of float4 element i: a shift when d/4 is a power of two (the table
// widths in use), else a division.
__device__ __forceinline__ int64_t row_of(int64_t i, int32_t d4, int32_t shift) {
  return shift >= 0 ? (i >> shift) : i / d4;
}

__global__ __launch_bounds__(256) void tg_dense_kernel(const float *__restrict__ table,
                                                       const float *__restrict__ coef,
                                                       int64_t n_user, const float *__restrict__ acc,
                                                       const int32_t *__restrict__ stamp,
                                                       int32_t gen, int64_t n_rows, int32_t d4,
                                                       int32_t shift, float *__restrict__ grad) {
  const float cu = coef ? coef[0] : 0.f, ci = coef ? coef[1] : 0.f;
  const int64_t n4 = n_rows * d4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = row_of(i, d4, shift);
    const float4 w = ld4(table + 4 * i);
    st4(grad + 4 * i, table_grad4(w, acc, stamp, gen, r, 4 * i, r < n_user ? cu : ci));
  }
}

// The W / m / v loads are non-temporal (each byte is touched once per step:
// nothing to keep): the C3 launch 0.692 / 0.703 -> 0.667 / 0.675 ms.
// Non-temporal stores measured no gain (0.691 / 0.686 ms), nor more float4
// groups per thread in flight (0.67-0.70 ms at 1, 2, 4: the kernel streams
// at ~5.3 TB/s either way).
typedef float adam_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 adam_ld4(const float *p) {
  const adam_f4 x = __builtin_nontemporal_load(reinterpret_cast<const adam_f4 *>(p));
  return make_float4(x.x, x.y, x.z, x.w);
}
__global__ __launch_bounds__(256) void tg_adam_kernel(float *__restrict__ param,
                                                      float *__restrict__ m, float *__restrict__ v,
                                                      const float *__restrict__ coef, int64_t n_user,
                                                      const float *__restrict__ acc,
                                                      const int32_t *__restrict__ stamp,
                                                      int32_t gen, int64_t n_rows, int32_t d4,
                                                      int32_t shift, mirec_adam_hparams_t h_arg,
                                                      const mirec_adam_hparams_t *__restrict__ h_dev,
                                                      float *__restrict__ sumsq) {
  __shared__ float red[2][256];
  const mirec_adam_hparams_t h = h_dev != nullptr ? *h_dev : h_arg;
  const float cu = coef ? coef[0] : 0.f, ci = coef ? coef[1] : 0.f;
  const int64_t n4 = n_rows * d4;
  float su = 0.f, si = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 p = adam_ld4(param + 4 * i), a = adam_ld4(m + 4 * i), b = adam_ld4(v + 4 * i);
    const int64_t r = row_of(i, d4, shift);
    const float4 g = table_grad4(p, acc, stamp, gen, r, 4 * i, r < n_user ? cu : ci);
    adam1(p.x, a.x, b.x, g.x, h);
    adam1(p.y, a.y, b.y, g.y, h);
    adam1(p.z, a.z, b.z, g.z, h);
    adam1(p.w, a.w, b.w, g.w, h);
    st4(param + 4 * i, p);
    st4(m + 4 * i, a);
    st4(v + 4 * i, b);
    const float s = p.x * p.x + p.y * p.y + p.z * p.z + p.w * p.w;
    if (r < n_user) su += s;
    else si += s;
  }
  if (sumsq == nullptr) return;
  red[0][threadIdx.x] = su;
  red[1][threadIdx.x] = si;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    sumsq[2 * blockIdx.x] = red[0][0];
    sumsq[2 * blockIdx.x + 1] = red[1][0];
  }
}

// norms[0..1] = sqrt of the block partials summed in a fixed order: 1024
// threads, thread j adds partials j, j + 1024, ... (8 loads in flight), then
// a tree over the threads.
__global__ __launch_bounds__(1024) void tg_norm_final_kernel(const float *__restrict__ sumsq,
                                                             int64_t blocks,
                                                             float *__restrict__ norms) {
  __shared__ float red[2][1024];
  float a = 0.f, b = 0.f;
  for (int64_t k0 = threadIdx.x; k0 < blocks; k0 += 8 * 1024) {
    float2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t k = k0 + (int64_t)u * 1024;
      v[u] = k < blocks ? *reinterpret_cast<const float2 *>(sumsq + 2 * k) : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a += v[u].x;
      b += v[u].y;
    }
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    norms[0] = sqrtf(red[0][0]);
    norms[1] = sqrtf(red[1][0]);
  }
}

// ------------------------------------- the owner's ordered sum of row blocks
// S of the own row block [lo, lo + n_own) from source blocks (ids, rows),
// added in block order — each block's ids distinct — exactly as a sequence
// of index_add_ launches would (0 + a, then + b, ...), in one pass: every
// block's ids are first inverted into a position map pos[q][r] (-1: absent),
// then one thread per (own row, float4 column) adds the blocks' rows in
// order, writing each output row once.  Up to kOsMax blocks per pass; more
// run as further passes that start from the output.
constexpr int kOsMax = 64;
struct OsBlocks {
  const int32_t *ids[kOsMax];
  const float4 *rows[kOsMax];
  int64_t off[kOsMax + 1];  // prefix of the block sizes
  int32_t n;
};

__global__ __launch_bounds__(256) void os_mark_kernel(OsBlocks b, int64_t lo, int64_t n_own,
                                                      int32_t *__restrict__ pos) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= b.off[b.n]) return;
  int q = 0;
  while (q + 1 < b.n && b.off[q + 1] <= e) ++q;
  const int64_t i = e - b.off[q];
  const int64_t r = (int64_t)b.ids[q][i] - lo;
  if (r >= 0 && r < n_own) pos[q * n_own + r] = (int32_t)i;
}

// (1 << lg lanes per own row as the row movers; the blocks four at a time:
// their positions, then their rows in flight together, then the adds in
// block order)
__global__ __launch_bounds__(256) void os_sum_kernel(OsBlocks b, const int32_t *__restrict__ pos,
                                                     int64_t n_own, int32_t d4, int32_t lg,
                                                     int accumulate, float4 *__restrict__ out) {
  const int c = threadIdx.x & ((1 << lg) - 1);
  const int64_t r = (int64_t)blockIdx.x * (256 >> lg) + (threadIdx.x >> lg);
  if (r >= n_own || c >= d4) return;
  const int64_t t = r * d4 + c;
  float4 acc = accumulate ? out[t] : f4_zero();
  for (int q0 = 0; q0 < b.n; q0 += 4) {
    int32_t i[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) i[u] = q0 + u < b.n ? pos[(q0 + u) * n_own + r] : -1;
    float4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      x[u] = i[u] >= 0 ? b.rows[q0 + u][(int64_t)i[u] * d4 + c] : f4_zero();
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i[u] >= 0) acc = f4_add(acc, x[u]);
  }
  out[t] = acc;
}


// The owner's fused step (data-parallel exchanges): S of the own row block
// as os_sum forms it — the blocks' rows at pos[q][r] added in block order
// from zero — and the table Adam of tg_adam_kernel on those rows, in one
// pass: S is neither written nor read back.  The same element mapping and
// block partials as tg_adam_kernel (norms bitwise equal).
__global__ __launch_bounds__(256) void os_adam_kernel(OsBlocks b, const int32_t *__restrict__ pos,
                                                      int64_t n_own, float *__restrict__ param,
                                                      float *__restrict__ m, float *__restrict__ v,
                                                      const float *__restrict__ coef,
                                                      int64_t n_user, int32_t d4, int32_t shift,
                                                      mirec_adam_hparams_t h,
                                                      float *__restrict__ sumsq) {
  __shared__ float red[2][256];
  const float cu = coef ? coef[0] : 0.f, ci = coef ? coef[1] : 0.f;
  const int64_t n4 = n_own * d4;
  float su = 0.f, si = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 p = adam_ld4(param + 4 * i), a = adam_ld4(m + 4 * i), bv = adam_ld4(v + 4 * i);
    const int64_t r = row_of(i, d4, shift);
    const int64_t c = i - r * d4;
    float4 s = f4_zero();
    for (int q0 = 0; q0 < b.n; q0 += 4) {
      int32_t k[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) k[u] = q0 + u < b.n ? pos[(q0 + u) * n_own + r] : -1;
      float4 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        x[u] = k[u] >= 0 ? b.rows[q0 + u][(int64_t)k[u] * d4 + c] : f4_zero();
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (k[u] >= 0) s = f4_add(s, x[u]);
    }
    const float cc = r < n_user ? cu : ci;
    const float4 g = make_float4(fmaf(cc, p.x, s.x), fmaf(cc, p.y, s.y), fmaf(cc, p.z, s.z),
                                 fmaf(cc, p.w, s.w));
    adam1(p.x, a.x, bv.x, g.x, h);
    adam1(p.y, a.y, bv.y, g.y, h);
    adam1(p.z, a.z, bv.z, g.z, h);
    adam1(p.w, a.w, bv.w, g.w, h);
    st4(param + 4 * i, p);
    st4(m + 4 * i, a);
    st4(v + 4 * i, bv);
    const float sq = p.x * p.x + p.y * p.y + p.z * p.z + p.w * p.w;
    if (r < n_user) su += sq;
    else si += sq;
  }
  if (sumsq == nullptr) return;
  red[0][threadIdx.x] = su;
  red[1][threadIdx.x] = si;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    sumsq[2 * blockIdx.x] = red[0][0];
    sumsq[2 * blockIdx.x + 1] = red[1][0];
  }
}

// ------------------------------------------------------------ host side
// The stable (key, value) radix sort of the entries, 11 bits per onesweep
// pass (rocprim's own choice for int pairs on gfx950 is 8: three passes over
// the 21-bit row ids of C3; 11 covers them in two: the C3 accumulate 0.389
// -> 0.367 ms, same order, bitwise equal sums).
static hipError_t tg_sort(void *tmp, size_t &bytes, const int32_t *ki, int32_t *ko, const int32_t *vi,
                          int32_t *vo, int n, int end_bit, hipStream_t st) {
  // up to 8 K entries the library's own two-launch sort (smallsort.hip)
  // instead of the radix sort's block sort + merge passes; the same order
  if (n <= kSmallSortMax) {
    if (tmp == nullptr) {
      bytes = small_sort_workspace(n);
      return hipSuccess;
    }
    return small_sort_pairs(tmp, bytes, ki, ko, vi, vo, n, st);
  }
  using Onesweep = rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>,
                                                       rocprim::kernel_config<1024, 8>, 11,
                                                       rocprim::block_radix_rank_algorithm::match>;
  // onesweep from 128 K entries up: rocprim's default merge-sort limit (1 M)
  // sent a micro-batch's ~0.9 M entries (the pipelined exchange, C = 2)
  // through ~20 block-sort / merge launches, 150 us against the full
  // batch's 85 us onesweep; both are stable, so the order is the same
  using Cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, Onesweep,
                                         (size_t)1 << 17>;
  return rocprim::radix_sort_pairs<Cfg>(tmp, bytes, ki, ko, vi, vo, (size_t)n, 0, end_bit, st);
}

// Lanes per chunk group: one entry per lane (kCh) up to 16, wider rows in a
// column loop.  Groups of 32 (d = 128: a whole row per group) repeated the
// chunk's key / plan bookkeeping in 24 lanes that carry no entry; 16-lane
// groups with a two-pass column loop: C3 accumulate 0.357 -> 0.345 ms, the
// same sums bit for bit (profiles/round6_tg_lanes.jsonl).
static int lanes_per_row(int32_t d) {
  const int d4 = (d + 3) / 4;
  int l = kCh;  // pass 1: one entry per lane of a group
  while (l < d4 && l < 16) l <<= 1;
  return l;
}

struct TgLayout {
  int64_t n_ent, n_tgt, n_chunks;
  size_t keys_in, keys_out, vals_in, vals_out, wt, plan, part, bsum, slot, scan, scan_bytes, sort,
      sort_bytes, total;
  int end_bit;
};

static int tg_layout(const mirec_row_grad_group_t *groups, int32_t n_groups, int32_t n_rows,
                     int32_t dim, TgLayout *L) {
  MIREC_CHECK_ARG(n_groups >= 1 && n_groups <= kMaxGroups && n_rows > 0 && dim > 0 &&
                  dim % 4 == 0 && groups);
  int64_t n_ent = 0, n_tgt = 0;
  for (int g = 0; g < n_groups; ++g) {
    const mirec_row_grad_group_t &q = groups[g];
    MIREC_CHECK_ARG(q.n_targets >= 0 && q.k >= 1 && q.dropout_p >= 0.f && q.dropout_p < 1.f);
    n_ent += q.n_targets * q.k;
    n_tgt += q.n_targets;
  }
  MIREC_CHECK_ARG(n_ent < ((int64_t)1 << 31) - kCh);
  const auto up = [](size_t b) { return (b + 255) / 256 * 256; };
  L->n_ent = n_ent;
  L->n_tgt = n_tgt;
  L->n_chunks = (n_ent + kCh - 1) / kCh;
  const size_t seg = up(sizeof(int32_t) * std::max<int64_t>(n_ent, 1));
  L->keys_in = 0;
  L->keys_out = seg;
  L->vals_in = 2 * seg;
  L->vals_out = 3 * seg;
  L->wt = 4 * seg;
  L->plan = L->wt + up(sizeof(float) * std::max<int64_t>(n_tgt, 1));
  L->part = L->plan + 2 * seg;
  L->bsum = L->part + up(sizeof(float) * 2 * std::max<int64_t>(L->n_chunks, 1) * dim);
  L->slot = L->bsum + up(sizeof(float) * std::max<int64_t>(L->n_chunks / kBlockChunks, 1) * dim);
  L->scan = L->slot + seg;
  size_t sb = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(
      nullptr, sb, hipcub::TransformInputIterator<int, TgHeadFlag, hipcub::CountingInputIterator<int>>(
                       hipcub::CountingInputIterator<int>(0), TgHeadFlag{nullptr, 0}),
      (int32_t *)nullptr, (int)std::max<int64_t>(n_ent, 1), (hipStream_t) nullptr);
  L->scan_bytes = sb;
  L->sort = L->scan + up(sb);
  int bits = 1;
  while (bits < 31 && ((int64_t)1 << bits) <= n_rows) ++bits;
  L->end_bit = bits;
  size_t tb = 0;
  (void)tg_sort(nullptr, tb, nullptr, nullptr, nullptr, nullptr, (int)std::max<int64_t>(n_ent, 1),
                bits, nullptr);
  L->sort_bytes = tb;
  L->total = L->sort + up(tb);
  return MIREC_OK;
}

}  // namespace mirec

using namespace mirec;

extern "C" int64_t mirec_row_grad_group_size(void) {
  return (int64_t)sizeof(mirec_row_grad_group_t);
}

extern "C" int mirec_table_grad_workspace(const mirec_row_grad_group_t *groups, int32_t n_groups,
                                          int32_t n_rows, int32_t dim, size_t *bytes) {
  MIREC_CHECK_ARG(bytes);
  TgLayout L;
  const int rc = tg_layout(groups, n_groups, n_rows, dim, &L);
  if (rc != MIREC_OK) return rc;
  *bytes = L.total;
  return MIREC_OK;
}

// Atomic form (plain groups: k = 1, no mean, no dropout): pass 1 stamps every
// touched row with gen and zeroes its acc row (idempotent, so repeated ids
// are harmless), pass 2 adds every entry's gradient row with float atomics.
// Two short launches instead of the sort; the summation order of a repeated
// id is not fixed (reruns can differ in the last bits).
__global__ __launch_bounds__(256) void tg_claim_kernel(GroupArgs ga, int64_t n_ent, int32_t d4,
                                                       int32_t n_rows, float *__restrict__ acc,
                                                       int32_t *__restrict__ stamp, int32_t gen) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ent * d4) return;
  const int64_t e = i / d4;
  const int c4 = (int)(i - e * d4);
  const int g = group_of(ga.ent_off, ga.n_groups, e);
  const int32_t id = pick(ga.ids, g)[e - pick(ga.ent_off, g)];
  if (id < 0 || id >= n_rows) return;
  if (c4 == 0) stamp[id] = gen;
  st4(acc + (int64_t)id * 4 * d4 + 4 * c4, f4_zero());
}

__global__ __launch_bounds__(256) void tg_atomic_add_kernel(GroupArgs ga, int64_t n_ent, int32_t d4,
                                                            int32_t n_rows,
                                                            float *__restrict__ acc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ent * d4) return;
  const int64_t e = i / d4;
  const int c4 = (int)(i - e * d4);
  const int g = group_of(ga.ent_off, ga.n_groups, e);
  const int64_t le = e - pick(ga.ent_off, g);
  const int32_t id = pick(ga.ids, g)[le];
  if (id < 0 || id >= n_rows) return;
  const float4 v = ld4(pick(ga.grad, g) + le * 4 * d4 + 4 * c4);
  float *dst = acc + (int64_t)id * 4 * d4 + 4 * c4;
  atomicAdd(dst, v.x);
  atomicAdd(dst + 1, v.y);
  atomicAdd(dst + 2, v.z);
  atomicAdd(dst + 3, v.w);
}

extern "C" int mirec_table_grad_atomic(const mirec_row_grad_group_t *groups, int32_t n_groups,
                                       int32_t n_rows, int32_t dim, float *acc, int32_t *stamp,
                                       int32_t gen, mirec_stream_t stream) {
  MIREC_CHECK_ARG(groups && n_groups >= 1 && n_groups <= kMaxGroups && n_rows >= 0 && dim > 0 &&
                  dim % 4 == 0 && acc && stamp && (uintptr_t)acc % 16 == 0);
  GroupArgs ga = {};
  ga.n_groups = n_groups;
  for (int g = 0; g < kMaxGroups; ++g) {
    const bool real = g < n_groups;
    const mirec_row_grad_group_t *q = real ? &groups[g] : nullptr;
    if (real) {
      MIREC_CHECK_ARG(q->n_targets >= 0 && q->k == 1 && q->mean == 0 && q->dropout_p == 0.f);
      MIREC_CHECK_ARG(q->n_targets == 0 ||
                      (q->ids && q->grad_out && (uintptr_t)q->grad_out % 16 == 0));
    }
    ga.ent_off[g + 1] = ga.ent_off[g] + (real ? q->n_targets : 0);
    ga.tgt_off[g + 1] = ga.ent_off[g + 1];
    ga.ids[g] = real ? q->ids : nullptr;
    ga.grad[g] = real ? q->grad_out : nullptr;
    ga.k[g] = 1;
  }
  const int64_t n_ent = ga.ent_off[kMaxGroups];
  if (n_ent == 0) return MIREC_OK;
  const int32_t d4 = dim / 4;
  const int64_t total = n_ent * d4;
  const dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(tg_claim_kernel, grid, dim3(256), 0, st, ga, n_ent, d4, n_rows, acc, stamp,
                     gen);
  MIREC_LAUNCH_CHECK();
  hipLaunchKernelGGL(tg_atomic_add_kernel, grid, dim3(256), 0, st, ga, n_ent, d4, n_rows, acc);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

// The sorted accumulate into `o` (dense or compact; compact: also the
// counts [1 + parts]).
static int tg_sorted(const mirec_row_grad_group_t *groups, int32_t n_groups, int32_t n_rows,
                     int32_t dim, TgOut o, int32_t parts, int32_t *counts, void *workspace,
                     size_t workspace_bytes, mirec_stream_t stream) {
  TgLayout L;
  const int rc = tg_layout(groups, n_groups, n_rows, dim, &L);
  if (rc != MIREC_OK) return rc;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (L.n_ent == 0) {
    if (counts != nullptr) MIREC_HIP(hipMemsetAsync(counts, 0, 4 * (size_t)(1 + parts), st));
    return MIREC_OK;
  }
  MIREC_CHECK_ARG(workspace);
  if (workspace_bytes < L.total) return MIREC_ERR_WORKSPACE;
  GroupArgs ga = {};
  ga.n_groups = n_groups;
  for (int g = 0; g < kMaxGroups; ++g) {
    const bool real = g < n_groups;
    const mirec_row_grad_group_t *q = real ? &groups[g] : nullptr;
    ga.ent_off[g + 1] = ga.ent_off[g] + (real ? q->n_targets * q->k : 0);
    ga.tgt_off[g + 1] = ga.tgt_off[g] + (real ? q->n_targets : 0);
    ga.ids[g] = real ? q->ids : nullptr;
    ga.grad[g] = real ? q->grad_out : nullptr;
    ga.k[g] = real ? q->k : 1;
    ga.mean[g] = real ? q->mean : 0;
    uint64_t key = 0;
    uint32_t th = 0;
    float sc = 1.f;
    if (real) {
      MIREC_CHECK_ARG(q->n_targets == 0 || (q->ids && q->grad_out));
      MIREC_CHECK_ARG(dropout_params(q->dropout_p, q->seed, &key, &th, &sc));
    }
    ga.key[g] = key;
    ga.thresh[g] = th;
    ga.scale[g] = sc;
  }
  char *ws = static_cast<char *>(workspace);
  int32_t *keys_in = reinterpret_cast<int32_t *>(ws + L.keys_in);
  int32_t *keys_out = reinterpret_cast<int32_t *>(ws + L.keys_out);
  int32_t *vals_in = reinterpret_cast<int32_t *>(ws + L.vals_in);
  int32_t *vals_out = reinterpret_cast<int32_t *>(ws + L.vals_out);
  float *wt = reinterpret_cast<float *>(ws + L.wt);
  int2 *plan = reinterpret_cast<int2 *>(ws + L.plan);
  float *part = reinterpret_cast<float *>(ws + L.part);
  float *bsum = reinterpret_cast<float *>(ws + L.bsum);
  const int64_t nprep = std::max(L.n_ent, L.n_tgt);
  hipLaunchKernelGGL(tg_prep_kernel, dim3((unsigned)((nprep + 255) / 256)), dim3(256), 0, st, ga,
                     L.n_ent, L.n_tgt, n_rows, keys_in, vals_in, wt);
  MIREC_LAUNCH_CHECK();
  size_t sort_bytes = L.sort_bytes;
  MIREC_HIP(tg_sort(ws + L.sort, sort_bytes, keys_in, keys_out, vals_in, vals_out, (int)L.n_ent,
                    L.end_bit, st));
  hipLaunchKernelGGL(tg_plan_kernel, dim3((unsigned)((L.n_ent + 255) / 256)), dim3(256), 0, st,
                     ga, vals_out, wt, L.n_ent, plan);
  MIREC_LAUNCH_CHECK();
  int32_t *slot = reinterpret_cast<int32_t *>(ws + L.slot);
  if (o.vals != nullptr) {  // compact: the run heads' slots
    size_t sb = L.scan_bytes;
    MIREC_HIP(hipcub::DeviceScan::ExclusiveSum(
        ws + L.scan, sb,
        hipcub::TransformInputIterator<int, TgHeadFlag, hipcub::CountingInputIterator<int>>(
            hipcub::CountingInputIterator<int>(0), TgHeadFlag{keys_out, n_rows}),
        slot, (int)L.n_ent, st));
    o.slot = slot;
  }
  const int lpr = lanes_per_row(dim);
  const int64_t threads = L.n_chunks * lpr;
  const int64_t n_blocks = L.n_chunks / kBlockChunks;
  const dim3 grid((unsigned)((threads + 255) / 256));
#define MIREC_TG_LAUNCH(LP)                                                                   \
  case LP:                                                                                   \
    hipLaunchKernelGGL(tg_sum_kernel<LP>, grid, dim3(256), 0, st, ga,        \
                       keys_out, plan, L.n_ent, dim, n_rows, o, part);                        \
    MIREC_LAUNCH_CHECK();                                                                    \
    if (n_blocks > 0) {                                                                      \
      hipLaunchKernelGGL(tg_block_kernel<LP>, dim3((unsigned)((n_blocks * LP + 255) / 256)),  \
                         dim3(256), 0, st, keys_out, L.n_ent, dim, n_rows, part, bsum);       \
      MIREC_LAUNCH_CHECK();                                                                  \
    }                                                                                        \
    hipLaunchKernelGGL(tg_fixup_kernel<LP>, grid, dim3(256), 0, st, keys_out, L.n_ent, dim,   \
                       n_rows, part, bsum, o);                                               \
    MIREC_LAUNCH_CHECK();                                                                    \
    break;
  switch (lpr) {  // lpr >= kCh (lanes_per_row)
    MIREC_TG_LAUNCH(8)
    MIREC_TG_LAUNCH(16)
    MIREC_TG_LAUNCH(32)
    MIREC_TG_LAUNCH(64)
    default:
      return MIREC_ERR_ARG;
  }
#undef MIREC_TG_LAUNCH
  if (o.slot != nullptr) {
    hipLaunchKernelGGL(tg_rows_count_kernel, dim3(1), dim3(256), 0, st, keys_out, slot, L.n_ent,
                       n_rows, parts, o.rows, counts);
    MIREC_LAUNCH_CHECK();
  }
  return MIREC_OK;
}

extern "C" int mirec_table_grad_sorted(const mirec_row_grad_group_t *groups, int32_t n_groups,
                                       int32_t n_rows, int32_t dim, float *acc, int32_t *stamp,
                                       int32_t gen, void *workspace, size_t workspace_bytes,
                                       mirec_stream_t stream) {
  MIREC_CHECK_ARG(acc && stamp);
  return tg_sorted(groups, n_groups, n_rows, dim, TgOut{acc, stamp, gen, nullptr, nullptr, nullptr},
                   1, nullptr, workspace, workspace_bytes, stream);
}

extern "C" int mirec_table_grad_sorted_rows(const mirec_row_grad_group_t *groups,
                                            int32_t n_groups, int32_t n_rows, int32_t dim,
                                            int32_t parts, int32_t *rows, float *vals,
                                            int32_t *counts, void *workspace,
                                            size_t workspace_bytes, mirec_stream_t stream) {
  MIREC_CHECK_ARG(rows && vals && counts && parts >= 1 && parts <= n_rows &&
                  (uintptr_t)vals % 16 == 0);
  return tg_sorted(groups, n_groups, n_rows, dim, TgOut{nullptr, nullptr, 0, nullptr, vals, rows},
                   parts, counts, workspace, workspace_bytes, stream);
}

static int32_t pow2_shift(int32_t d4) {
  for (int s = 0; s < 31; ++s)
    if ((1 << s) == d4) return s;
  return -1;
}

static unsigned tg_blocks(int64_t n4) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n4 + 255) / 256, 65536));
}

extern "C" int64_t mirec_adam_table_sumsq_floats(int64_t n_rows, int32_t dim) {
  if (n_rows < 0 || dim <= 0 || dim % 4) return -1;
  return 2 * (int64_t)tg_blocks(n_rows * (dim / 4));
}

extern "C" int mirec_table_grad_dense(const float *table, const float *coef, int64_t n_user,
                                      const float *acc, const int32_t *stamp, int32_t gen,
                                      int64_t n_rows, int32_t dim, float *grad,
                                      mirec_stream_t stream) {
  MIREC_CHECK_ARG(table && acc && stamp && grad && n_rows >= 0 && dim > 0 && dim % 4 == 0 &&
                  n_user >= 0 && n_user <= n_rows);
  MIREC_CHECK_ARG(((uintptr_t)table | (uintptr_t)acc | (uintptr_t)grad) % 16 == 0);
  if (n_rows == 0) return MIREC_OK;
  const int64_t n4 = n_rows * (dim / 4);
  hipLaunchKernelGGL(tg_dense_kernel, dim3(tg_blocks(n4)), dim3(256), 0, (hipStream_t)stream,
                     table, coef, n_user, acc, stamp, gen, n_rows, dim / 4, pow2_shift(dim / 4),
                     grad);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

static int adam_table(float *param, float *exp_avg, float *exp_avg_sq, const float *coef,
                      int64_t n_user, const float *acc, const int32_t *stamp, int32_t gen,
                      int64_t n_rows, int32_t dim, const mirec_adam_hparams_t *h,
                      const mirec_adam_hparams_t *h_dev, float *sumsq, float *norms,
                      mirec_stream_t stream) {
  MIREC_CHECK_ARG(param && exp_avg && exp_avg_sq && acc && stamp && (h || h_dev) &&
                  n_rows >= 0 && dim > 0 && dim % 4 == 0 && n_user >= 0 && n_user <= n_rows);
  MIREC_CHECK_ARG(((uintptr_t)param | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq |
                   (uintptr_t)acc) % 16 == 0);
  MIREC_CHECK_ARG((sumsq == nullptr) == (norms == nullptr));
  if (n_rows == 0) return MIREC_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t n4 = n_rows * (dim / 4);
  const unsigned blocks = tg_blocks(n4);
  const mirec_adam_hparams_t h0 = h ? *h : mirec_adam_hparams_t{};
  hipLaunchKernelGGL(tg_adam_kernel, dim3(blocks), dim3(256), 0, st, param, exp_avg, exp_avg_sq,
                     coef, n_user, acc, stamp, gen, n_rows, dim / 4, pow2_shift(dim / 4), h0,
                     h ? nullptr : h_dev, sumsq);
  MIREC_LAUNCH_CHECK();
  if (norms) {
    hipLaunchKernelGGL(tg_norm_final_kernel, dim3(1), dim3(1024), 0, st, sumsq, (int64_t)blocks,
                       norms);
    MIREC_LAUNCH_CHECK();
  }
  return MIREC_OK;
}

extern "C" int mirec_adam_table(float *param, float *exp_avg, float *exp_avg_sq, const float *coef,
                                int64_t n_user, const float *acc, const int32_t *stamp,
                                int32_t gen, int64_t n_rows, int32_t dim,
                                const mirec_adam_hparams_t *h, float *sumsq, float *norms,
                                mirec_stream_t stream) {
  MIREC_CHECK_ARG(h != nullptr);
  return adam_table(param, exp_avg, exp_avg_sq, coef, n_user, acc, stamp, gen, n_rows, dim, h,
                    nullptr, sumsq, norms, stream);
}

extern "C" int mirec_adam_table_dev(float *param, float *exp_avg, float *exp_avg_sq,
                                    const float *coef, int64_t n_user, const float *acc,
                                    const int32_t *stamp, int32_t gen, int64_t n_rows,
                                    int32_t dim, const mirec_adam_hparams_t *h_device,
                                    float *sumsq, float *norms, mirec_stream_t stream) {
  MIREC_CHECK_ARG(h_device != nullptr);
  return adam_table(param, exp_avg, exp_avg_sq, coef, n_user, acc, stamp, gen, n_rows, dim,
                    nullptr, h_device, sumsq, norms, stream);
}

// coef[i] = norm[i ns] > 0 ? g[i gs] / norm[i ns] : 0 (i < n): the norm-term
// coefficients of a table gradient, d|x|/dx = x / |x| (0 for a zero table,
// as torch's norm backward); g = the loss's gradient w.r.t. the norm.
__global__ void norm_coef_kernel(const float *__restrict__ g, int gs,
                                 const float *__restrict__ norm, int ns, int n,
                                 float *__restrict__ coef) {
  const int i = threadIdx.x;
  if (i < n) {
    const float nv = norm[i * ns];
    coef[i] = nv > 0.f ? g[i * gs] / nv : 0.f;
  }
}

extern "C" int mirec_norm_coef(const float *g, int32_t g_stride, const float *norm,
                               int32_t norm_stride, int32_t n, float *coef,
                               mirec_stream_t stream) {
  MIREC_CHECK_ARG(g && norm && coef && n >= 0 && n <= 1024 && g_stride >= 0 && norm_stride >= 0);
  if (n == 0) return MIREC_OK;
  hipLaunchKernelGGL(norm_coef_kernel, dim3(1), dim3(64 * ((n + 63) / 64)), 0,
                     (hipStream_t)stream, g, g_stride, norm, norm_stride, n, coef);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

// The owner's pos maps of blocks [q0, q0 + b.n) into `pos` (cleared first).
static int os_blocks(const mirec_row_block_t *blocks, int32_t q0, int32_t n_blocks, int64_t lo,
                     int64_t n_own, int32_t *pos, hipStream_t st, OsBlocks &b) {
  b = OsBlocks{};
  b.n = std::min<int32_t>(kOsMax, n_blocks - q0);
  b.off[0] = 0;
  for (int q = 0; q < b.n; ++q) {
    const mirec_row_block_t &x = blocks[q0 + q];
    MIREC_CHECK_ARG(x.n >= 0 && (x.n == 0 || (x.ids && x.rows)));
    MIREC_CHECK_ARG(((uintptr_t)x.rows & 15u) == 0);
    b.ids[q] = x.ids;
    b.rows[q] = reinterpret_cast<const float4 *>(x.rows);
    b.off[q + 1] = b.off[q] + x.n;
  }
  MIREC_HIP(hipMemsetAsync(pos, 0xff, (size_t)(4 * b.n * n_own), st));
  if (b.off[b.n] > 0) {
    hipLaunchKernelGGL(os_mark_kernel, dim3((unsigned)((b.off[b.n] + 255) / 256)), dim3(256), 0,
                       st, b, lo, n_own, pos);
    MIREC_LAUNCH_CHECK();
  }
  return MIREC_OK;
}

extern "C" int64_t mirec_owner_sum_workspace(int32_t n_blocks, int64_t n_own) {
  if (n_blocks < 0 || n_own < 0) return -1;
  return 4 * (int64_t)std::min<int32_t>(std::max<int32_t>(n_blocks, 1), mirec::kOsMax) * n_own;
}

extern "C" int mirec_owner_sum(const mirec_row_block_t *blocks, int32_t n_blocks, int64_t lo,
                               int64_t n_own, int32_t dim, void *workspace,
                               size_t workspace_bytes, float *out, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(n_blocks >= 0 && n_own >= 0 && dim > 0 && dim % 4 == 0);
  MIREC_CHECK_ARG(n_blocks == 0 || blocks);
  if (n_own == 0) return MIREC_OK;
  MIREC_CHECK_ARG(out && ((uintptr_t)out & 15u) == 0);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t d4 = dim / 4;
  if (n_blocks == 0) {
    MIREC_HIP(hipMemsetAsync(out, 0, (size_t)(n_own * dim) * 4, st));
    return MIREC_OK;
  }
  MIREC_CHECK_ARG(workspace);
  if ((int64_t)workspace_bytes < mirec_owner_sum_workspace(n_blocks, n_own))
    return MIREC_ERR_WORKSPACE;
  int32_t *pos = static_cast<int32_t *>(workspace);
  for (int32_t q0 = 0; q0 < n_blocks; q0 += kOsMax) {
    OsBlocks b;
    const int rc = os_blocks(blocks, q0, n_blocks, lo, n_own, pos, st, b);
    if (rc != MIREC_OK) return rc;
    const int lg = row_lg(d4);
    MIREC_CHECK_ARG(lg <= 8);
    hipLaunchKernelGGL(os_sum_kernel, dim3((unsigned)((n_own + (256 >> lg) - 1) / (256 >> lg))),
                       dim3(256), 0, st, b, pos, n_own, (int32_t)d4, lg, q0 > 0 ? 1 : 0,
                       reinterpret_cast<float4 *>(out));
    MIREC_LAUNCH_CHECK();
  }
  return MIREC_OK;
}

extern "C" int mirec_owner_adam(const mirec_row_block_t *blocks, int32_t n_blocks, int64_t lo,
                                int64_t n_own, int32_t dim, float *param, float *exp_avg,
                                float *exp_avg_sq, const float *coef, int64_t n_user,
                                const mirec_adam_hparams_t *h, float *sumsq, float *norms,
                                void *workspace, size_t workspace_bytes, mirec_stream_t stream) {
  MIREC_CHECK_ARG(n_blocks >= 0 && n_blocks <= kOsMax && n_own >= 0 && dim > 0 &&
                  dim % 4 == 0 && h);
  MIREC_CHECK_ARG(n_blocks == 0 || blocks);
  MIREC_CHECK_ARG((norms == nullptr) == (sumsq == nullptr));
  if (n_own == 0) return MIREC_OK;
  MIREC_CHECK_ARG(param && exp_avg && exp_avg_sq && workspace);
  MIREC_CHECK_ARG((((uintptr_t)param | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) & 15u) == 0);
  if ((int64_t)workspace_bytes < mirec_owner_sum_workspace(n_blocks, n_own))
    return MIREC_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int32_t *pos = static_cast<int32_t *>(workspace);
  OsBlocks b;
  const int rc = os_blocks(blocks, 0, n_blocks, lo, n_own, pos, st, b);
  if (rc != MIREC_OK) return rc;
  const int64_t n4 = n_own * (dim / 4);
  const unsigned nblk = tg_blocks(n4);
  hipLaunchKernelGGL(os_adam_kernel, dim3(nblk), dim3(256), 0, st, b, pos, n_own, param, exp_avg,
                     exp_avg_sq, coef, n_user, dim / 4, pow2_shift(dim / 4), *h, sumsq);
  MIREC_LAUNCH_CHECK();
  if (norms) {
    hipLaunchKernelGGL(tg_norm_final_kernel, dim3(1), dim3(1024), 0, st, sumsq, (int64_t)nblk,
                       norms);
    MIREC_LAUNCH_CHECK();
  }
  return MIREC_OK;
}
