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
#include <algorithm>
#include <climits>

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

// ------------------------------------------------------- streaming score top-k
// SURVEY K8 without the [n_eval x M] rating matrix: scores U_b · Iᵀ are
// produced tile by tile on MFMA (v_mfma_f32_32x32x2_f32) and filtered into
// per-user candidate buffers as they are made; nothing of the score matrix
// reaches HBM.
//
// Stage 1, workgroup (64 users, one chunk of the items), two waves of 32
// users.  Lane (i, h) of a wave: user i, k-slice h of every MFMA; the user's
// embedding stays in registers (the B operand, D/2 floats), item tiles of 32
// rows stream through LDS (double-buffered, the A operand), so the
// accumulator lane (i, h) holds 16 item scores of user i.  A score enters the
// user's LDS candidate buffer (64 entries, LDS atomic slot) only if it beats
// the user's current k-th best (kept per lane after each compaction); a
// train positive scores -1024 (trainer.py:132-137), checked by binary search
// in the user's sorted CSR row only for a score that would otherwise enter.
// When a user's buffer could overflow on the next tile, the wave sorts it
// (bitonic across the 64 lanes), keeps the best k and raises the threshold;
// at the chunk's end every user's best k go to the partial list
// [n_eval][n_chunks][k].  Expected insertions per user ~ k (1 + ln(M/k)).
// Stage 2: one wave per user merges its n_chunks x k partial entries (as
// mirec_topk_masked's lane lists).  Order: score descending, ties to the
// lower item id — deterministic, independent of insertion order.
constexpr int kStUsers = 64;  // users per workgroup (2 waves of 32)
// candidate slots per user: k + 32 at least (after a compaction the k best
// stay and a tile brings up to 32 more); 52 for k <= 20 fits four
// workgroups per CU at D <= 64 (39.9 KB of LDS), 64 otherwise (three)
constexpr int kStCapSmall = 52, kStCapLarge = 64, kStCapSmallK = 20;
constexpr int kStMaxChunk = 65536;  // items per chunk: slot ids are 16-bit offsets
constexpr int kStTile = 32;   // items per MFMA tile

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32x2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Is item node `node` in user u's train row?  (sorted copy of the row when
// the CSR carries one, else a scan)
__device__ __forceinline__ bool user_has(const int64_t *__restrict__ rowptr,
                                         const int32_t *__restrict__ col,
                                         const int32_t *__restrict__ sorted, int64_t n_sorted,
                                         int64_t u, int32_t node) {
  const int64_t beg = rowptr[u], deg = rowptr[u + 1] - beg;
  if (sorted != nullptr && u < n_sorted) {
    const int32_t *a = sorted + (beg - rowptr[0]);
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

// Train positives of a user slot inside the workgroup's item chunk, kept in
// LDS (at most kStPos; a user with more falls back to the binary search of
// its CSR row in global memory): a candidate's mask test is then a scan of
// a few LDS words instead of dependent global loads.  (Per C2 user ~20
// positives over 100 K items, ~2 inside one chunk.)
constexpr int kStPos = 8;

// LDS visibility among the lanes of one wave (the candidate buffers are
// wave-private): the wave's LDS operations complete in order, the fences
// keep the compiler from moving accesses across.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// x of lane (lane ^ stride), stride a power of two < 64, on the VALU instead
// of the LDS crossbar (ds_bpermute: a round trip per exchange, 42 dependent
// ones per sort): DPP quad_perm for 1 and 2; row_half_mirror then a
// reversing quad_perm for 4 (i -> 7 - i within 8, then within 4: i ^ 4);
// row_ror:8 for 8 (within 16: i + 8 = i ^ 8); v_permlane16_swap /
// v_permlane32_swap (gfx950) for 16 / 32, each lane taking the half it
// lacks.
__device__ __forceinline__ int lane_xor(int x, int stride) {
  const int lane = threadIdx.x & 63;
  switch (stride) {
    case 1: return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    case 2: return __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    case 4: {
      const int h = __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false);  // row_half_mirror
      return __builtin_amdgcn_mov_dpp(h, 0x1B, 0xF, 0xF, false);          // quad_perm [3,2,1,0]
    }
    case 8: return __builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, false);  // row_ror:8
    case 16: {
      const auto r = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
      return (int)((lane & 16) ? r[0] : r[1]);
    }
    default: {
      const auto r = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)x, false, false);
      return (int)((lane & 32) ? r[0] : r[1]);
    }
  }
}

// Bitonic sort of one (value, index) pair per lane over the wave, best first.
__device__ __forceinline__ void wave_sort_desc(float &v, int &ix) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const float ov = __int_as_float(lane_xor(__float_as_int(v), stride));
      const int oi = lane_xor(ix, stride);
      const bool up = ((lane & size) == 0);    // this lane's block sorts best-first
      const bool lower = (lane & stride) == 0;  // the lane keeps the better of the pair
      const bool mine_better = better(v, ix, ov, oi);
      const bool keep_mine = (lower == up) ? mine_better : !mine_better;
      if (!keep_mine) {
        v = ov;
        ix = oi;
      }
    }
  }
}

// (Score tiles on the bf16 MFMA pipe through the exact three-term split of
// gemm.hip passed the float64 near-tie check but measured slower at C2, 6.73
// vs 5.69 ms per 10 K users: its bf16 planes take 62.7 KB of LDS per
// workgroup, two per CU instead of three)

template <int D, int CAP>
__global__ __launch_bounds__(128) void score_topk_kernel(
    const float *__restrict__ U, int64_t n_eval, const float *__restrict__ I, int64_t m_items,
    const int32_t *__restrict__ users, const int64_t *__restrict__ rowptr,
    const int32_t *__restrict__ col, const int32_t *__restrict__ sorted, int64_t n_sorted,
    int64_t n_users, int k, int64_t chunk, float *__restrict__ part_val,
    int32_t *__restrict__ part_idx) {
  constexpr int LD = D + 4;
  constexpr int KS = D / 2;  // MFMA steps
  // D > 128: the users' rows live in LDS (their register image would take
  // D/2 VGPRs) and the B operand is read from there, four k-steps per
  // float4; the item tile is then single-buffered (LDS 132 KB: one
  // workgroup per CU).  k-step s of lane half h covers dim h·D/2 + s; A and
  // B use the same map.
  constexpr bool UL = D > 128;
  constexpr int NB = UL ? 1 : 2;
  constexpr int kSI = kStTile * LD;  // floats per buffer
  __shared__ __attribute__((aligned(16))) float sI[NB][kSI];
  __shared__ __attribute__((aligned(16))) float sU[UL ? kStUsers * LD : 4];
  __shared__ float cv[kStUsers][CAP];
  __shared__ uint16_t ci[kStUsers][CAP];  // item - it0 (chunk <= kStMaxChunk items)
  // per user its train positives inside the chunk (kStPos at most; npos >
  // kStPos = overflow: the global binary search)
  __shared__ int posl[kStUsers][kStPos];
  __shared__ int npos[kStUsers];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int ul = 32 * w + i;  // user slot in the workgroup
  const int64_t ub = (int64_t)blockIdx.x * kStUsers + ul;
  const bool uok = ub < n_eval;
  const int64_t it0 = (int64_t)blockIdx.y * chunk;
  const int64_t it1 = min(m_items, it0 + chunk);
  // the user's embedding as the B operand: ue[s] = U[ub][h D/2 + s]
  float ue[UL ? 1 : KS];
  if constexpr (!UL) {
#pragma unroll
    for (int s4 = 0; s4 < KS / 4; ++s4) {
      const float4 x = uok ? ld4(U + ub * D + h * KS + 4 * s4) : f4_zero();
      ue[4 * s4] = x.x, ue[4 * s4 + 1] = x.y, ue[4 * s4 + 2] = x.z, ue[4 * s4 + 3] = x.w;
    }
  } else {
    for (int e = t; e < kStUsers * D / 4; e += 128) {
      const int row = e / (D / 4), c4 = e % (D / 4);
      const int64_t b = (int64_t)blockIdx.x * kStUsers + row;
      st4(sU + row * LD + 4 * c4, b < n_eval ? ld4(U + b * D + 4 * c4) : f4_zero());
    }
  }
  if (t < kStUsers) npos[t] = 0;
  __syncthreads();
  if (rowptr != nullptr && users != nullptr) {
    // two threads per user slot walk its row
    const int u = t >> 1;
    const int64_t b = (int64_t)blockIdx.x * kStUsers + u;
    if (b < n_eval) {
      const int64_t us = users[b];
      for (int64_t e = rowptr[us] + (t & 1); e < rowptr[us + 1]; e += 2) {
        const int64_t item = (int64_t)col[e] - n_users;
        if (item < it0 || item >= it1) continue;
        const int q = atomicAdd(&npos[u], 1);
        if (q < kStPos) posl[u][q] = (int)item;
      }
    }
  }
  float thr = -INFINITY;  // the user's k-th best score so far (after the last compaction)
  // item tile loader: 32 rows x D floats, float4 per thread (D % 4 == 0)
  constexpr int PER = (kStTile * D / 4 + 127) / 128;
  auto load = [&](int64_t base, float4 (&r)[PER]) {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = t + 128 * q, row = e / (D / 4), c4 = e % (D / 4);
      r[q] = (e < kStTile * D / 4 && base + row < it1) ? ld4(I + (base + row) * D + 4 * c4)
                                                         : f4_zero();
    }
  };
  auto stage = [&](int buf, const float4 (&r)[PER]) {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = t + 128 * q, row = e / (D / 4), c4 = e % (D / 4);
      if (e >= kStTile * D / 4) continue;
      st4(sI[buf] + row * LD + 4 * c4, r[q]);
    }
  };
  // user slot u's buffer entry of this lane, with the train-positive mask
  // applied now (entries go in with their raw scores; one parallel round of
  // membership tests per compaction instead of one per insertion)
  // cn = the entries in user i's buffer, kept in a register of both its
  // lanes (only they insert for it; a compaction run by the whole wave hands
  // the count back to them): no LDS counter, no atomics
  int cn = 0;
  auto entry = [&](int u, int n, float &v, int &ix) {
    v = lane < n ? cv[u][lane] : -INFINITY;
    ix = lane < n ? (int)it0 + ci[u][lane] : INT_MAX;
    const int64_t b = (int64_t)blockIdx.x * kStUsers + u;
    if (lane < n && rowptr != nullptr && users != nullptr && b < n_eval && v != -1024.f) {
      const int np = npos[u];
      bool hit = false;
      if (np <= kStPos) {
#pragma unroll
        for (int q = 0; q < kStPos; ++q) hit |= q < np && posl[u][q] == ix;
      } else {
        hit = user_has(rowptr, col, sorted, n_sorted, users[b], (int32_t)(n_users + ix));
      }
      if (hit) v = -1024.f;
    }
  };
  // keep the best k of user slot `u` (one wave, lanes = entries)
  auto compact = [&](int u, int n) {
    float v;
    int ix;
    entry(u, n, v, ix);
    wave_sort_desc(v, ix);
    if (lane < k) {
      cv[u][lane] = v;
      ci[u][lane] = (uint16_t)(ix - (int)it0);
    }
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k - 1));  // (-inf while fewer than k)
  };
  float4 rg[PER];
  int cur = 0;
  if (it0 < it1) {
    load(it0, rg);
    stage(0, rg);
  }
  __syncthreads();
  for (int64_t base = it0; base < it1; base += kStTile) {
    const bool more = base + kStTile < it1;
    if (more) load(base + kStTile, rg);  // in flight during the products
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    if constexpr (!UL) {
      // four k-steps per 16-byte LDS read (row stride D + 4: the 16 lanes of
      // a read phase hit distinct 4-bank groups)
      const float *arow = sI[cur] + i * LD + h * KS;
#pragma unroll
      for (int s4 = 0; s4 < KS / 4; ++s4) {
        const float4 a = ld4(arow + 4 * s4);
        acc = mfma32x2(a.x, ue[4 * s4], acc);
        acc = mfma32x2(a.y, ue[4 * s4 + 1], acc);
        acc = mfma32x2(a.z, ue[4 * s4 + 2], acc);
        acc = mfma32x2(a.w, ue[4 * s4 + 3], acc);
      }
    } else {
      const float *arow = sI[cur] + i * LD + h * KS;
      const float *brow = sU + ul * LD + h * KS;
#pragma unroll 8
      for (int s4 = 0; s4 < KS / 4; ++s4) {
        const float4 a = ld4(arow + 4 * s4), bq = ld4(brow + 4 * s4);
        acc = mfma32x2(a.x, bq.x, acc);
        acc = mfma32x2(a.y, bq.y, acc);
        acc = mfma32x2(a.z, bq.z, acc);
        acc = mfma32x2(a.w, bq.w, acc);
      }
    }
    // candidates: acc[r] = score of item base + (r & 3) + 8 (r >> 2) + 4 h
    // for user i; the test against the user's k-th is conservative (a train
    // positive would score -1024: the mask is applied when the buffer is
    // compacted).  A user's buffer is compacted only when this tile's
    // candidates would not fit (then they are tested again against the
    // raised k-th): a full 64-entry buffer per compaction, not room kept for
    // a whole tile — ~3x fewer compactions.  The buffers are the wave's own
    // (its 32 users): wave-level LDS ordering, no workgroup barrier.
    unsigned bits = 0u;
    // 32-bit item ids (m_items < 2^31).  The test is `score >= k-th` (ties
    // enter too; the compaction orders them exactly), and a masked train
    // positive's -1024 is folded in per lane: any score passes once the k-th
    // is <= -1024.  Bitwise, not short-circuit: no per-score exec-mask
    // branches.  Rows past the chunk (staged as zeros) are cut only on a
    // ragged last tile.
    const int ib = (int)base + 4 * h;
    const bool full = base + kStTile <= it1;
    auto test_tile = [&]() {
      const unsigned low = thr <= -1024.f ? 0xFFFFu : 0u;
      bits = 0u;
#pragma unroll
      for (int r = 0; r < 16; ++r) bits |= (unsigned)(acc[r] >= thr) << r;
      bits |= low;
      if (!full) {
        const int lim = (int)(it1 - base);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if ((r & 3) + 8 * (r >> 2) + 4 * h >= lim) bits &= ~(1u << r);
      }
      if (!uok) bits = 0u;
    };
    test_tile();
    const int mine = __builtin_popcount(bits);
    const int both = mine + lane_xor(mine, 32);  // the user's two lane halves (permlane32)
    unsigned long long need = __ballot(h == 0 && cn + both > CAP);
    if (need) {
      while (need) {
        const int j = __ffsll(need) - 1;
        need &= need - 1;
        const int nj = __builtin_amdgcn_readlane(cn, j);  // (j uniform)
        const float th = compact(32 * w + j, nj);
        if (i == j) {
          thr = th;
          cn = min(nj, k);
        }
      }
      wave_lds_sync();
      test_tile();
    }
    // insertion: every lane takes its lowest remaining candidate per round,
    // so the wave runs max(candidates per lane) rounds (~1-3), not one per
    // tile position some lane has
    // (the user's two lanes take slots cn and cn + 1 in a round where both
    // insert: lane half 1 after half 0)
    while (__ballot(bits != 0u)) {
      const int take = bits != 0u ? 1 : 0;
      const int other = lane_xor(take, 32);
      if (take) {
        const int r = __builtin_ctz(bits);
        bits &= bits - 1u;
        float sc = acc[0];
#pragma unroll
        for (int q = 1; q < 16; ++q) sc = r == q ? acc[q] : sc;
        const int slot = cn + (h ? other : 0);
        cv[ul][slot] = sc;
        ci[ul][slot] = (uint16_t)(ib - (int)it0 + (r & 3) + 8 * (r >> 2));
      }
      cn += take + other;
    }
    wave_lds_sync();
    if constexpr (UL) __syncthreads();  // the single buffer's reads done
    if (more) stage(UL ? 0 : cur ^ 1, rg);
    __syncthreads();  // the next tile staged; (double buffer) this tile's reads done
    if constexpr (!UL) cur ^= 1;
  }
  // final: every user's best k of this chunk
  const int64_t n_chunks = gridDim.y;
  for (int j = 0; j < 32; ++j) {
    const int u = 32 * w + j;
    const int64_t b = (int64_t)blockIdx.x * kStUsers + u;
    if (b >= n_eval) break;
    float v;
    int ix;
    entry(u, __builtin_amdgcn_readlane(cn, j), v, ix);
    wave_sort_desc(v, ix);
    if (lane < k) {
      part_val[(b * n_chunks + blockIdx.y) * k + lane] = v;
      part_idx[(b * n_chunks + blockIdx.y) * k + lane] = ix;
    }
  }
}

// Stage 2: one wave per user over its n_chunks x k partial entries.
template <int KMAX>
__global__ __launch_bounds__(64) void topk_merge_kernel(const float *__restrict__ part_val,
                                                        const int32_t *__restrict__ part_idx,
                                                        int64_t n_eval, int64_t n_part, int k,
                                                        int32_t *__restrict__ topk_idx,
                                                        float *__restrict__ topk_val) {
  __shared__ float s_val[64 * KMAX];
  __shared__ int s_idx[64 * KMAX];
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  float vals[KMAX];
  int idxs[KMAX];
#pragma unroll
  for (int q = 0; q < KMAX; ++q) {
    vals[q] = -INFINITY;
    idxs[q] = INT_MAX;
  }
  float thr = -INFINITY;
  int thr_i = INT_MAX;
  for (int64_t e = lane; e < n_part; e += 64) {
    const float x = part_val[b * n_part + e];
    const int j = part_idx[b * n_part + e];
    if (better(x, j, thr, thr_i)) insert_sorted<KMAX>(vals, idxs, k, x, j, thr, thr_i);
  }
#pragma unroll
  for (int q = 0; q < KMAX; ++q) {
    s_val[lane * KMAX + q] = vals[q];
    s_idx[lane * KMAX + q] = idxs[q];
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
      for (int q = 0; q < KMAX; ++q) {
        if (q < k) {
          const bool ta = better(av[pa], ai[pa], bv[pb], bi[pb]);
          ov[q] = ta ? av[pa] : bv[pb];
          oi[q] = ta ? ai[pa] : bi[pb];
          pa += ta ? 1 : 0;
          pb += ta ? 0 : 1;
        }
      }
    }
    __syncthreads();
    if (lane < active) {
#pragma unroll
      for (int q = 0; q < KMAX; ++q)
        if (q < k) {
          s_val[lane * KMAX + q] = ov[q];
          s_idx[lane * KMAX + q] = oi[q];
        }
    }
    __syncthreads();
  }
  for (int q = lane; q < k; q += 64) {
    topk_idx[b * k + q] = s_idx[q];
    if (topk_val != nullptr) topk_val[b * k + q] = s_val[q];
  }
}

// Workgroups of score_topk_kernel<D, CAP> resident on the chip at once (CUs
// x the occupancy its LDS / registers allow: 4 / 3 per CU at D <= 64 with
// the small / large buffers, 2 at 128, 1 at 256), from the runtime, once per
// instantiation.
static int64_t st_slots(int D, int k);
static int st_cap(int k) { return k <= kStCapSmallK ? kStCapSmall : kStCapLarge; }

// Items per stage-1 workgroup.  The grid is (user groups) x (item chunks) and
// every workgroup of a chunk takes the same time, so the launch lasts
// ceil(workgroups / slots) rounds of one chunk: pick the chunk count that
// minimises rounds x (tiles per chunk + a chunk's fixed cost, ~24 tiles of
// final sorts and partial writes), at least 32 tiles per chunk, fewest
// chunks on a tie (less stage-2 merging).  (C2, 10 K users x 100 K items at
// D = 64: 157 user groups, 768 slots -> 9 chunks in 2 full rounds instead of
// the 7 = 1.43 rounds of a fixed >= 1024-workgroup rule.)
static void st_chunks(int64_t n_eval, int64_t m_items, int D, int k, int64_t *chunk,
                      int64_t *n_chunks) {
  const int64_t ut = (n_eval + kStUsers - 1) / kStUsers;
  const int64_t slots = std::max<int64_t>(1, st_slots(D, k));
  const int64_t tiles_all = (m_items + kStTile - 1) / kStTile;
  const int64_t max_n = std::max<int64_t>(1, tiles_all / 32);
  // at most kStMaxChunk items per chunk (16-bit candidate ids)
  const int64_t min_n = (tiles_all + kStMaxChunk / kStTile - 1) / (kStMaxChunk / kStTile);
  int64_t best_n = min_n, best_cost = -1;
  for (int64_t n = min_n; n <= std::max<int64_t>(min_n, std::min<int64_t>(max_n, 256)); ++n) {
    const int64_t tiles = (tiles_all + n - 1) / n;
    const int64_t rounds = (ut * n + slots - 1) / slots;
    const int64_t cost = rounds * (tiles + 24);
    if (best_cost < 0 || cost < best_cost) {
      best_cost = cost;
      best_n = n;
    }
  }
  const int64_t c = (tiles_all + best_n - 1) / best_n * kStTile;
  *chunk = c;
  *n_chunks = (m_items + c - 1) / c;
}

template <int D, int CAP>
static int64_t st_slots_of() {
  static int64_t slots = -1;
  if (slots < 0) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, score_topk_kernel<D, CAP>, 128, 0) !=
            hipSuccess)
      return 1024;  // no device answer: the old fixed target
    slots = (int64_t)cus * std::max(per, 1);
  }
  return slots;
}

template <int CAP>
static int64_t st_slots_cap(int D) {
  switch (D) {
    case 16: return st_slots_of<16, CAP>();
    case 32: return st_slots_of<32, CAP>();
    case 64: return st_slots_of<64, CAP>();
    case 128: return st_slots_of<128, CAP>();
    default: return st_slots_of<256, CAP>();
  }
}

static int64_t st_slots(int D, int k) {
  return st_cap(k) == kStCapSmall ? st_slots_cap<kStCapSmall>(D) : st_slots_cap<kStCapLarge>(D);
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

extern "C" int64_t mirec_score_topk_workspace(int64_t n_eval, int64_t m_items, int32_t k) {
  using namespace mirec;
  if (n_eval < 0 || m_items <= 0 || k < 1 || k > 32) return -1;
  // the largest partial-list count over the dims the kernel takes (the
  // chunking follows the dim's occupancy; the workspace call has no dim)
  int64_t most = 1;
  for (int D : {16, 32, 64, 128, 256}) {
    int64_t chunk, n_chunks;
    st_chunks(std::max<int64_t>(n_eval, 1), m_items, D, k, &chunk, &n_chunks);
    most = std::max(most, n_chunks);
  }
  return n_eval * most * k * (int64_t)(sizeof(float) + sizeof(int32_t));
}

extern "C" int mirec_score_topk(const float *user_emb, int64_t n_eval, const float *item_emb,
                                int64_t m_items, int32_t dim, const int32_t *users,
                                const mirec_csr_t *csr, int64_t n_users, int32_t k,
                                int32_t *topk_idx, float *topk_val, void *workspace,
                                size_t workspace_bytes, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(n_eval >= 0 && m_items > 0 && m_items < INT32_MAX && k >= 1 && k <= 32 &&
                  k <= m_items);
  MIREC_CHECK_ARG(dim == 16 || dim == 32 || dim == 64 || dim == 128 || dim == 256);
  MIREC_CHECK_ARG(csr == nullptr || (users && csr->rowptr && csr->col));
  if (n_eval == 0) return MIREC_OK;
  MIREC_CHECK_ARG(user_emb && item_emb && topk_idx && workspace);
  MIREC_CHECK_ARG(((uintptr_t)user_emb | (uintptr_t)item_emb) % 16 == 0);
  const int64_t need = mirec_score_topk_workspace(n_eval, m_items, k);
  if ((int64_t)workspace_bytes < need) return MIREC_ERR_WORKSPACE;
  int64_t chunk, n_chunks;
  st_chunks(n_eval, m_items, dim, k, &chunk, &n_chunks);
  float *pv = static_cast<float *>(workspace);
  int32_t *pi = reinterpret_cast<int32_t *>(pv + n_eval * n_chunks * k);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t *rp = csr ? csr->rowptr : nullptr;
  const int32_t *cl = csr ? csr->col : nullptr;
  const int32_t *so = csr ? csr->col_sorted : nullptr;
  const int64_t ns = csr ? csr->n_sorted : 0;
  const dim3 grid((unsigned)((n_eval + kStUsers - 1) / kStUsers), (unsigned)n_chunks);
#define MIREC_ST_LAUNCH(DD, CC)                                                              \
  hipLaunchKernelGGL((score_topk_kernel<DD, CC>), grid, dim3(128), 0, st, user_emb, n_eval,  \
                     item_emb, m_items, users, rp, cl, so, ns, n_users, (int)k, chunk, pv, pi)
#define MIREC_ST_CASE(DD)                                  \
  case DD:                                                 \
    if (st_cap(k) == kStCapSmall) MIREC_ST_LAUNCH(DD, kStCapSmall); \
    else MIREC_ST_LAUNCH(DD, kStCapLarge);                 \
    break;
  switch (dim) {
    MIREC_ST_CASE(16)
    MIREC_ST_CASE(32)
    MIREC_ST_CASE(64)
    MIREC_ST_CASE(128)
    MIREC_ST_CASE(256)
  }
#undef MIREC_ST_CASE
#undef MIREC_ST_LAUNCH
  MIREC_LAUNCH_CHECK();
  hipLaunchKernelGGL((topk_merge_kernel<64>), dim3((unsigned)n_eval), dim3(64), 0, st, pv, pi,
                     n_eval, n_chunks * k, (int)k, topk_idx, topk_val);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}
