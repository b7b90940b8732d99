// LightGCN propagation on gfx950: CSR segment-gather SpMM with a fused
// layer epilogue.
//
// Replaces PyG LGConv (model/lgcn.py:66,82) / rAdjConv (model/radj.py:28-44):
//   out[i] = sum_{(j -> i)} x[j] / sqrt(deg_i * deg_j)
// which the reference evaluates as a [nnz, D] gather, a scale and an atomic
// scatter-add.  A wave owns G = 64/LPR consecutive rows (LPR = D/4 lanes read
// one neighbour row as float4s: D=64 -> 16 lanes x 16 B = one 256-B row).
// Short rows (degree <= narrow_max) are gathered one per lane group; a wave
// with a longer row walks its rows one at a time with the whole wave: the
// row's column indices are read once, coalesced (64 per load), broadcast
// with ds_bpermute, and G x UNROLL neighbour rows are in flight per
// instruction; groups hold disjoint neighbour subsets in registers and are
// combined with a xor-butterfly.  No atomics, a fixed summation order per
// row (deterministic).
//
// Masks (byte maps over nodes, optional; 1.1 MB at C2, L2-resident):
//   row_mask  rows whose byte is 0 are skipped entirely (nothing written);
//             with frontier row lists the rows come from the lists instead
//             (narrow rows G per wave, wide rows one workgroup each);
//   in_mask   neighbours whose byte is 0 contribute exactly 0 and are not
//             read: the 64 candidates of a chunk are tested at once and the
//             valid ones compacted to the front with ds_permute.
// Frontier pruning uses them to compute only the rows the BPR loss depends
// on; skipped terms are exact zeros, so results equal the dense pass up to
// fp32 summation order (the compaction regroups the surviving neighbours).
//
// Rows longer than csr->split are cut into segments processed by extra waves
// of the same launch (partial sums to scratch) and summed in segment order by
// a finalize launch, so a Zipf-skewed item cannot serialise the grid (the
// row phase leaves them to their segments entirely).
//
// Epilogue (per row, LPR lanes): z = dinv_i * sum + seed[slot_i];
// xs_out = dinv_i * z (next layer's pre-scaled input);
// o = (z + addend)/divisor + seed2[slot_i]; out = o or Adam(param; grad=o).
#include "common.h"

namespace mirec {

struct PropK {
  const int64_t *rowptr;
  const int32_t *col;
  const float *dinv;
  int64_t n_rows;
  int64_t n_seg;
  const int32_t *seg_row;
  const int64_t *seg_beg;
  int32_t split;
  const float *x_in;
  const int32_t *slot;
  const float *seed_in;
  const float *seed;
  const float *addend;
  const float *seed2;
  float divisor;
  float *out;
  float *xs_out;
  float *param;
  float *m;
  float *v;
  mirec_adam_hparams_t adam;
  float *partial;
  const uint8_t *row_mask;
  const uint8_t *in_mask;
  const uint8_t *out_mask;   // rows whose `out` (and addend read) is skipped when 0
  const int32_t *row_list;   // rows to process (deduplicated), or NULL = all rows
  const int32_t *row_count;  // device count of row_list entries
  int64_t row_waves;         // waves of the row phase (host upper bound)
  int32_t narrow_max;        // rows up to this degree are gathered group-per-row
  const int32_t *wide_list;  // rows gathered by a whole workgroup each (list mode)
  const int32_t *wide_count;
};

__device__ __forceinline__ bool bit_set(const uint8_t *bm, int64_t i) { return bm[i] != 0; }

__device__ __forceinline__ void adam_elem(float &p, float &m, float &v, float g,
                                          const mirec_adam_hparams_t &h) {
  // torch.optim.Adam single-tensor path (torch/optim/adam.py:457-547):
  // exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2);
  // denom = sqrt(v)/sqrt(bc2) + eps; p.addcdiv_(m, denom, -lr/bc1) — the
  // shared expression of every Adam kernel (common.h)
  adam1(p, m, v, g, h);
}

// Sum of the input rows listed in col[beg, end) (pre-scaled / raw x dinv_j /
// sparse seeds x dinv_j), restricted to in_mask when MASKED.  Returns this
// lane's group partial (a disjoint subset of the neighbours).
template <int D, int UNROLL, int MODE, bool MASKED>
__device__ __forceinline__ float4 gather_rows(const PropK &a, int64_t beg, int64_t end,
                                              int lane) {
  constexpr int LPR = D / 4;
  constexpr int G = 64 / LPR;
  const int grp = lane / LPR;
  const int sub = lane % LPR;
  float4 acc = f4_zero();
  if (MODE == MIREC_IN_NONE) return acc;
  const float *src = (MODE == MIREC_IN_SPARSE) ? a.seed_in : a.x_in;
  for (int64_t base = beg; base < end; base += 64) {
    int cnt = (int)min((int64_t)64, end - base);
    int myc = lane < cnt ? a.col[base + lane] : 0;
    // SPARSE: the seed-row slot itself is the filter (slot >= 0 <=> node in
    // S), one dependent load less than a byte-map test followed by the slot
    // (with an in_mask, SPARSE tests the byte map first and reads the slot
    // of the hits only: fewer slot reads when many neighbours are seeded)
    const bool slot_filter = MODE == MIREC_IN_SPARSE && a.in_mask == nullptr;
    int myr = slot_filter ? (lane < cnt ? a.slot[myc] : -1) : myc;
    if (MASKED) {
      const bool ok = lane < cnt && (slot_filter ? myr >= 0 : bit_set(a.in_mask, myc));
      const unsigned long long m = __ballot(ok);
      const int nv = __popcll(m);
      if (nv == 0) continue;  // wave-uniform
      if (nv < cnt) {
        const int below = __popcll(m & ((1ull << lane) - 1ull));
        const int dst = ok ? below : nv + (lane - below);
        myc = __builtin_amdgcn_ds_permute(dst << 2, myc);
        if (slot_filter) myr = __builtin_amdgcn_ds_permute(dst << 2, myr);
      }
      cnt = nv;
    }
    if (MODE != MIREC_IN_SPARSE) myr = myc;
    else if (!slot_filter) myr = lane < cnt ? a.slot[myc] : 0;
    float myw = 1.f;
    if (MODE == MIREC_IN_RAW || MODE == MIREC_IN_SPARSE) {
      if (lane < cnt) myw = a.dinv[myc];
    }
    if (MODE == MIREC_IN_SPARSE && myr < 0) {  // byte map set without a seed row
      myr = 0;
      myw = 0.f;
    }
    for (int k = 0; k < cnt; k += G * UNROLL) {
      float4 v[UNROLL];
      float w[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int idx = k + u * G + grp;
        const int j = __shfl(myr, idx & 63);
        w[u] = (MODE != MIREC_IN_PRESCALED) ? __shfl(myw, idx & 63) : 1.f;
        if (idx < cnt)
          v[u] = ld4(src + (int64_t)j * D + sub * 4);
        else
          v[u] = f4_zero();
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        if (MODE != MIREC_IN_PRESCALED)
          acc = f4_fma(w[u], v[u], acc);
        else
          acc = f4_add(acc, v[u]);
      }
    }
  }
  return acc;
}

// Group-per-row gather (short rows): each LPR-lane group owns one row and
// walks its neighbours LPR at a time (one coalesced col load per chunk),
// UNROLL float4 row loads in flight per lane.  G rows progress per wave, so
// latency-bound short rows get G x the memory-level parallelism of the
// wave-per-row path.  Control flow is group-uniform; shuffles stay inside
// the group.
template <int D, int UNROLL, int MODE, bool MASKED>
__device__ __forceinline__ float4 gather_narrow(const PropK &a, int64_t beg, int64_t end,
                                                int lane) {
  constexpr int LPR = D / 4;
  const int grp = lane / LPR;
  const int sub = lane % LPR;
  const int gbase = grp * LPR;
  float4 acc = f4_zero();
  if (MODE == MIREC_IN_NONE) return acc;
  const float *src = (MODE == MIREC_IN_SPARSE) ? a.seed_in : a.x_in;
  for (int64_t c = beg; c < end; c += LPR) {
    int cnt = (int)min((int64_t)LPR, end - c);
    int myc = sub < cnt ? a.col[c + sub] : 0;
    const bool slot_filter = MODE == MIREC_IN_SPARSE && a.in_mask == nullptr;
    int myr = slot_filter ? (sub < cnt ? a.slot[myc] : -1) : myc;
    if (MASKED) {
      const bool ok = sub < cnt && (slot_filter ? myr >= 0 : bit_set(a.in_mask, myc));
      const unsigned long long bal = __ballot(ok);
      const unsigned long long gm =
          (LPR == 64) ? bal : ((bal >> gbase) & ((1ull << LPR) - 1ull));
      const int nv = __popcll(gm);
      if (nv == 0) continue;  // group-uniform
      if (nv < cnt) {
        const int below = __popcll(gm & ((1ull << sub) - 1ull));
        const int dst = gbase + (ok ? below : nv + (sub - below));
        myc = __builtin_amdgcn_ds_permute(dst << 2, myc);
        if (slot_filter) myr = __builtin_amdgcn_ds_permute(dst << 2, myr);
      }
      cnt = nv;
    }
    if (MODE != MIREC_IN_SPARSE) myr = myc;
    else if (!slot_filter) myr = sub < cnt ? a.slot[myc] : 0;
    float myw = 1.f;
    if (MODE == MIREC_IN_RAW || MODE == MIREC_IN_SPARSE) {
      if (sub < cnt) myw = a.dinv[myc];
    }
    if (MODE == MIREC_IN_SPARSE && myr < 0) {  // byte map set without a seed row
      myr = 0;
      myw = 0.f;
    }
    for (int k = 0; k < cnt; k += UNROLL) {
      float4 v[UNROLL];
      float w[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int idx = k + u;
        const int srcl = gbase + (idx & (LPR - 1));
        const int j = __shfl(myr, srcl);
        w[u] = (MODE != MIREC_IN_PRESCALED) ? __shfl(myw, srcl) : 1.f;
        if (idx < cnt)
          v[u] = ld4(src + (int64_t)j * D + sub * 4);
        else
          v[u] = f4_zero();
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        if (MODE != MIREC_IN_PRESCALED)
          acc = f4_fma(w[u], v[u], acc);
        else
          acc = f4_add(acc, v[u]);
      }
    }
  }
  return acc;
}

// Combine the G group partials: afterwards every group holds the row sum.
template <int D>
__device__ __forceinline__ float4 combine_groups(float4 s) {
  constexpr int LPR = D / 4;
#pragma unroll
  for (int m = LPR; m < 64; m <<= 1) s = f4_add(s, f4_shfl_xor(s, m));
  return s;
}

template <int D>
__device__ __forceinline__ void row_epilogue(const PropK &a, int64_t row, float4 s, int sub) {
  const float di = a.dinv[row];
  const int64_t off = row * D + sub * 4;
  float4 z = f4_scale(di, s);
  int sl = -1;
  if (a.slot != nullptr && (a.seed != nullptr || a.seed2 != nullptr)) sl = a.slot[row];
  if (a.seed != nullptr && sl >= 0) z = f4_add(z, ld4(a.seed + (int64_t)sl * D + sub * 4));
  if (a.xs_out != nullptr && a.param == nullptr) st4(a.xs_out + off, f4_scale(di, z));
  if (a.out == nullptr && a.param == nullptr) return;
  if (a.out_mask != nullptr && a.param == nullptr && a.out_mask[row] == 0) return;
  float4 o = z;
  if (a.addend != nullptr) o = f4_add(o, ld4(a.addend + off));
  if (a.divisor != 1.f) o = f4_div(o, a.divisor);
  if (a.seed2 != nullptr && sl >= 0) o = f4_add(o, ld4(a.seed2 + (int64_t)sl * D + sub * 4));
  if (a.param != nullptr) {
    float4 p = ld4(a.param + off), m = ld4(a.m + off), v = ld4(a.v + off);
    adam_elem(p.x, m.x, v.x, o.x, a.adam);
    adam_elem(p.y, m.y, v.y, o.y, a.adam);
    adam_elem(p.z, m.z, v.z, o.z, a.adam);
    adam_elem(p.w, m.w, v.w, o.w, a.adam);
    st4(a.param + off, p);
    st4(a.m + off, m);
    st4(a.v + off, v);
    if (a.out != nullptr) st4(a.out + off, o);
    // with Adam, xs_out receives the pre-scaled UPDATED parameter
    if (a.xs_out != nullptr) st4(a.xs_out + off, f4_scale(di, p));
  } else {
    st4(a.out + off, o);
  }
}

constexpr int kWavesPerBlock = 4;

// Row phase: wave w takes the G rows w*G .. w*G+G-1 (of the row list if
// given).  If all of them have degree <= narrow_max each group gathers its
// own row (gather_narrow); otherwise the wave walks them one by one with the
// whole wave per row (gather_rows).  Segment phase: wave row_waves + s
// gathers segment s of a long row into `partial`.
// With a row list the list length is known only on the device: the grid is
// capped (kListBlocks) and blocks stride over the list's work items, so a
// short list does not pay for its host-side capacity in empty waves.
// MASKED = in_mask filter on neighbours, ROWMASK = row_mask filter on rows
// (separate instantiations so profiles tell full and pruned launches apart).
template <int D, int UNROLL, int MODE, bool MASKED, bool ROWMASK>
__device__ __forceinline__ void prop_work(const PropK &a, int64_t w, int64_t nrows,
                                          int64_t row_waves) {
  constexpr int LPR = D / 4;
  constexpr int G = 64 / LPR;
  constexpr int NARROW_UNROLL = UNROLL < 4 ? 4 : UNROLL;
  const int lane = threadIdx.x & 63;
  const int sub = lane % LPR;
  const int grp = lane / LPR;
  if (w < row_waves) {
    const int64_t idx = w * G + grp;
    bool have = idx < nrows;
    int32_t row = 0;
    if (have) row = (ROWMASK && a.row_list != nullptr) ? a.row_list[idx] : (int32_t)idx;
    if (ROWMASK && have) have = bit_set(a.row_mask, row);
    int64_t beg = 0, end = 0;
    if (have) {
      beg = a.rowptr[row];
      end = a.rowptr[row + 1];
      if (a.split > 0 && end - beg > a.split) {  // segments handle it
        have = false;
        beg = end = 0;  // the narrow gather must not walk the long row
      }
    }
    const int64_t deg = have ? end - beg : 0;
    if (G > 1 && __ballot(deg > a.narrow_max) == 0ull) {
      float4 s = gather_narrow<D, NARROW_UNROLL, MODE, MASKED>(a, beg, end, lane);
      if (have) row_epilogue<D>(a, row, s, sub);
      return;
    }
#pragma unroll 1
    for (int g = 0; g < G; ++g) {
      const int src = g * LPR;
      if (!__shfl((int)have, src)) continue;  // wave-uniform
      const int32_t r = __shfl(row, src);
      const int64_t rb = __shfl((long long)beg, src);
      const int64_t re = __shfl((long long)end, src);
      float4 s = gather_rows<D, UNROLL, MODE, MASKED>(a, rb, re, lane);
      s = combine_groups<D>(s);
      if (lane < LPR) row_epilogue<D>(a, r, s, sub);
    }
  } else {
    const int64_t sg = w - row_waves;
    if (sg >= a.n_seg) return;
    const int64_t row = a.seg_row[sg];
    if (ROWMASK && !bit_set(a.row_mask, row)) return;
    const int64_t beg = a.seg_beg[sg];
    const int64_t end = min(beg + (int64_t)a.split, a.rowptr[row + 1]);
    float4 s = gather_rows<D, UNROLL, MODE, MASKED>(a, beg, end, lane);
    s = combine_groups<D>(s);
    if (lane < LPR) st4(a.partial + sg * D + sub * 4, s);
  }
}

// One row gathered by the whole 256-thread workgroup: wave q takes the q-th
// quarter of the row's entries, the four wave sums are added in wave order
// through LDS (deterministic), wave 0 runs the epilogue.  Block-uniform
// control flow (contains barriers).
template <int D, int UNROLL, int MODE, bool MASKED>
__device__ __forceinline__ void block_row(const PropK &a, int32_t row) {
  constexpr int LPR = D / 4;
  __shared__ float4 red[kWavesPerBlock - 1][LPR];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int sub = lane % LPR;
  const int64_t beg = a.rowptr[row], end = a.rowptr[row + 1];
  if (a.split > 0 && end - beg > a.split) return;  // segments handle it (uniform)
  const int64_t q = (end - beg + kWavesPerBlock - 1) / kWavesPerBlock;
  const int64_t wb = min(beg + wid * q, end), we = min(wb + q, end);
  float4 s = gather_rows<D, UNROLL, MODE, MASKED>(a, wb, we, lane);
  s = combine_groups<D>(s);
  if (wid > 0 && lane < LPR) red[wid - 1][sub] = s;
  __syncthreads();
  if (wid == 0 && lane < LPR) {
#pragma unroll
    for (int k = 0; k < kWavesPerBlock - 1; ++k) s = f4_add(s, red[k][sub]);
    row_epilogue<D>(a, row, s, sub);
  }
  __syncthreads();  // red[] is reused by the block's next row
}

// One row gathered by one wave.
template <int D, int UNROLL, int MODE, bool MASKED>
__device__ __forceinline__ void wave_row(const PropK &a, int32_t row) {
  constexpr int LPR = D / 4;
  const int lane = threadIdx.x & 63;
  const int64_t beg = a.rowptr[row], end = a.rowptr[row + 1];
  if (a.split > 0 && end - beg > a.split) return;  // segments handle it
  float4 s = gather_rows<D, UNROLL, MODE, MASKED>(a, beg, end, lane);
  s = combine_groups<D>(s);
  if (lane < LPR) row_epilogue<D>(a, row, s, lane % LPR);
}

// Grid of the list launches (their row counts live on the device): 4x the
// waves resident at 8 per SIMD.  4096 -> 8192: the row-masked launches
// 0.366 -> 0.357 ms, the SPARSE one 0.224 -> 0.208 ms, C2 4.666 -> 4.630
// ms per step (profiles/round6_ab_list_blocks.txt; 2048: 4.79, 16384: 4.63).
constexpr int64_t kListBlocks = 8192;

// Occupancy floor (waves per SIMD): keeps the register allocator at <= 72
// VGPRs so 7-8 waves per SIMD keep enough gathers in flight.
template <int D, int UNROLL, int MODE, bool MASKED, bool ROWMASK>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7, 8)))
MIREC_NO_PK_F32 void prop_kernel(PropK a) {
  constexpr int G = 64 / (D / 4);
  // wave index made provably uniform (SGPR): loop control stays scalar
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if constexpr (!ROWMASK) {
    prop_work<D, UNROLL, MODE, MASKED, ROWMASK>(a, (int64_t)blockIdx.x * kWavesPerBlock + wid,
                                                a.n_rows, a.row_waves);
  } else {
    if (a.row_list == nullptr) {
      prop_work<D, UNROLL, MODE, MASKED, ROWMASK>(a, (int64_t)blockIdx.x * kWavesPerBlock + wid,
                                                  a.n_rows, a.row_waves);
      return;
    }
    // List mode: the list lengths are known only on the device, so the grid
    // is capped (kListBlocks) and blocks stride over the work: first one
    // block per wide row, then G rows per wave of the narrow list, then the
    // long-row segments.
    // SPARSE launches mostly scan indices (few seeded neighbours): a wave
    // per wide row is enough there; gathering launches use a workgroup.
    constexpr int WPB = (MODE == MIREC_IN_SPARSE) ? kWavesPerBlock : 1;  // wide rows / block
    const int64_t n_wide = a.wide_list != nullptr ? (int64_t)*a.wide_count : 0;
    const int64_t wide_blocks = (n_wide + WPB - 1) / WPB;
    const int64_t nrows = *a.row_count;
    const int64_t row_waves = (nrows + G - 1) / G;
    const int64_t waves = row_waves + a.n_seg;
    const int64_t total = wide_blocks + (waves + kWavesPerBlock - 1) / kWavesPerBlock;
#pragma unroll 1
    for (int64_t b = blockIdx.x; b < total; b += gridDim.x) {
      if (b < wide_blocks) {
        if constexpr (WPB == 1) {
          block_row<D, UNROLL, MODE, MASKED>(a, a.wide_list[b]);
        } else {
          const int64_t i = b * WPB + wid;
          if (i < n_wide) wave_row<D, UNROLL, MODE, MASKED>(a, a.wide_list[i]);
        }
      } else {
        const int64_t w = (b - wide_blocks) * kWavesPerBlock + wid;
        if (w < waves) prop_work<D, UNROLL, MODE, MASKED, ROWMASK>(a, w, nrows, row_waves);
      }
    }
  }
}

// One workgroup per long row: its NG = 256 / LPR lane groups sum the
// segments sg0 + k, sg0 + k + NG, ... (group k, 4 partial rows in flight),
// then group 0 adds the NG group sums in order and runs the epilogue.  A
// fixed two-level order (deterministic); a Zipf hub row of 800 segments is
// 50 loads deep per group instead of a serial walk of 800 dependent loads
// (258 -> ~15 us per launch on the C2 Zipf graph).
template <int D>
__global__ __launch_bounds__(256) MIREC_NO_PK_F32 void prop_finalize(PropK a, const int32_t *long_rows,
                                                     const int64_t *long_segptr, int64_t n_long) {
  constexpr int LPR = D / 4;
  constexpr int NG = 256 / LPR;
  constexpr int kF = 4;  // partial rows in flight per group
  __shared__ float4 red[NG][LPR];
  const int sub = threadIdx.x % LPR, grp = threadIdx.x / LPR;
  const int64_t li = blockIdx.x;
  if (li >= n_long) return;
  const int64_t row = long_rows[li];
  if (a.row_mask != nullptr && !bit_set(a.row_mask, row)) return;
  const int64_t s0 = long_segptr[li], s1 = long_segptr[li + 1];
  float4 s = f4_zero();
  for (int64_t sg = s0 + grp; sg < s1; sg += (int64_t)kF * NG) {
    float4 x[kF];
#pragma unroll
    for (int u = 0; u < kF; ++u) {
      const int64_t q = sg + (int64_t)u * NG;
      x[u] = q < s1 ? ld4(a.partial + q * D + sub * 4) : f4_zero();
    }
#pragma unroll
    for (int u = 0; u < kF; ++u)
      if (sg + (int64_t)u * NG < s1) s = f4_add(s, x[u]);
  }
  red[grp][sub] = s;
  __syncthreads();
  if (grp != 0) return;
  float4 t = red[0][sub];
#pragma unroll
  for (int k = 1; k < NG; ++k) t = f4_add(t, red[k][sub]);
  row_epilogue<D>(a, row, t, sub);
}

template <int D, int UNROLL, int MODE, bool MASKED>
static void launch_main(dim3 grid, hipStream_t st, const PropK &k) {
  if (k.row_mask != nullptr)
    hipLaunchKernelGGL((prop_kernel<D, UNROLL, MODE, MASKED, true>), grid, dim3(256), 0, st, k);
  else
    hipLaunchKernelGGL((prop_kernel<D, UNROLL, MODE, MASKED, false>), grid, dim3(256), 0, st, k);
}

template <int D, int UNROLL>
static int launch_prop(const mirec_csr_t *c, PropK k, int64_t list_cap, int mode,
                       hipStream_t st) {
  constexpr int G = 64 / (D / 4);
  const int64_t rows = k.row_list != nullptr ? list_cap : c->n_rows;
  k.row_waves = (rows + G - 1) / G;
  const int64_t work = k.row_waves + c->n_seg;
  int64_t blocks = (work + kWavesPerBlock - 1) / kWavesPerBlock;
  if (k.row_list != nullptr) {
    if (k.wide_list != nullptr) blocks += list_cap;
    blocks = std::min(blocks, kListBlocks);
  }
  const bool masked = k.in_mask != nullptr;
  if (blocks > 0) {
    const dim3 g((unsigned)blocks);
    if (mode == MIREC_IN_PRESCALED && !masked)
      launch_main<D, UNROLL, MIREC_IN_PRESCALED, false>(g, st, k);
    else if (mode == MIREC_IN_PRESCALED)
      launch_main<D, UNROLL, MIREC_IN_PRESCALED, true>(g, st, k);
    else if (mode == MIREC_IN_RAW && !masked)
      launch_main<D, UNROLL, MIREC_IN_RAW, false>(g, st, k);
    else if (mode == MIREC_IN_RAW)
      launch_main<D, UNROLL, MIREC_IN_RAW, true>(g, st, k);
    else if (mode == MIREC_IN_SPARSE)  // always filtered (by slot >= 0)
      launch_main<D, UNROLL, MIREC_IN_SPARSE, true>(g, st, k);
    else
      launch_main<D, UNROLL, MIREC_IN_NONE, false>(g, st, k);
    MIREC_LAUNCH_CHECK();
  }
  if (c->n_long > 0) {
    hipLaunchKernelGGL((prop_finalize<D>), dim3((unsigned)c->n_long), dim3(256), 0, st, k,
                       c->long_rows,
                       c->long_segptr, c->n_long);
    MIREC_LAUNCH_CHECK();
  }
  return MIREC_OK;
}

// x~ = dinv ⊙ x (row scale), float4.
__global__ __launch_bounds__(256) void prescale_kernel(const float *__restrict__ x,
                                                       const float *__restrict__ dinv, int64_t n4,
                                                       int32_t d4, float *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
    st4(out + 4 * i, f4_scale(dinv[i / d4], ld4(x + 4 * i)));
}

}  // namespace mirec

extern "C" int mirec_propagate(const mirec_csr_t *c, const mirec_prop_t *p,
                               mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(c != nullptr && p != nullptr);
  MIREC_CHECK_ARG(c->rowptr != nullptr && c->dinv != nullptr && c->n_rows >= 0);
  MIREC_CHECK_ARG(c->nnz == 0 || c->col != nullptr);
  if (!dim_supported(p->dim)) return MIREC_ERR_DIM;
  MIREC_CHECK_ARG(p->in_mode >= 0 && p->in_mode <= 3);
  if (p->in_mode == MIREC_IN_SPARSE)
    MIREC_CHECK_ARG(p->slot != nullptr && p->seed_in != nullptr);
  else if (p->in_mode != MIREC_IN_NONE)
    MIREC_CHECK_ARG(p->x_in != nullptr);
  MIREC_CHECK_ARG(p->in_mode != MIREC_IN_NONE || p->in_mask == nullptr);
  MIREC_CHECK_ARG((p->seed == nullptr && p->seed2 == nullptr) || p->slot != nullptr);
  MIREC_CHECK_ARG(p->param == nullptr || (p->exp_avg != nullptr && p->exp_avg_sq != nullptr));
  MIREC_CHECK_ARG(p->divisor != 0.f);
  MIREC_CHECK_ARG(p->row_list == nullptr ||
                  (p->row_count != nullptr && p->row_list_cap >= 0 && p->row_mask != nullptr));
  MIREC_CHECK_ARG(p->wide_list == nullptr || (p->row_list != nullptr && p->wide_count != nullptr));
  if (c->n_seg > 0) {
    MIREC_CHECK_ARG(c->split > 0 && c->seg_row && c->seg_beg && c->long_rows && c->long_segptr);
    if (p->partial == nullptr) return MIREC_ERR_WORKSPACE;
  }
  PropK k;
  k.rowptr = c->rowptr;
  k.col = c->col;
  k.dinv = c->dinv;
  k.n_rows = c->n_rows;
  k.n_seg = c->n_seg;
  k.seg_row = c->seg_row;
  k.seg_beg = c->seg_beg;
  k.split = c->n_seg > 0 ? c->split : 0;
  k.x_in = p->x_in;
  k.slot = p->slot;
  k.seed_in = p->seed_in;
  k.seed = p->seed;
  k.addend = p->addend;
  k.seed2 = p->seed2;
  k.divisor = p->divisor;
  k.out = p->out;
  k.xs_out = p->xs_out;
  k.param = p->param;
  k.m = p->exp_avg;
  k.v = p->exp_avg_sq;
  k.adam = p->adam;
  k.partial = p->partial;
  k.row_mask = p->row_mask;
  k.in_mask = p->in_mask;
  k.out_mask = p->out_mask;
  k.row_list = p->row_list;
  k.row_count = p->row_count;
  k.row_waves = 0;
  k.narrow_max = p->narrow_max;
  k.wide_list = p->wide_list;
  k.wide_count = p->wide_count;
  const int64_t cap = p->row_list_cap;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (p->dim) {
    case 4: return launch_prop<4, 1>(c, k, cap, p->in_mode, st);
    case 8: return launch_prop<8, 1>(c, k, cap, p->in_mode, st);
    case 16: return launch_prop<16, 1>(c, k, cap, p->in_mode, st);
    case 32: return launch_prop<32, 2>(c, k, cap, p->in_mode, st);
    case 64: return launch_prop<64, 4>(c, k, cap, p->in_mode, st);
    case 128: return launch_prop<128, 4>(c, k, cap, p->in_mode, st);
    case 256: return launch_prop<256, 8>(c, k, cap, p->in_mode, st);
  }
  return MIREC_ERR_DIM;
}

extern "C" int mirec_prescale(const float *x, const float *dinv, int64_t n_rows, int32_t dim,
                              float *out, mirec_stream_t stream) {
  using namespace mirec;
  MIREC_CHECK_ARG(x && dinv && out && n_rows >= 0);
  if (!dim_supported(dim)) return MIREC_ERR_DIM;
  const int64_t n4 = n_rows * dim / 4;
  if (n4 == 0) return MIREC_OK;
  const int64_t blocks = std::min<int64_t>((n4 + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(prescale_kernel, dim3(blocks), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), x, dinv, n4, dim / 4, out);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}
