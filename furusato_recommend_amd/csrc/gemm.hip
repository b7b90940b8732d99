// f32 GEMMs of the Linear layers of the SASRec block and the GraphSAGE hop
// (model/sasrec.py:385-421, model/graphsage.py:311-324: nn.Linear forward,
// input gradient and weight / bias gradient) on gfx950 MFMA.
//
// The token-row activations are tall and thin (tens of thousands of rows x
// d = 128..384), so two shapes cover every product:
//   gemm_nt:  C[n, No] = A[n, Kr] · B[No, Kr]ᵀ (+ bias[No])
//             forward y = x Wᵀ + b, and dX = dY W with B = Wᵀ (a copy of the
//             small weight), so both operands are k-contiguous rows.
//   gemm_tn:  C[M, No] = Σ_r A[r, M] B[r, No] over the n rows (+ the column
//             sums of A): dW = dYᵀ X and db = Σ_r dY.  The long reduction is
//             cut into row slices (one workgroup per slice and 128 x 128
//             output tile, partial tiles in a workspace) and the slices are
//             summed in a fixed order by a second kernel: deterministic.
// The f32 products run on the bf16 MFMA pipe as an exact three-term split
// (below: six v_mfma_f32_32x32x16_bf16 per 16-deep block, f32-class error),
// the operands staged once per element as bf16 planes in LDS.  A
// 256-thread workgroup owns a 128 x 128 output tile, each of its 4 waves a
// 64 x 64 quarter (2 x 2 MFMA tiles, 64 accumulator registers); the k loop
// runs in chunks of 32 staged through LDS with the next chunk's global loads
// in flight (in registers) while the current chunk is multiplied.  At K =
// 128 with enough rows (the QKV in-projection) gemm_nt runs a resident-B
// form instead: each workgroup splits its 128-column slice of B once into
// LDS and its waves stream 32-row units of A (gemm_nt_res_kernel, below).
//
#include <algorithm>

#include "common.h"

namespace mirec {


// ---------------------------------------------- f32 products on bf16 MFMA
// Every f32 operand is split exactly into three
// bf16 terms, x = x_h + x_m + x_l (round-to-nearest at each stage; the
// residuals x - x_h and (x - x_h) - x_m are exact in f32, |x_m| <= 2^-8 |x|,
// |x_l| <= 2^-16 |x|, and x_l carries the rest to 2^-25 |x|), and a·b is
// taken as the six products whose size is at least 2^-16 |ab|:
//   a_l b_h + a_h b_l + a_m b_m + a_m b_h + a_h b_m + a_h b_h
// on v_mfma_f32_32x32x16_bf16 (bf16 x bf16 products are exact in f32, f32
// accumulate).  The dropped terms (a_m b_l, a_l b_m, a_l b_l) are below
// 2^-23 |ab|: the error per product is that of one f32 rounding, i.e. the
// f32 GEMM's own accuracy (tests against float64 at 1e-6), at 6 x 32 = 192
// MFMA cycles per 32x32x16 block instead of 8 x 64 = 512 with
// v_mfma_f32_32x32x2_f32 (MI355X_MICROARCH.md cycle constants).
// (bf16x8, Split3, pk_bf16, split3: common.h)

// (mfma_x6, x6_k: common.h)

// LDS visibility among the lanes of one wave (the epilogue slabs are
// wave-private: no workgroup barrier)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int kTile = 128;   // output tile edge
constexpr int kChunk = 32;          // k per LDS stage
constexpr int kC4 = kChunk / 4;        // float4 per staged row (gemm_nt)
constexpr int kLdNT = kChunk + 4;   // gemm_nt LDS row stride [row][k]: 16-B reads, 4-bank groups
constexpr int kLdO = 40;            // epilogue slab stride [row][col]: lane halves (rows
                                    // r, r + 4) 32 banks apart, 16-B row reads

// bf16 planes ([row][k] operands of gemm_nt): the staging thread splits
// its float4s once and stores the three terms as bf16 planes
// [3][rows][kLdP], each 16-deep k block permuted so that a lane half's 8 values (x6_k order) are contiguous: one 16-byte
// read per plane and operand.  Row stride 80 B: the 16 lanes of a read phase
// hit distinct 4-bank groups.  Halves the split VALU of a wave-side split
// (every element would be split by both waves that read it).
constexpr int kLdP = kChunk + 8;  // bf16 units
constexpr int kLdK = kTile + 32;  // bf16 units (k-major planes, below)
template <int BM>
constexpr int nt_lds_floats() {
  // [row][k] planes of A and B, or of A with the [k][n] planes of B
  constexpr int pl = 3 * BM * kLdP / 2 +
                     (3 * kTile * kLdP > 3 * kChunk * kLdK ? 3 * kTile * kLdP : 3 * kChunk * kLdK) / 2;
  return pl > (BM + kTile) * kLdNT ? pl : (BM + kTile) * kLdNT;
}

struct Split3x4 {
  uint2 h, m, l;
};
// a float4 -> three planes of 4 packed bf16 (the split3 arithmetic)
__device__ __forceinline__ Split3x4 split3x4(float4 v) {
  const float x[4] = {v.x, v.y, v.z, v.w};
  uint32_t H[2], M[2], L[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const float a = x[2 * p], b = x[2 * p + 1];
    const uint32_t ph = pk_bf16(a, b);
    const float ra = a - __uint_as_float(ph << 16), rb = b - __uint_as_float(ph & 0xffff0000u);
    const uint32_t pm = pk_bf16(ra, rb);
    const float sa = ra - __uint_as_float(pm << 16), sb = rb - __uint_as_float(pm & 0xffff0000u);
    H[p] = ph;
    M[p] = pm;
    L[p] = pk_bf16(sa, sb);
  }
  return Split3x4{make_uint2(H[0], H[1]), make_uint2(M[0], M[1]), make_uint2(L[0], L[1])};
}
// bf16 position of float4 column c4 (k = 4 c4 .. +3) of a staged chunk row
__device__ __forceinline__ int plane_pos(int c4) {
  return (c4 >> 2) * 16 + 8 * (c4 & 1) + 4 * ((c4 >> 1) & 1);
}

// k-major operands ([k][n] B of gemm_nn / the fused dX kernel, both operands
// of gemm_tn): planes [3][kChunk][kLdK] in the natural [k][col] order (a
// float4 of 4 columns -> one 8-byte store per plane) read back with the
// gfx950 transposing LDS read ds_read_b64_tr_b16: per 16-lane group a 4-row
// x 16-column block arrives column-major, lane i holding column i's 4 rows —
// two reads (rows 4h.. and 8 + 4h..) give a lane half h its 8 values in the
// x6_k order.  Row stride 320 B (80 dwords = 16 mod 64): the 32 lanes of a
// half (4 rows x 2 groups x 4 column quads) hit 64 distinct banks.
typedef short v4i16 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4i16 lds_tr16(const uint16_t *p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4i16 *)(const_cast<uint16_t *>(p)));
}
// the 32x32x16 operand of columns [c0, c0 + 32) of one plane, k block s16
__device__ __forceinline__ bf16x8 tr_operand(const uint16_t *plane, int c0, int s16, int lane) {
  const int G = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3, h = G >> 1;
  const uint16_t *a = plane + (s16 * 16 + 4 * h + q) * kLdK + c0 + 16 * (G & 1) + 4 * pq;
  const v4i16 x = lds_tr16(a), y = lds_tr16(a + 8 * kLdK);
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const v8i16 v = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ Split3 tr_split3(const uint16_t *planes, int plane_stride, int c0,
                                            int s16, int lane) {
  return Split3{tr_operand(planes, c0, s16, lane), tr_operand(planes + plane_stride, c0, s16, lane),
                tr_operand(planes + 2 * plane_stride, c0, s16, lane)};
}

// ------------------------------------------------------------------ gemm_nt
// Workgroup (tile_m, tile_n): rows [BM tile_m, +BM) of C, columns
// [128 tile_n, +128); waves 2 x 2, each BM/2 x 64 (BM/64 x 2 MFMA tiles).
// LDS: bf16 planes of A [3][BM][kLdP] and B [3][128][kLdP] (k-contiguous
// rows) or [3][kChunk][kLdK] ([k][n] B).  PF chunks of global
// loads are in flight ahead of the one being multiplied (register staging).
//
// Fused forms (the GraphSAGE hop, model/graphsage.py:314-315, without the
// concatenation): A may be two row-major blocks side by side — columns
// [0, Ks) from A (row stride Ks) and [Ks, Kr) from A2 (row stride Kr - Ks);
// Amask (same layout as a single A) zeroes A elements whose mask is <= 0 (the
// ReLU backward, dY * (y > 0), applied as dY is loaded); C may be split the
// same way at column Ns into C / C2; relu applies max(., 0) after the bias.
//
// B layout: [No, Kr] rows (k contiguous: C = A Bᵀ, a Linear forward with B =
// W), or with bkn [Kr, No] rows (n contiguous: C = A B, the input gradient
// dX = dY W of a Linear with B = W, no transposed copy), staged in LDS as
// [n][k] or [k][n] respectively.
struct NtArgs {
  const float *A2;
  const float *Amask;
  float *C2;
  int Ks, Ns, relu, bkn;
};

// The k loop of gemm_nt (shared by the plain and the LayerNorm epilogues):
// acc[TM][2] of wave (wm, wn) over output rows [m0, +BM), columns [n0, +128);
// smem holds (BM + 128) * kLdNT floats.
template <int BM, int PF, bool BKN, bool MASK = false>
__device__ __forceinline__ void nt_mainloop(float *smem, const float *__restrict__ A,
                                            const float *__restrict__ B, int64_t n, int Kr,
                                            int No, const NtArgs &fx, int64_t m0, int n0,
                                            f32x16 (&acc)[BM / 64][2]) {
  constexpr int TM = BM / 64;        // 32-row MFMA tiles per wave
  constexpr int QA = BM * kC4 / 256;     // float4 of A per thread per chunk
  constexpr int QB = kTile * kC4 / 256;  // float4 of B per thread per chunk
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int wm = w >> 1, wn = w & 1;
  // element e = t + 256 q: row e / kC4, float4 column e % kC4.  Rows past n
  // load row n - 1 (unconditional loads: counted waits); their products are
  // never stored (or stored as row n - 1's own values, gemm_nt_kernel).  The
  // ReLU mask is loaded beside A and applied when the chunk is staged.
  float4 ra[PF][QA], rb[PF][QB], rm[MASK ? PF : 1][QA];
  auto load = [&](int p, int k0) {
    // A columns [k0, k0 + 32): from A, or from A2 past Ks (chunk-uniform)
    const float *Ab = A;
    int lda = Kr, kc = k0;
    if (fx.A2 != nullptr) {
      if (k0 < fx.Ks) {
        lda = fx.Ks;
      } else {
        Ab = fx.A2;
        lda = Kr - fx.Ks;
        kc = k0 - fx.Ks;
      }
    }
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int e = t + 256 * q, r = e / kC4, c4 = e % kC4;
      const int64_t row = min(m0 + r, n - 1);
      ra[p][q] = ld4(Ab + row * lda + kc + 4 * c4);
      if constexpr (MASK) rm[p][q] = ld4(fx.Amask + row * Kr + k0 + 4 * c4);
    }
    if constexpr (BKN) {  // element e: k row e / 32, float4 column e % 32 of the 128 n
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        const int e = t + 256 * q, kk = e >> 5, c4 = e & 31;
        rb[p][q] = ld4(B + (int64_t)(k0 + kk) * No + n0 + 4 * c4);
      }
    } else {
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        const int e = t + 256 * q, r = e / kC4, c4 = e % kC4;
        rb[p][q] = ld4(B + (int64_t)(n0 + r) * Kr + k0 + 4 * c4);
      }
    }
  };
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  uint16_t *pA = reinterpret_cast<uint16_t *>(smem);      // [3][BM][kLdP]
  uint16_t *pB = pA + 3 * BM * kLdP;  // [3][128][kLdP], or [3][kChunk][kLdK] ([k][n] B)
  constexpr int kPB = BKN ? kChunk * kLdK : kTile * kLdP;  // B plane stride
  auto stage_planes = [&](int p) {
    const float4(&xb)[QB] = rb[p];
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int e = t + 256 * q, r = e / kC4, c4 = e % kC4;
      float4 a = ra[p][q];
      if constexpr (MASK) {
        const float4 mk = rm[p][q];
        a.x = mk.x > 0.f ? a.x : 0.f;
        a.y = mk.y > 0.f ? a.y : 0.f;
        a.z = mk.z > 0.f ? a.z : 0.f;
        a.w = mk.w > 0.f ? a.w : 0.f;
      }
      const Split3x4 v = split3x4(a);
      uint16_t *d = pA + r * kLdP + plane_pos(c4);
      *reinterpret_cast<uint2 *>(d) = v.h;
      *reinterpret_cast<uint2 *>(d + BM * kLdP) = v.m;
      *reinterpret_cast<uint2 *>(d + 2 * BM * kLdP) = v.l;
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const Split3x4 v = split3x4(xb[q]);
      uint16_t *d;
      if constexpr (BKN) {  // [k][n] as in memory
        const int e = t + 256 * q, kk = e >> 5, c4 = e & 31;
        d = pB + kk * kLdK + 4 * c4;
      } else {
        const int e = t + 256 * q, r = e / kC4, c4 = e % kC4;
        d = pB + r * kLdP + plane_pos(c4);
      }
      *reinterpret_cast<uint2 *>(d) = v.h;
      *reinterpret_cast<uint2 *>(d + kPB) = v.m;
      *reinterpret_cast<uint2 *>(d + 2 * kPB) = v.l;
    }
  };
  auto compute = [&]() {
#pragma unroll
      for (int s16 = 0; s16 < kChunk / 16; ++s16) {
        Split3 sa[TM], sb[2];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          const uint16_t *ap = pA + (wm * (BM / 2) + tm * 32 + i) * kLdP + s16 * 16 + 8 * h;
          sa[tm].h = *reinterpret_cast<const bf16x8 *>(ap);
          sa[tm].m = *reinterpret_cast<const bf16x8 *>(ap + BM * kLdP);
          sa[tm].l = *reinterpret_cast<const bf16x8 *>(ap + 2 * BM * kLdP);
        }
#pragma unroll
        for (int tn = 0; tn < 2; ++tn) {
          if constexpr (BKN) {
            sb[tn] = tr_split3(pB, kPB, wn * 64 + tn * 32, s16, lane);
          } else {
            const uint16_t *bp = pB + (wn * 64 + tn * 32 + i) * kLdP + s16 * 16 + 8 * h;
            sb[tn].h = *reinterpret_cast<const bf16x8 *>(bp);
            sb[tn].m = *reinterpret_cast<const bf16x8 *>(bp + kTile * kLdP);
            sb[tn].l = *reinterpret_cast<const bf16x8 *>(bp + 2 * kTile * kLdP);
          }
        }
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < 2; ++tn) acc[tm][tn] = mfma_x6(sa[tm], sb[tn], acc[tm][tn]);
      }
  };
  const int nc = Kr / kChunk;
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (p < nc) load(p, p * kChunk);
  for (int c0 = 0; c0 < nc; c0 += PF) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {  // chunk c0 + p lives in staging slot p
      const int c = c0 + p;
      if (c < nc) {
        __syncthreads();  // the previous chunk's LDS reads are done
        stage_planes(p);
        __syncthreads();
        if (c + PF < nc) load(p, (c + PF) * kChunk);  // in flight during the products
        compute();
      }
    }
  }
}

template <int BM, int PF, bool BKN, bool MASK>
__global__ __launch_bounds__(256, 2) MIREC_NO_PK_F32 void gemm_nt_kernel(const float *__restrict__ A,
                                                        const float *__restrict__ B,
                                                        const float *__restrict__ bias,
                                                        float *__restrict__ C, int64_t n,
                                                        int Kr, int No, NtArgs fx) {
  constexpr int TM = BM / 64;
  __shared__ __attribute__((aligned(16))) float smem[nt_lds_floats<BM>()];
  static_assert(4 * 32 * kLdO <= (BM + kTile) * kLdNT, "epilogue staging fits");
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int wm = w >> 1, wn = w & 1;
  // column tile fastest: the column tiles of one row tile run together and
  // share its A rows through L2
  const int ncol = No / kTile;
  const int64_t m0 = (int64_t)(blockIdx.x / ncol) * BM;
  const int n0 = (int)(blockIdx.x % ncol) * kTile;
  f32x16 acc[TM][2];
  nt_mainloop<BM, PF, BKN, MASK>(smem, A, B, n, Kr, No, fx, m0, n0, acc);
  // C layout of 32x32: lane holds column i, rows (r & 3) + 8 (r >> 2) + 4 h.
  // Stored through LDS: each 32x32 block goes to a wave-private [row][col]
  // slab and leaves as float4 rows (4 dwordx4 per lane instead of 16 dword
  // stores: the store tail is issue-bound, not bandwidth-bound)
  __syncthreads();  // every wave's reads of the last chunk are done
  float *sO = smem + w * 32 * kLdO;
#pragma unroll
  for (int tn = 0; tn < 2; ++tn) {
    const int col = n0 + wn * 64 + tn * 32 + i;
    const float bv = bias ? bias[col] : 0.f;
    // output block of these 32 columns (a split at Ns is tile-aligned)
    const int cbase = n0 + wn * 64 + tn * 32;
    float *cb = C;
    int ldc = No, cc = cbase;
    if (fx.C2 != nullptr) {
      if (cbase < fx.Ns) {
        ldc = fx.Ns;
      } else {
        cb = fx.C2;
        ldc = No - fx.Ns;
        cc = cbase - fx.Ns;
      }
    }
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float y = acc[tm][tn][r] + bv;
        if (fx.relu) y = fmaxf(y, 0.f);
        sO[((r & 3) + 8 * (r >> 2) + 4 * h) * kLdO + i] = y;
      }
      wave_sync();  // the slab is wave-private
      const int64_t rbase = m0 + wm * (BM / 2) + tm * 32;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = lane + 64 * q, rr = e >> 3, c4 = e & 7;
        const float4 v = ld4(sO + rr * kLdO + 4 * c4);
        // rows past n hold row n - 1's products (clamped loads): stored
        // there as its own values, no branch
        st4(cb + min(rbase + rr, n - 1) * ldc + cc + 4 * c4, v);
      }
      wave_sync();  // the slab is wave-private
    }
  }
}

// ------------------------------------------ gemm_nt at K = 128, B resident
// C[n, No] = A[n, 128] · B[No, 128]ᵀ (+ bias, ReLU, split output): the
// QKV in-projection of the SASRec block.  A workgroup splits its 128-column
// slice of B once into bf16 planes that stay in LDS (104 KB) while its eight
// waves (two per SIMD) stream 32-row units of A through them: a wave loads
// its unit's rows straight into the MFMA operand layout (two float4 per lane
// and 16-deep block, the next unit's loads in flight during the current
// unit's products) and splits them in registers — once per element, the
// wave owns all 128 columns of the slice.  No barrier after the one that
// publishes B; per unit the LDS carries B operand reads and the epilogue
// slab only.  (gemm_nt_kernel re-stages and re-splits the B slice for every
// 64-row tile and synchronises its waves twice per 32-deep chunk: at K = 128
// its load / split / LDS phases took ~32 of the QKV forward's 49 µs.)  The
// operand values, the k blocks, their order and the six products per block
// are gemm_nt_kernel's: bitwise the same C.
constexpr int kRK = 128;        // the k extent of this form
constexpr int kLdR = kRK + 8;   // bf16 row stride of the B planes (68 dwords: a 16-lane
                                // group's 16-byte reads hit 16 distinct 4-bank groups)
constexpr int kRWaves = 8;      // waves per workgroup sharing one B image
constexpr size_t kResLds = sizeof(uint16_t) * 3 * kTile * kLdR + sizeof(float) * kRWaves * 32 * kLdO;
constexpr int kResMinUnitsPerCU = 16;  // below: the tiled kernel (gemm_nt)

__global__ __launch_bounds__(64 * kRWaves, 1) void gemm_nt_res_kernel(
    const float *__restrict__ A, const float *__restrict__ B, const float *__restrict__ bias,
    float *__restrict__ C, int64_t n, int No, int groups, NtArgs fx) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  uint16_t *pB = reinterpret_cast<uint16_t *>(smem);  // [3][128][kLdR]
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform unit indices
  const int i = lane & 31, h = lane >> 5;
  const int ncol = No / kTile;
  const int n0 = (int)(blockIdx.x % ncol) * kTile;
  const int64_t grp = blockIdx.x / ncol;
  // the B slice (rows n0 .. n0 + 127) -> planes, each float4 at its plane_pos
#pragma unroll
  for (int q = 0; q < kTile * kRK / 4 / (64 * kRWaves); ++q) {
    const int e = t + 64 * kRWaves * q, r = e >> 5, c4 = e & 31;
    const Split3x4 v = split3x4(ld4(B + (int64_t)(n0 + r) * kRK + 4 * c4));
    uint16_t *d = pB + r * kLdR + plane_pos(c4);
    *reinterpret_cast<uint2 *>(d) = v.h;
    *reinterpret_cast<uint2 *>(d + kTile * kLdR) = v.m;
    *reinterpret_cast<uint2 *>(d + 2 * kTile * kLdR) = v.l;
  }
  __syncthreads();
  float *sO = smem + 3 * kTile * kLdR / 2 + w * 32 * kLdO;  // wave-private slab
  const int64_t units = (n + 31) / 32, stride = (int64_t)groups * kRWaves;
  int64_t u = grp * kRWaves + w;
  if (u >= units) return;  // (no barrier follows)
  float bv[4];  // loaded before the first unit: an epilogue load would wait behind the prefetch
#pragma unroll
  for (int tn = 0; tn < 4; ++tn) bv[tn] = bias ? bias[n0 + tn * 32 + i] : 0.f;
  // unit u: rows [32 u, +32); lane (i, h) holds row 32 u + i, k = 16 s + 4 h
  // + (0..3) and 16 s + 8 + 4 h + (0..3) of block s (the x6_k order).  Rows
  // past n load row n - 1 (unconditional loads: counted waits) and are not
  // stored.
  auto rowp = [&](int64_t uu) {
    return A + std::min<int64_t>(32 * uu + i, n - 1) * kRK + 4 * h;
  };
  float4 x[2 * kRK / 16];
  {
    const float *p = rowp(u);
#pragma unroll
    for (int s = 0; s < kRK / 16; ++s) {
      x[2 * s] = ld4(p + 16 * s);
      x[2 * s + 1] = ld4(p + 16 * s + 8);
    }
  }
  for (;;) {
    const int64_t un = u + stride;
    const bool more = un < units;
    // the next unit's rows (the last unit reloads its own: unconditional
    // loads into the same registers keep every wait counted)
    const float *pn = rowp(more ? un : u);
    f32x16 acc[4];
#pragma unroll
    for (int tn = 0; tn < 4; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tn][r] = 0.f;
#pragma unroll
    for (int s = 0; s < kRK / 16; ++s) {
      const float v[8] = {x[2 * s].x,     x[2 * s].y,     x[2 * s].z,     x[2 * s].w,
                          x[2 * s + 1].x, x[2 * s + 1].y, x[2 * s + 1].z, x[2 * s + 1].w};
      const Split3 sa = split3(v);
      x[2 * s] = ld4(pn + 16 * s);  // block s of the next unit into the registers just split
      x[2 * s + 1] = ld4(pn + 16 * s + 8);
      __builtin_amdgcn_sched_barrier(0);  // issued here, a unit ahead of their use
      Split3 sb[4];
#pragma unroll
      for (int tn = 0; tn < 4; ++tn) {
        const uint16_t *bp = pB + (tn * 32 + i) * kLdR + s * 16 + 8 * h;
        sb[tn] = Split3{*reinterpret_cast<const bf16x8 *>(bp),
                        *reinterpret_cast<const bf16x8 *>(bp + kTile * kLdR),
                        *reinterpret_cast<const bf16x8 *>(bp + 2 * kTile * kLdR)};
      }
#pragma unroll
      for (int tn = 0; tn < 4; ++tn) acc[tn] = mfma_x6(sa, sb[tn], acc[tn]);
    }
    // epilogue as gemm_nt_kernel's: bias, ReLU, split output, float4 rows
    // through the wave's slab
    const int64_t rbase = 32 * u;
#pragma unroll
    for (int tn = 0; tn < 4; ++tn) {
      const int cbase = n0 + tn * 32;
      float *cb = C;
      int ldc = No, cc = cbase;
      if (fx.C2 != nullptr) {
        if (cbase < fx.Ns) {
          ldc = fx.Ns;
        } else {
          cb = fx.C2;
          ldc = No - fx.Ns;
          cc = cbase - fx.Ns;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float y = acc[tn][r] + bv[tn];
        if (fx.relu) y = fmaxf(y, 0.f);
        sO[((r & 3) + 8 * (r >> 2) + 4 * h) * kLdO + i] = y;
      }
      wave_sync();
      float4 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = ld4(sO + (lane >> 3) * kLdO + 8 * q * kLdO + 4 * (lane & 7));
      // rows past n computed row n - 1's product from its operands (clamped
      // loads): they store those same values there — no branch, and every
      // wait stays counted
#pragma unroll
      for (int q = 0; q < 4; ++q)
        st4(cb + std::min<int64_t>(rbase + (lane >> 3) + 8 * q, n - 1) * ldc + cc + 4 * (lane & 7),
            v[q]);
      wave_sync();
    }
    if (!more) break;
    u = un;
  }
}

// ------------------------------------------------------- gemm + row tail
// z = A Bᵀ over the whole row (No = d = 128: one column tile) followed in the
// same workgroup by the SASRec block's row tail of mirec_resnorm_fwd
// (model/sasrec.py:385-397): pre = res + dropout(z + bias), out = relu?(pre),
// y = LayerNorm(out).  z never leaves the chip (the unfused pair writes and
// re-reads it: 2 x 28.8 MB and a launch per stage at C4).  The tile goes
// to LDS as [row][132]; then 32 lanes per row, one float4 each, with the
// arithmetic of resnorm_fwd_kernel<32, 1> (same sums in the same order:
// identical out / y / mean / rstd).
struct RnArgs {
  const float *res, *bias, *gamma, *beta;
  float *out, *y, *mean, *rstd;
  int relu;
  uint64_t key;
  uint32_t thresh;
  float scale, eps;
  const uint64_t *key_base;
};

constexpr int kLdRow = kTile + 4;  // [row][col] stride of the tile image

template <int BM>
constexpr int rn_lds_floats() {
  return nt_lds_floats<BM>() > BM * kLdRow ? nt_lds_floats<BM>() : BM * kLdRow;
}

template <int BM>
__global__ __launch_bounds__(256, 2) void gemm_resnorm_kernel(const float *__restrict__ A,
                                                              const float *__restrict__ B,
                                                              int64_t n, int Kr, RnArgs a) {
  constexpr int TM = BM / 64;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int wm = w >> 1, wn = w & 1;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const NtArgs fx{nullptr, nullptr, nullptr, 0, 0, 0, 0};
  // the residual rows of this thread's lane group (32 lanes per row, one
  // float4 each) are loaded before the k loop: in flight behind the products
  const int g = t >> 5, c = 4 * (t & 31);
  constexpr int RPG = BM / 8;
  float4 rv[RPG];
#pragma unroll
  for (int q = 0; q < RPG; ++q) {
    const int64_t r = m0 + g + 8 * q;
    rv[q] = a.res ? ld4(a.res + min(r, n - 1) * kTile + c) : f4_zero();  // (as gemm_nn_rnbwd)
  }
  f32x16 acc[TM][2];
  nt_mainloop<BM, 1, false>(smem, A, B, n, Kr, kTile, fx, m0, 0, acc);
  __syncthreads();  // every wave's reads of the last chunk are done
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < 2; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        smem[(wm * (BM / 2) + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * kLdRow + wn * 64 +
             tn * 32 + i] = acc[tm][tn][r];
  __syncthreads();
  const uint64_t key = a.thresh != 0u ? run_key(a.key, a.key_base) : 0ull;
  const float inv_d = 1.f / (float)kTile;
  const float4 bia = a.bias ? ld4(a.bias + c) : f4_zero();
  const float4 gam = a.gamma ? ld4(a.gamma + c) : make_float4(1.f, 1.f, 1.f, 1.f);
  const float4 bet = a.beta ? ld4(a.beta + c) : f4_zero();
#pragma unroll
  for (int q = 0; q < RPG; ++q) {
    const int rr = g + 8 * q;
    const int64_t r = m0 + rr;
    if (r >= n) break;  // whole 32-lane groups (a row each) leave together
    const int64_t e = r * kTile + c;
    float4 x = f4_add(ld4(smem + rr * kLdRow + c), bia);
    if (a.thresh != 0u) x = drop4(x, key, (uint64_t)e, a.thresh, a.scale);
    if (a.res) x = f4_add(x, rv[q]);
    if (a.relu)
      x = make_float4(fmaxf(x.x, 0.f), fmaxf(x.y, 0.f), fmaxf(x.z, 0.f), fmaxf(x.w, 0.f));
    if (a.out) st4(a.out + e, x);
    if (a.y == nullptr) continue;
    const float mu = group_sum<32>((x.x + x.y) + (x.z + x.w)) * inv_d;
    const float4 tq = make_float4(x.x - mu, x.y - mu, x.z - mu, x.w - mu);
    const float rs = rsqrtf(group_sum<32>(f4_dot(tq, tq)) * inv_d + a.eps);
    const float4 tt = make_float4(rs * tq.x, rs * tq.y, rs * tq.z, rs * tq.w);
    st4(a.y + e, make_float4(tt.x * gam.x + bet.x, tt.y * gam.y + bet.y, tt.z * gam.z + bet.z,
                             tt.w * gam.w + bet.w));
    if ((t & 31) == 0) {
      a.mean[r] = mu;
      a.rstd[r] = rs;
    }
  }
}

// ----------------------------------------------- gemm + row tail backward
// g_y = A W (W [Kr][d] as stored, d = 128: the input gradient of the next
// Linear, which is the gradient of this row tail's LayerNorm output) and, in
// the same workgroup, mirec_resnorm_bwd of that row tail: the tile goes to
// LDS as [row][132], then 32 lanes per row with resnorm_bwd_kernel<32, 1>'s
// per-row expressions (d_res / d_z within an ulp: the compiler contracts
// them differently here); the column sums (d_gamma,
// d_beta, d_bias) leave as one [3][128] partial per workgroup, added in
// workgroup order by the resnorm reduce.  g_y never reaches HBM.  The out /
// g_out rows and the row statistics are loaded before the k loop.
struct RbArgs {
  const float *g_out, *out, *mean, *rstd, *gamma;
  float *d_res, *d_z, *partial;
  int relu;
  uint64_t key;
  uint32_t thresh;
  float scale;
  const uint64_t *key_base;
};

template <int BM>
constexpr int rb_lds_floats() {
  return std::max(std::max(nt_lds_floats<BM>(), BM * kLdRow), 8 * 3 * kTile);
}

template <int BM>
__global__ __launch_bounds__(256, 2) void gemm_nn_rnbwd_kernel(const float *__restrict__ A,
                                                               const float *__restrict__ W,
                                                               int64_t n, int Kr, RbArgs a) {
  constexpr int TM = BM / 64;
  constexpr int RPG = BM / 8;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int wm = w >> 1, wn = w & 1;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int g = t >> 5, c = 4 * (t & 31);
  float4 ov[RPG], gv[RPG];
  float mv[RPG], sv[RPG];
  // unconditional loads of a clamped row index (rows past n are never
  // stored): with exec-masked loads (r < n ? load : 0) here, the bf16x6 k
  // loop below returned, in up to 1 of 2 launches at n = 56 K, one row whose
  // row-tail statistics were wrong while its g_y was right (always a
  // second-pass row of an upper half-wave, local rows 9 / 11 / 13 / 15);
  // never with the f32 loop, never with these loads (0 in 120 launches over
  // two builds) — test_gemm_nn_resnorm_bwd_repeatable; the cause is the
  // packed-f32 op_sel hazard of DESIGN.md §9.1 (tools/op_sel_repro.hip).
#pragma unroll
  for (int q = 0; q < RPG; ++q) {
    const int64_t r = min(m0 + g + 8 * q, n - 1);
    ov[q] = ld4(a.out + r * kTile + c);
    gv[q] = a.g_out ? ld4(a.g_out + r * kTile + c) : f4_zero();
    mv[q] = a.mean[r];
    sv[q] = a.rstd[r];
  }
  const NtArgs fx{nullptr, nullptr, nullptr, 0, 0, 0, 1};
  f32x16 acc[TM][2];
  nt_mainloop<BM, 1, true>(smem, A, W, n, Kr, kTile, fx, m0, 0, acc);
  __syncthreads();  // every wave's reads of the last chunk are done
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < 2; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        smem[(wm * (BM / 2) + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * kLdRow + wn * 64 +
             tn * 32 + i] = acc[tm][tn][r];
  __syncthreads();
  const uint64_t key = a.thresh != 0u ? run_key(a.key, a.key_base) : 0ull;
  const float inv_d = 1.f / (float)kTile;
  const float4 gam = a.gamma ? ld4(a.gamma + c) : make_float4(1.f, 1.f, 1.f, 1.f);
  float4 pg = f4_zero(), pb = f4_zero(), pz = f4_zero();
#pragma unroll
  for (int q = 0; q < RPG; ++q) {
    const int rr = g + 8 * q;
    const int64_t r = m0 + rr;
    if (r >= n) break;  // whole 32-lane groups (a row each) leave together
    const int64_t e = r * kTile + c;
    const float4 gy = ld4(smem + rr * kLdRow + c), v = ov[q];
    const float mu = mv[q], rs = sv[q];
    const float4 mu4 = make_float4(mu, mu, mu, mu);
    const float4 xh = f4_scale(rs, f4_sub(v, mu4));
    const float4 gx = make_float4(gy.x * gam.x, gy.y * gam.y, gy.z * gam.z, gy.w * gam.w);
    const float m1 = group_sum<32>((gx.x + gx.y) + (gx.z + gx.w)) * inv_d;
    const float m2 = group_sum<32>(f4_dot(gx, xh)) * inv_d;
    // dx = rstd * (gx - mean(gx) - xhat * mean(gx * xhat)) (+ g_out)
    const float4 tq = f4_sub(f4_sub(gx, make_float4(m1, m1, m1, m1)), f4_scale(m2, xh));
    const float4 gr = f4_fma(rs, tq, gv[q]);
    pg = f4_add(pg, make_float4(gy.x * xh.x, gy.y * xh.y, gy.z * xh.z, gy.w * xh.w));
    pb = f4_add(pb, gy);
    float4 x = a.relu ? make_float4(v.x > 0.f ? gr.x : 0.f, v.y > 0.f ? gr.y : 0.f,
                                    v.z > 0.f ? gr.z : 0.f, v.w > 0.f ? gr.w : 0.f)
                      : gr;
    if (a.d_res) st4(a.d_res + e, x);
    if (a.thresh != 0u) x = drop4(x, key, (uint64_t)e, a.thresh, a.scale);
    if (a.d_z) st4(a.d_z + e, x);
    pz = f4_add(pz, x);
  }
  if (a.partial == nullptr) return;  // workgroup-uniform
  __syncthreads();                   // the tile image is no longer read
  float *red = smem;                 // [8 groups][3][128]
  st4(red + (g * 3 + 0) * kTile + c, pg);
  st4(red + (g * 3 + 1) * kTile + c, pb);
  st4(red + (g * 3 + 2) * kTile + c, pz);
  __syncthreads();
  for (int k = t; k < 3 * kTile; k += 256) {
    const int kk = k / kTile, col = k - kk * kTile;
    float sacc = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) sacc += red[(q * 3 + kk) * kTile + col];
    a.partial[(int64_t)blockIdx.x * 3 * kTile + k] = sacc;
  }
}

// ------------------------------------------------------------------ gemm_tn
// Workgroup (slice s, tile_m, tile_n): partial C tile over rows
// [s * rows_per_slice, +rows_per_slice) -> work[s][M][No]; with colsum, the
// tile_n == 0 workgroups also write the slice's column sums of A ->
// work_cs[s][M].  LDS: bf16 planes [3][kChunk][kLdK] of A and of B
// (k-major, as in memory).
// Fused forms: Amask zeroes A elements whose mask (same layout) is <= 0 (the
// ReLU backward); B may be two blocks side by side, columns [0, Ns) from B
// (row stride Ns) and [Ns, No) from B2 (row stride No - Ns), Ns % 128 == 0.
struct TnArgs {
  const float *Amask;
  const float *B2;
  int Ns;
};

template <bool MASK, int PF>
__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(const float *__restrict__ A,
                                                        const float *__restrict__ B,
                                                        float *__restrict__ work,
                                                        float *__restrict__ work_cs,
                                                        int64_t n, int M, int No,
                                                        int64_t rows_per_slice, TnArgs fx) {
  // both k-major operands as [k][col] bf16 planes read back with the
  // transposing LDS read (as gemm_nt's [k][n] B); the column sums of A are
  // taken from the staged f32 values
  constexpr int kPl = kChunk * kLdK;  // one plane (bf16 units)
  constexpr int kTnLds = 3 * kPl;
  __shared__ __attribute__((aligned(16))) float smem[kTnLds];
  static_assert(4 * 32 * kLdO <= kTnLds && 8 * kTile <= kTnLds, "epilogue staging fits");
  uint16_t *pA = reinterpret_cast<uint16_t *>(smem), *pB = pA + 3 * kPl;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int wm = w >> 1, wn = w & 1;
  const int s = blockIdx.x;
  const int m0 = blockIdx.y * kTile, n0 = blockIdx.z * kTile;
  const int64_t r_beg = (int64_t)s * rows_per_slice;
  const int64_t r_end = min(n, r_beg + rows_per_slice);
  const bool do_cs = work_cs != nullptr && blockIdx.z == 0;
  // B columns [n0, +128): from B, or from B2 past the split (workgroup-uniform)
  const float *Bc = B + n0;
  int64_t ldb = No;
  if (fx.B2 != nullptr) {
    if (n0 < fx.Ns) {
      ldb = fx.Ns;
    } else {
      Bc = fx.B2 + (n0 - fx.Ns);
      ldb = No - fx.Ns;
    }
  }
  // element e = t + 256 q: chunk row e >> 5, float4 column e & 31.  Rows
  // past the slice load its last row (unconditional loads: counted waits)
  // and are zeroed when staged; PF chunks of loads are in flight.
  constexpr int QT = kChunk * 32 / 256;
  float4 ra[PF][QT], rb[PF][QT], rm[MASK ? PF : 1][QT];
  auto load = [&](int p, int64_t r0) {
    const int lim = (int)min<int64_t>(r_end - r0, kChunk);  // rows of this chunk in the slice
#pragma unroll
    for (int q = 0; q < QT; ++q) {
      const int e = t + 256 * q, kk = e >> 5, c4 = e & 31;
      const int64_t r = r0 + min(kk, lim - 1);
      ra[p][q] = ld4(A + r * M + m0 + 4 * c4);
      rb[p][q] = ld4(Bc + r * ldb + 4 * c4);
      if constexpr (MASK) rm[p][q] = ld4(fx.Amask + r * M + m0 + 4 * c4);
    }
  };
  float4 csv = f4_zero();  // this thread's column sums (columns 4 c4 ..)
  auto stage = [&](int p, int64_t r0) {
    const int lim = (int)min<int64_t>(r_end - r0, kChunk);
#pragma unroll
    for (int q = 0; q < QT; ++q) {
      const int e = t + 256 * q, kk = e >> 5, c4 = e & 31;
      const bool ok = lim == kChunk || kk < lim;  // (the slice's last chunk may be short)
      float4 a = ra[p][q], b = rb[p][q];
      if constexpr (MASK) {
        const float4 mk = rm[p][q];
        a.x = mk.x > 0.f ? a.x : 0.f;
        a.y = mk.y > 0.f ? a.y : 0.f;
        a.z = mk.z > 0.f ? a.z : 0.f;
        a.w = mk.w > 0.f ? a.w : 0.f;
      }
      if (!ok) {
        a = f4_zero();
        b = f4_zero();
      }
      if (do_cs) csv = f4_add(csv, a);
      const Split3x4 va = split3x4(a), vb = split3x4(b);
      uint16_t *da = pA + kk * kLdK + 4 * c4, *db = pB + kk * kLdK + 4 * c4;
      *reinterpret_cast<uint2 *>(da) = va.h;
      *reinterpret_cast<uint2 *>(da + kPl) = va.m;
      *reinterpret_cast<uint2 *>(da + 2 * kPl) = va.l;
      *reinterpret_cast<uint2 *>(db) = vb.h;
      *reinterpret_cast<uint2 *>(db + kPl) = vb.m;
      *reinterpret_cast<uint2 *>(db + 2 * kPl) = vb.l;
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int64_t nc = (r_end - r_beg + kChunk - 1) / kChunk;
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (p < nc) load(p, r_beg + p * kChunk);
  for (int64_t c0 = 0; c0 < nc; c0 += PF) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {  // chunk c0 + p lives in staging slot p
      const int64_t c = c0 + p;
      if (c < nc) {
        __syncthreads();  // the previous chunk's LDS reads are done
        stage(p, r_beg + c * kChunk);
        __syncthreads();
        if (c + PF < nc) load(p, r_beg + (c + PF) * kChunk);  // in flight during the products
#pragma unroll
        for (int s16 = 0; s16 < kChunk / 16; ++s16) {
          Split3 sa[2], sb[2];
#pragma unroll
          for (int tm = 0; tm < 2; ++tm) sa[tm] = tr_split3(pA, kPl, wm * 64 + tm * 32, s16, lane);
#pragma unroll
          for (int tn = 0; tn < 2; ++tn) sb[tn] = tr_split3(pB, kPl, wn * 64 + tn * 32, s16, lane);
#pragma unroll
          for (int tm = 0; tm < 2; ++tm)
#pragma unroll
            for (int tn = 0; tn < 2; ++tn) acc[tm][tn] = mfma_x6(sa[tm], sb[tn], acc[tm][tn]);
        }
      }
    }
  }
  // partial tile out through a wave-private LDS slab as float4 rows (as in
  // gemm_nt_kernel)
  float *out = work + (int64_t)s * M * No;
  __syncthreads();
  float *sO = smem + w * 32 * kLdO;
#pragma unroll
  for (int tn = 0; tn < 2; ++tn)
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sO[((r & 3) + 8 * (r >> 2) + 4 * h) * kLdO + i] = acc[tm][tn][r];
      wave_sync();  // the slab is wave-private
      const int rbase = m0 + wm * 64 + tm * 32, cbase = n0 + wn * 64 + tn * 32;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = lane + 64 * q, rr = e >> 3, c4 = e & 7;
        st4(out + (int64_t)(rbase + rr) * No + cbase + 4 * c4, ld4(sO + rr * kLdO + 4 * c4));
      }
      wave_sync();  // the slab is wave-private
    }
  if (!do_cs) return;  // workgroup-uniform
  __syncthreads();     // the slabs are no longer read
  st4(smem + (t >> 5) * kTile + 4 * (t & 31), csv);
  __syncthreads();
  if (t < kTile) {  // the 8 row groups added in group order
    float c = 0.f;
#pragma unroll
    for (int g8 = 0; g8 < 8; ++g8) c += smem[g8 * kTile + t];
    work_cs[(int64_t)s * M + m0 + t] = c;
  }
}

// C[e] = Σ_s work[s][e] (float4 e), colsum[m] = Σ_s work_cs[s][m].  A
// 1024-thread block owns 64 float4 elements: wave g sums the slices s ≡ g
// (mod 16) of its lane's element, then the 16 partials are added in wave
// order through LDS (a fixed order: deterministic).  Block 0..M/64 also
// reduce colsum the same way.
constexpr int kRedGroups = 16;
constexpr int kRedU = 16;
__global__ __launch_bounds__(1024) void gemm_tn_reduce_kernel(const float *__restrict__ work,
                                                              const float *__restrict__ work_cs,
                                                              float *__restrict__ C,
                                                              float *__restrict__ colsum,
                                                              int slices, int64_t n4, int M) {
  __shared__ float4 part[kRedGroups][64];
  __shared__ float pcs[kRedGroups][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  float4 a = f4_zero();
  float c = 0.f;
  if (e < n4) {
    // kRedU slices' loads in flight per round (the sum order is unchanged:
    // s = g, g + 16, ... ascending)
    for (int s0 = g; s0 < slices; s0 += kRedGroups * kRedU) {
      float4 x[kRedU];
#pragma unroll
      for (int u = 0; u < kRedU; ++u) {
        const int s = s0 + kRedGroups * u;
        x[u] = s < slices ? ld4(work + ((int64_t)s * n4 + e) * 4) : f4_zero();
      }
#pragma unroll
      for (int u = 0; u < kRedU; ++u)
        if (s0 + kRedGroups * u < slices) a = f4_add(a, x[u]);
    }
  }
  const bool do_cs = colsum != nullptr && e < M;
  if (do_cs) {
    for (int s0 = g; s0 < slices; s0 += kRedGroups * kRedU) {
      float x[kRedU];
#pragma unroll
      for (int u = 0; u < kRedU; ++u) {
        const int s = s0 + kRedGroups * u;
        x[u] = s < slices ? work_cs[(int64_t)s * M + e] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kRedU; ++u)
        if (s0 + kRedGroups * u < slices) c += x[u];
    }
  }
  part[g][lane] = a;
  pcs[g][lane] = c;
  __syncthreads();
  if (g == 0) {
    for (int q = 1; q < kRedGroups; ++q) {
      a = f4_add(a, part[q][lane]);
      c += pcs[q][lane];
    }
    if (e < n4) st4(C + e * 4, a);
    if (do_cs) colsum[e] = c;
  }
}

// Row slices of gemm_tn: enough workgroups to fill the chip twice over,
// at least 64 rows (2 chunks) per slice.  (256 is 3 us faster on the
// 56 K x 128 x 128 weight gradient run alone, but the C4 step, whose inputs
// arrive from the kernels before it, runs faster with more, shorter slices:
// 256 -> 128 rows 1.45 -> 1.43 ms (two same-box A/B pairs), 128 -> 64 rows
// another 1.2 % (three pairs); C3 unchanged (its large weight gradients
// are not bound by the minimum).  tools/ab_tn.sh, tools/ab_libs.sh.)
constexpr int64_t kTnMinRows = 64;
// A single 128 x 128 output tile (the d = 128 projection / FFN weight
// gradients of C4) takes 256 slices instead: half the partial tiles for the
// reduce, and its load-latency-bound slices lose less than the reduce saves
// (split bf16 loop: 30.4 -> 25.7 us, C4 1.259 -> 1.232 ms/step, same box;
// 256 workgroups in total lose on 2- and 3-tile gradients: 125 -> 172 us,
// 49.6 -> 52.9 us).
constexpr int64_t kTnWant = 512, kTnWant1 = 256;  // workgroups (several tiles / one tile)
// chunks of gemm_tn loads in flight: two measured 1-3 % slower on the C3 / C4
// weight gradients (profiles/round5_gemm_tn.txt)
constexpr int kTnPF = 1;
static void tn_slices(int64_t n, int M, int No, int *slices, int64_t *rows) {
  const int64_t tiles = (int64_t)(M / kTile) * (No / kTile);
  const int64_t total = tiles == 1 ? kTnWant1 : kTnWant;
  const int64_t want = std::max<int64_t>(1, (total + tiles - 1) / tiles);
  int64_t r = std::max<int64_t>(kTnMinRows, (n + want - 1) / want);
  r = (r + kChunk - 1) / kChunk * kChunk;
  *rows = r;
  *slices = (int)std::max<int64_t>(1, (n + r - 1) / r);
}

// Column sums out[c] = Σ_r A[r, c] of a row-major [n, m] matrix in a fixed
// order (the bias gradient db = Σ_rows dY of Linear layers whose widths the
// GEMM tiles do not take).  Slices of a fixed 64 rows while n <= 64 x 2048 /
// ceil(m / 256): zero rows appended to A (the captured SASRec step's token
// capacity padding) leave every partial and the result bitwise unchanged,
// which torch's sum(0) — its reduction tree follows the row count — does not
// (DESIGN.md §9.2).  Pass 1: workgroup
// (slice s, column block) — one lane per column walks the slice's rows in
// order with four row-interleaved partial sums added as ((p0 + p1) + (p2 +
// p3)); pass 2: one lane per column adds the slices' partials in slice order.
constexpr int kCsRows = 64;  // rows per slice (at least)
__global__ __launch_bounds__(256) void col_sums_slice_kernel(const float *__restrict__ A,
                                                             float *__restrict__ work, int64_t n,
                                                             int m, int64_t rows) {
  const int64_t c = (int64_t)blockIdx.y * 256 + threadIdx.x;
  if (c >= m) return;
  const int64_t r0 = (int64_t)blockIdx.x * rows, r1 = min(n, r0 + rows);
  float p[4] = {0.f, 0.f, 0.f, 0.f};
  int64_t r = r0;
  for (; r + 4 <= r1; r += 4) {
    const float a0 = A[r * m + c], a1 = A[(r + 1) * m + c];
    const float a2 = A[(r + 2) * m + c], a3 = A[(r + 3) * m + c];
    p[0] += a0;
    p[1] += a1;
    p[2] += a2;
    p[3] += a3;
  }
  for (int k = 0; r < r1; ++r, ++k) p[k] += A[r * m + c];
  work[(int64_t)blockIdx.x * m + c] = (p[0] + p[1]) + (p[2] + p[3]);
}

__global__ __launch_bounds__(256) void col_sums_final_kernel(const float *__restrict__ work,
                                                             float *__restrict__ out, int slices,
                                                             int m) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= m) return;
  float s = 0.f;
  for (int q = 0; q < slices; ++q) s += work[(int64_t)q * m + c];
  out[c] = s;
}

static void cs_slices(int64_t n, int m, int *slices, int64_t *rows) {
  // about 2048 workgroups over the chip, at least kCsRows rows each
  const int64_t cb = (m + 255) / 256;
  const int64_t want = std::max<int64_t>(1, 2048 / cb);
  int64_t r = std::max<int64_t>(kCsRows, (n + want - 1) / want);
  *rows = r;
  *slices = (int)std::max<int64_t>(1, (n + r - 1) / r);
}

}  // namespace mirec

using namespace mirec;

extern "C" int64_t mirec_col_sums_work_floats(int64_t n, int32_t m) {
  if (n < 0 || m <= 0) return -1;
  int slices;
  int64_t rows;
  cs_slices(std::max<int64_t>(n, 1), m, &slices, &rows);
  return (int64_t)slices * m;
}

extern "C" int mirec_col_sums(const float *A, int64_t n, int32_t m, float *out, float *work,
                              mirec_stream_t stream) {
  MIREC_CHECK_ARG(n >= 0 && m > 0 && out && work && (n == 0 || A));
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    MIREC_HIP(hipMemsetAsync(out, 0, sizeof(float) * m, st));
    return MIREC_OK;
  }
  int slices;
  int64_t rows;
  cs_slices(n, m, &slices, &rows);
  const unsigned cb = (unsigned)((m + 255) / 256);
  hipLaunchKernelGGL(col_sums_slice_kernel, dim3((unsigned)slices, cb), dim3(256), 0, st, A,
                     work, n, (int)m, rows);
  MIREC_LAUNCH_CHECK();
  hipLaunchKernelGGL(col_sums_final_kernel, dim3(cb), dim3(256), 0, st, work, out, slices, (int)m);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

static int gemm_nt(const float *A, const float *A2, int32_t Ks, const float *Amask,
                   const float *B, const float *bias, float *C, float *C2, int32_t Ns,
                   int32_t relu, int64_t n, int32_t Kr, int32_t No, mirec_stream_t stream,
                   int bkn = 0) {
  MIREC_CHECK_ARG(n >= 0 && Kr > 0 && No > 0 && Kr % kChunk == 0 && No % kTile == 0);
  if (n == 0) return MIREC_OK;  // (empty tensors may carry null pointers)
  MIREC_CHECK_ARG(A && B && C && ((uintptr_t)A | (uintptr_t)B) % 16 == 0);
  MIREC_CHECK_ARG(A2 == nullptr || (Ks > 0 && Ks < Kr && Ks % kChunk == 0 &&
                                    (uintptr_t)A2 % 16 == 0));
  MIREC_CHECK_ARG(Amask == nullptr || (A2 == nullptr && (uintptr_t)Amask % 16 == 0));
  MIREC_CHECK_ARG(C2 == nullptr || (Ns > 0 && Ns < No && Ns % kTile == 0 &&
                                    (uintptr_t)C2 % 16 == 0));
  MIREC_CHECK_ARG((uintptr_t)C % 16 == 0);  // float4 row stores
  NtArgs fx{A2, Amask, C2, Ks, Ns, relu ? 1 : 0, bkn};
  const unsigned ncol = (unsigned)(No / kTile);
  hipStream_t st = (hipStream_t)stream;
  // 128- or 64-row tiles: the one whose grid needs fewer tile-rounds of the
  // chip's workgroup slots (2 per CU), ties to 64 rows when the grid spans
  // more than one round (tools/gemm_bench.py: 64 rows win at 48, 1200,
  // 1320 and 2400 tiles of 128 — C3 hop 126 -> 112 us, C4 QKV forward 73 ->
  // 64 us — and lose at 440: the N = 128 projections at 56 K rows)
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t slots = 2 * (int64_t)std::max(cus, 1);
  const int64_t t128 = (n + 127) / 128 * ncol, t64 = (n + 63) / 64 * ncol;
  const int64_t r128 = 2 * ((t128 + slots - 1) / slots), r64 = (t64 + slots - 1) / slots;
  // the resident-B form when every wave of a full grid gets two units or
  // more: below that the per-workgroup B split is not amortised (a 4 K-row
  // call: 14 vs 8 µs)
  const int64_t res_units = (n + 31) / 32 * (int64_t)ncol;
  if (Kr == kRK && !bkn && A2 == nullptr && Amask == nullptr &&
      res_units >= (int64_t)kResMinUnitsPerCU * std::max(cus, 1)) {
    static int rc = -1;  // dynamic LDS above 64 KiB needs the opt-in (once)
    if (rc < 0)
      rc = hipFuncSetAttribute((const void *)gemm_nt_res_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kResLds) ==
                   hipSuccess
               ? 0
               : 1;
    if (rc != 0) return MIREC_ERR_HIP;
    // one workgroup per CU and column slice, each wave a unit or more
    const int64_t units = (n + 31) / 32;
    const int groups = (int)std::min<int64_t>(std::max<int>(cus / (int)ncol, 1),
                                              (units + kRWaves - 1) / kRWaves);
    hipLaunchKernelGGL(gemm_nt_res_kernel, dim3((unsigned)(groups * ncol)), dim3(64 * kRWaves),
                       kResLds, st, A, B, bias, C, n, (int)No, groups, fx);
    MIREC_LAUNCH_CHECK();
    return MIREC_OK;
  }
  const bool bm64 = r64 < r128 || (r64 == r128 && t128 > slots);
#define MIREC_NT_LAUNCH(BM, BKN, MASK)                                             \
  hipLaunchKernelGGL((gemm_nt_kernel<BM, 1, BKN, MASK>),                           \
                     dim3((unsigned)((n + BM - 1) / BM) * ncol), dim3(256), 0, st, A, B, bias, C, \
                     n, (int)Kr, (int)No, fx)
#define MIREC_NT_LAUNCH_M(BM, BKN)                        \
  do {                                                    \
    if (Amask != nullptr) MIREC_NT_LAUNCH(BM, BKN, true); \
    else MIREC_NT_LAUNCH(BM, BKN, false);                 \
  } while (0)
  if (bm64) {
    if (bkn) MIREC_NT_LAUNCH_M(64, true);
    else MIREC_NT_LAUNCH_M(64, false);
  } else {
    if (bkn) MIREC_NT_LAUNCH_M(128, true);
    else MIREC_NT_LAUNCH_M(128, false);
  }
#undef MIREC_NT_LAUNCH_M
#undef MIREC_NT_LAUNCH
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_gemm_nt(const float *A, const float *B, const float *bias, float *C,
                             int64_t n, int32_t Kr, int32_t No, mirec_stream_t stream) {
  return gemm_nt(A, nullptr, 0, nullptr, B, bias, C, nullptr, 0, 0, n, Kr, No, stream);
}

extern "C" int mirec_gemm_nt_ex(const float *A, const float *A2, int32_t Ks, const float *Amask,
                                const float *B, const float *bias, float *C, float *C2,
                                int32_t Ns, int32_t relu, int64_t n, int32_t Kr, int32_t No,
                                mirec_stream_t stream) {
  return gemm_nt(A, A2, Ks, Amask, B, bias, C, C2, Ns, relu, n, Kr, No, stream);
}

extern "C" int mirec_gemm_nn_ex(const float *A, const float *Amask, const float *B, float *C,
                                float *C2, int32_t Ns, int64_t n, int32_t Kr, int32_t No,
                                mirec_stream_t stream) {
  return gemm_nt(A, nullptr, 0, Amask, B, nullptr, C, C2, Ns, 0, n, Kr, No, stream, 1);
}

extern "C" int64_t mirec_gemm_tn_work_floats(int64_t n, int32_t M, int32_t No) {
  if (n < 0 || M <= 0 || No <= 0 || M % kTile || No % kTile) return -1;
  int slices;
  int64_t rows;
  tn_slices(std::max<int64_t>(n, 1), M, No, &slices, &rows);
  return (int64_t)slices * M * No + (int64_t)slices * M;
}

static int gemm_tn(const float *A, const float *Amask, const float *B, const float *B2,
                   int32_t Ns, float *C, float *colsum, int64_t n, int32_t M, int32_t No,
                   float *work, mirec_stream_t stream) {
  MIREC_CHECK_ARG(C && work && n >= 0 && M > 0 && No > 0 && M % kTile == 0 && No % kTile == 0);
  MIREC_CHECK_ARG(n == 0 || (A && B));  // (empty tensors may carry null pointers)
  MIREC_CHECK_ARG(((uintptr_t)A | (uintptr_t)B | (uintptr_t)C | (uintptr_t)work) % 16 == 0);
  MIREC_CHECK_ARG(Amask == nullptr || (uintptr_t)Amask % 16 == 0);
  MIREC_CHECK_ARG(B2 == nullptr || (Ns > 0 && Ns < No && Ns % kTile == 0 &&
                                    (uintptr_t)B2 % 16 == 0));
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    MIREC_HIP(hipMemsetAsync(C, 0, sizeof(float) * M * No, st));
    if (colsum) MIREC_HIP(hipMemsetAsync(colsum, 0, sizeof(float) * M, st));
    return MIREC_OK;
  }
  int slices;
  int64_t rows;
  tn_slices(n, M, No, &slices, &rows);
  float *work_cs = work + (int64_t)slices * M * No;
  const dim3 grid((unsigned)slices, (unsigned)(M / kTile), (unsigned)(No / kTile));
  TnArgs fx{Amask, B2, Ns};
  if (Amask != nullptr)
    hipLaunchKernelGGL((gemm_tn_kernel<true, kTnPF>), grid, dim3(256), 0, st, A, B, work,
                       colsum ? work_cs : nullptr, n, (int)M, (int)No, rows, fx);
  else
    hipLaunchKernelGGL((gemm_tn_kernel<false, kTnPF>), grid, dim3(256), 0, st, A, B, work,
                       colsum ? work_cs : nullptr, n, (int)M, (int)No, rows, fx);
  MIREC_LAUNCH_CHECK();
  const int64_t n4 = (int64_t)M * No / 4;
  const int64_t blocks = (std::max<int64_t>(n4, M) + 63) / 64;
  hipLaunchKernelGGL(gemm_tn_reduce_kernel, dim3((unsigned)blocks), dim3(1024), 0, st, work,
                     work_cs, C, colsum, slices, n4, (int)M);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_gemm_tn(const float *A, const float *B, float *C, float *colsum, int64_t n,
                             int32_t M, int32_t No, float *work, mirec_stream_t stream) {
  return gemm_tn(A, nullptr, B, nullptr, 0, C, colsum, n, M, No, work, stream);
}

extern "C" int mirec_gemm_tn_ex(const float *A, const float *Amask, const float *B,
                                const float *B2, int32_t Ns, float *C, float *colsum, int64_t n,
                                int32_t M, int32_t No, float *work, mirec_stream_t stream) {
  return gemm_tn(A, Amask, B, B2, Ns, C, colsum, n, M, No, work, stream);
}

template <int BM>
static int launch_gemm_resnorm(const float *A, const float *B, int64_t n, int32_t Kr,
                               const RnArgs &a, hipStream_t st) {
  constexpr size_t lds = sizeof(float) * rn_lds_floats<BM>();
  static int rc = -1;  // dynamic LDS above 64 KiB needs the opt-in (once)
  if (rc < 0)
    rc = hipFuncSetAttribute((const void *)gemm_resnorm_kernel<BM>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess
             ? 0
             : 1;
  if (rc != 0) return MIREC_ERR_HIP;
  hipLaunchKernelGGL(gemm_resnorm_kernel<BM>, dim3((unsigned)((n + BM - 1) / BM)), dim3(256), lds,
                     st, A, B, n, (int)Kr, a);
  MIREC_LAUNCH_CHECK();
  return MIREC_OK;
}

extern "C" int mirec_gemm_resnorm(const float *A, const float *W, int64_t n, int32_t Kr, int32_t d,
                                  const float *res, const float *bias, const float *gamma,
                                  const float *beta, int32_t relu, float dropout_p, uint64_t seed,
                                  const uint64_t *seed_base, float eps, float *out, float *y,
                                  float *mean, float *rstd, mirec_stream_t stream) {
  MIREC_CHECK_ARG(n >= 0 && d == kTile && Kr > 0 && Kr % kChunk == 0);
  RnArgs a{res, bias, gamma, beta, out, y, mean, rstd, relu ? 1 : 0, 0, 0u, 1.f, eps, seed_base};
  MIREC_CHECK_ARG(dropout_params(dropout_p, seed, &a.key, &a.thresh, &a.scale));
  if (n == 0) return MIREC_OK;  // (empty tensors may carry null pointers)
  MIREC_CHECK_ARG(A && W && out && ((uintptr_t)A | (uintptr_t)W | (uintptr_t)out) % 16 == 0);
  MIREC_CHECK_ARG(y == nullptr || (mean && rstd && (uintptr_t)y % 16 == 0));
  MIREC_CHECK_ARG(((uintptr_t)res | (uintptr_t)bias | (uintptr_t)gamma | (uintptr_t)beta) % 16 ==
                  0);
  hipStream_t st = (hipStream_t)stream;
  // the row-tile choice of gemm_nt (one column tile: 128 rows unless that
  // takes more rounds of the chip's workgroup slots)
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t slots = 2 * (int64_t)std::max(cus, 1);
  const int64_t t128 = (n + 127) / 128, t64 = (n + 63) / 64;
  const int64_t r128 = 2 * ((t128 + slots - 1) / slots), r64 = (t64 + slots - 1) / slots;
  if (r64 < r128 || (r64 == r128 && t128 > slots)) return launch_gemm_resnorm<64>(A, W, n, Kr, a, st);
  return launch_gemm_resnorm<128>(A, W, n, Kr, a, st);
}

// row tile of the fused backward: 64 rows (its preloaded out / g_out rows
// keep 128-row tiles above the register budget)
constexpr int kRbBM = 64;

extern "C" int64_t mirec_gemm_nn_resnorm_bwd_work_floats(int64_t n, int32_t d) {
  if (n < 0 || d != kTile) return -1;
  return std::max<int64_t>(1, (n + kRbBM - 1) / kRbBM) * 3 * (int64_t)d;
}

extern "C" int mirec_gemm_nn_resnorm_bwd(const float *A, const float *W, int64_t n, int32_t Kr,
                                         int32_t d, const float *g_out, const float *out,
                                         const float *mean, const float *rstd,
                                         const float *gamma, int32_t relu, float dropout_p,
                                         uint64_t seed, const uint64_t *seed_base, float *d_res,
                                         float *d_z, float *work, float *d_gamma, float *d_beta,
                                         float *d_bias, mirec_stream_t stream) {
  MIREC_CHECK_ARG(n >= 0 && d == kTile && Kr > 0 && Kr % kChunk == 0);
  RbArgs a{g_out, out, mean, rstd, gamma, d_res, d_z, work, relu ? 1 : 0, 0, 0u, 1.f, seed_base};
  MIREC_CHECK_ARG(dropout_params(dropout_p, seed, &a.key, &a.thresh, &a.scale));
  hipStream_t st = (hipStream_t)stream;
  const bool sums = d_gamma || d_beta || d_bias;
  if (n == 0) {  // empty sums; empty tensors may carry null pointers
    if (d_gamma) MIREC_HIP(hipMemsetAsync(d_gamma, 0, sizeof(float) * d, st));
    if (d_beta) MIREC_HIP(hipMemsetAsync(d_beta, 0, sizeof(float) * d, st));
    if (d_bias) MIREC_HIP(hipMemsetAsync(d_bias, 0, sizeof(float) * d, st));
    return MIREC_OK;
  }
  MIREC_CHECK_ARG(A && W && out && mean && rstd && (!sums || work));
  MIREC_CHECK_ARG(((uintptr_t)A | (uintptr_t)W | (uintptr_t)out | (uintptr_t)g_out |
                   (uintptr_t)gamma | (uintptr_t)d_res | (uintptr_t)d_z) % 16 == 0);
  if (!sums) a.partial = nullptr;
  constexpr size_t lds = sizeof(float) * rb_lds_floats<kRbBM>();
  static int rc = -1;
  if (rc < 0)
    rc = hipFuncSetAttribute((const void *)gemm_nn_rnbwd_kernel<kRbBM>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess
             ? 0
             : 1;
  if (rc != 0) return MIREC_ERR_HIP;
  const int64_t grid = (n + kRbBM - 1) / kRbBM;
  hipLaunchKernelGGL(gemm_nn_rnbwd_kernel<kRbBM>, dim3((unsigned)grid), dim3(256), lds, st, A, W,
                     n, (int)Kr, a);
  MIREC_LAUNCH_CHECK();
  if (sums) return mirec_resnorm_reduce_partials(work, grid, d, d_gamma, d_beta, d_bias, stream);
  return MIREC_OK;
}
