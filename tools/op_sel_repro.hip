// Minimal probe for the fused dX + LayerNorm-backward finding (DESIGN.md
// §9.1): a packed-f32 VALU op that reads the HIGH dword of a 64-bit VGPR
// pair through op_sel (v_pk_add_f32 ... op_sel:[0,1]), the pair built before
// a bf16 MFMA loop and read after it — the shape the compiler gave the
// failing kernel.  Every lane checks that it got its own high dword.  Not
// part of libmirec: built and run by tools/op_sel_repro.py.
//
// Knobs: iters (MFMAs before the read), use_opsel (0: the same value built
// without op_sel), mfma_odd_only (only the waves in an odd hardware wave
// slot of their SIMD run the MFMA loop — HW_ID.WAVE_ID, read with s_getreg —
// so waves that issue no MFMA share every SIMD with waves that do: does
// another wave's MFMA matter?), nop_rounds
// (s_nop 7 x rounds between the loop and the read), pair64 (the pair built
// by v_mov_b64 or by two v_mov_b32).  bad[128]: wrong lanes by (wave slot
// parity, lane); out keeps every lane's two results for the host to classify.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

extern "C" __global__ __launch_bounds__(256) void op_sel_probe(const float *__restrict__ in,
                                                               float *__restrict__ out,
                                                               int32_t *__restrict__ bad,
                                                               int iters, int use_opsel,
                                                               int mfma_odd_only, int nop_rounds,
                                                               int pair64) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  // HW_REG_HW_ID (hwreg 4) bits [3:0]: the wave's slot on its SIMD
  const int par = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 4) & 1;
  const f32x2 src = {in[2 * t], in[2 * t + 1]};
  f32x2 pair;
  if (pair64) {
    asm volatile("v_mov_b64 %0, %1" : "=v"(pair) : "v"(src));
  } else {
    float lo, hi;
    asm volatile("v_mov_b32 %0, %1" : "=v"(lo) : "v"(src.x));
    asm volatile("v_mov_b32 %0, %1" : "=v"(hi) : "v"(src.y));
    pair = f32x2{lo, hi};
  }
  // MFMA work between the pair's definition and its use (operands from the
  // thread index so the loop is not folded)
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  bf16x8 a, b;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    a[e] = (__bf16)(float)((t + e) & 7);
    b[e] = (__bf16)(float)((t * 3 + e) & 5);
  }
  const int my_iters = (mfma_odd_only && par == 0) ? 0 : iters;
  for (int i = 0; i < my_iters; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  for (int i = 0; i < nop_rounds; ++i) asm volatile("s_nop 7");
  const f32x2 zero = {0.f, 0.f};
  f32x2 r;
  if (use_opsel) {
    // low lane <- 0 + pair.hi, high lane <- 0 + pair.hi
    asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]"
                 : "=v"(r) : "v"(zero), "v"(pair));
  } else {
    f32x2 hh = {pair.y, pair.y};
    asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(zero), "v"(hh));
  }
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) s += acc[q];
  out[3 * t] = r.x;
  out[3 * t + 1] = r.y;
  out[3 * t + 2] = s;
  if (r.x != src.y || r.y != src.y) atomicAdd(bad + 64 * par + (threadIdx.x & 63), 1);
}

extern "C" int op_sel_probe_launch(const float *in, float *out, int32_t *bad, int blocks, int iters,
                                   int use_opsel, int mfma_odd_only, int nop_rounds, int pair64) {
  hipLaunchKernelGGL(op_sel_probe, dim3(blocks), dim3(256), 0, 0, in, out, bad, iters, use_opsel,
                     mfma_odd_only, nop_rounds, pair64);
  return (int)hipGetLastError();
}
