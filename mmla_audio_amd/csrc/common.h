// Shared device helpers for the mmla HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MMLA_DEV __device__ __forceinline__

// lo halves of the 3xFP16 split of two scaled values a, b whose hi halves are the f16 pair `hi`
// (bits 0-15 = f16(a), 16-31 = f16(b)): f16(a - hi.a), f16(b - hi.b) by v_fma_mix -- the exact
// difference rounded once, bit-identical to cvt(a - f32(hi.a)) (a - hi is exact in f32); two VALU
// where clang emits cvt + sub + cvt per value.  a, b must be plain VALU results (no MFMA / trans
// producer hazard is visible to the compiler inside the asm).
MMLA_DEV uint32_t split_lo2(float a, float b, uint32_t hi) {
  uint32_t lo;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %3, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(lo) : "v"(a), "v"(hi), "v"(b));
  return lo;
}

// 16 ELU(u) from u16 = 16 u (TF Elu: exp(x) - 1 for x < 0; the power-of-two scaling commutes with every
// rounding).  With e = 16 exp(u) - 16: u > 0 gives 0 < u < e (or e = inf), u <= 0 gives u <= e <= 0,
// so ELU is the median of (u, e, 0) -- one v_med3 instead of a compare and a select.  (Where the
// rounding of e puts it a hair below u, for |u16| ~ 1e-3, the median returns u: within 1e-6.)  Every
// 3xFP16 ELU (rbs, odu, conv_h3's PRO_BN_ELU) uses it, so the fused kernels stay bit-identical to the
// conv_h3 launches they replace.
MMLA_DEV float elu16(float u16) {
  constexpr float L2E_16 = 1.4426950408889634f / 16.0f;   // log2(e) / 2^4
  const float e = fmaf(__builtin_amdgcn_exp2f(u16 * L2E_16), 16.0f, -16.0f);
  return __builtin_amdgcn_fmed3f(u16, e, 0.0f);
}

// XCD-aware workgroup order (MI355X_MICROARCH.md, workgroup dispatch): blocks b and b + 8 share an
// XCD's L2, so the logical id handed to a kernel puts consecutive ids on one XCD -- neighbouring
// tiles of one clip, whose input halos overlap, then meet in the same L2.  Bijective for any count.
MMLA_DEV uint32_t xcd_block_id() {
  const uint32_t nwg = gridDim.x, orig = blockIdx.x;
  const uint32_t xcd = orig % 8u, q = nwg / 8u, r = nwg % 8u;
  return (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + orig / 8u;
}


struct cf {  // complex float held in two VGPRs
  float x, y;
};
MMLA_DEV cf cadd(cf a, cf b) { return {a.x + b.x, a.y + b.y}; }
MMLA_DEV cf csub(cf a, cf b) { return {a.x - b.x, a.y - b.y}; }
MMLA_DEV cf cmul(cf a, cf b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
MMLA_DEV cf cconj(cf a) { return {a.x, -a.y}; }
MMLA_DEV cf cmul_negi(cf a) { return {a.y, -a.x}; }  // -i * a
MMLA_DEV cf cscale(cf a, float s) { return {a.x * s, a.y * s}; }

struct cd {  // complex double
  double x, y;
};
MMLA_DEV cd cadd(cd a, cd b) { return {a.x + b.x, a.y + b.y}; }
MMLA_DEV cd csub(cd a, cd b) { return {a.x - b.x, a.y - b.y}; }
MMLA_DEV cd cmul(cd a, cd b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
MMLA_DEV cd cconj(cd a) { return {a.x, -a.y}; }
MMLA_DEV cd cmul_negi(cd a) { return {a.y, -a.x}; }
MMLA_DEV cd cscale(cd a, double s) { return {a.x * s, a.y * s}; }

template <typename T>
MMLA_DEV T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
template <typename T>
MMLA_DEV T wave_min(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}
template <typename T>
MMLA_DEV T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// A wave that re-reads global memory it stored itself in the same launch must wait for its own
// stores first.  __threadfence_block() does NOT do that on gfx950 (workgroup scope on one CU lowers
// to no vmcnt wait), so a load issued behind it can overtake the store and return the OLD bytes --
// seen only under load: kernels co-running on the CU delayed the stores of the front-ends' scratch /
// cepstra rows, and the re-read took the previous micro-batch's values (tests/test_gpu_corun.py).
// vmcnt(0) returns once every store of the wave is acknowledged by L2; the re-reading loads then
// miss this CU's L1 (no earlier load of these lines in this launch) and read L2.
MMLA_DEV void wave_stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Kernel launch wrappers are declared extern "C++" here and defined in the .hip files; the C ABI
// (capi.cpp) calls them.
struct OdFeTables;  // device constant tables for the OD front-end
