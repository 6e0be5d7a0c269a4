// SpeakerIdentification res_unit without pooling (speaker_identification.py:168-190; units 2-3, 5-6,
// 8-9 of the nine):
//     y = x + Conv1D_b(ReLU(BN_mid(Conv1D_a(ReLU(BN_in(x))))))        Conv1D(C, 3, 'same')
// as ONE kernel per unit.  The SI Conv1D layers run at 3-5.4 TB/s of HBM (profiles/
// pmc_traffic_si_pipeline.json against the kernel stats): the stack is bandwidth-bound, and the
// two-launch form moves t1 out to HBM and back (write + read) and x twice.  Here a workgroup stages
// ROWS + 2 rows of x (BN_in + ReLU + 3xFP16 split, as conv_h3's staging), computes the ROWS rows of
// t1 its output rows need (GEMM a), writes them back into the same LDS already BN_mid + ReLU'd and
// split, and computes ROWS - 2 output rows (GEMM b) + bias + residual.  t1 never leaves the CU.
//
// The pool units (1, 4, 7: MaxPool1D(2, 'same') of x into BN_in, and the residual is the shortcut
// Conv1D(C, 1, strides=2) of x) run the same way with POOL: x's two source rows are max-pooled while
// staging (conv_h3's PIN) and the epilogue computes the shortcut as a small 3xFP16 GEMM per 32-row
// tile (conv_h3's EPI_ADD_SC), so the pool unit's t1 stays on chip too.
//
// Bit-identical to the conv_h3 pair it replaces: the same staged operands (values and 2^4 scale),
// the same MFMA sequence per output element (channel chunks of 32, then taps, then k-steps, the three
// 3xFP16 products in conv_h3's order into one accumulator), the same epilogue arithmetic, and the
// same zero rows for taps that leave a clip (conv_h3's TW = 1 zero row) or the row sequence.
#include "common.h"
#include "conv.h"
#include "siu.h"

#include <type_traits>



namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

constexpr int CK = 32;                 // channel chunk (conv_h3's k order)
constexpr int KS = CK / 16;
constexpr int TAPS = 3;
constexpr float ACT_SCALE = 16.0f;
constexpr float ACT_RANGE = 65504.0f / ACT_SCALE;

MMLA_DEV float bn_relu(float v, float sc, float sh) { return fmaxf(fmaf(v, sc, sh), 0.0f); }

// CIN input / C output channels; NW waves; ROWS = t1 rows per workgroup = a multiple of the waves'
// 32-row MFMA tiles; output rows per workgroup R = ROWS - 2 (t1 needs one row of halo each side, x
// two).  POOL: a pool unit (rows are pooled rows, a.t_src the unpooled rows per clip)
// FIN (the last unit): the epilogue writes BN + ReLU + AveragePooling1D(4) of the unit's output
// (speaker_identification.py:208-212, nets.hip bn_relu_avgpool4_kernel's arithmetic) instead of the
// output itself; tiles then hold a multiple of 4 output rows, so no pool window straddles two
template <int CIN, int C, int ROWS, int NW, bool POOL, bool FIN, int MINW = 2>
__global__ void __launch_bounds__(64 * NW, MINW) siu_kernel(SiuArgs a) {
  constexpr int NT = 64 * NW;
  constexpr int WN = C / 32;           // waves along N (32 columns each), as conv_h3 with BN = C
  constexpr int WM = NW / WN;
  constexpr int MT = ROWS / (WM * 32);
  constexpr int NCHX = CIN / CK;       // channel chunks of GEMM a / GEMM b
  constexpr int NCH = C / CK;
  constexpr int LDPX = CIN + 8;        // fp16 per staged x row (16-B pad, as conv_h3)
  constexpr int LDP = C + 8;           // ... per t1 row
  constexpr int R = FIN ? (ROWS - 2) / 4 * 4 : ROWS - 2;
  constexpr int XR = ROWS + 2;         // staged x rows r0 - 2 .. r0 + ROWS - 1
  constexpr int ZR = XR;               // the zero row (taps leaving a clip), in either row pitch
  constexpr int QPP = CK / 4;          // float4 per row and chunk
  constexpr int MAXT = (XR * QPP + NT - 1) / NT;
  static_assert(WM * WN == NW && MT * WM * 32 == ROWS && NT % QPP == 0, "tiling");
  static_assert(POOL || CIN == C, "a unit without pooling keeps its width");
  __shared__ __attribute__((aligned(16))) _Float16 lhi[(XR + 1) * LDP];
  __shared__ __attribute__((aligned(16))) _Float16 llo[(XR + 1) * LDP];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int64_t HH = (int64_t)a.n * a.t;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int koff = (lane >> 5) * 8;
  bool rbad = false;

  if (tid < LDPX / 8) {   // the zero row (x pitch)
    *reinterpret_cast<f16x8*>(lhi + ZR * LDPX + 8 * tid) = f16x8{};
    *reinterpret_cast<f16x8*>(llo + ZR * LDPX + 8 * tid) = f16x8{};
  }

  // ---- stage x: rows r0 - 2 + j, BN_in + ReLU, x 2^4, split (all chunks, one barrier) ------------
  //      (POOL: row g = (clip, tt) is the max of the clip's unpooled rows 2 tt, 2 tt + 1)
  {
    const int q = tid % QPP;
#pragma unroll 1
    for (int ch = 0; ch < NCHX; ++ch) {
      const int ci = ch * CK + 4 * q;
      const float4 sc = *reinterpret_cast<const float4*>(a.s_in + ci);
      const float4 sh = *reinterpret_cast<const float4*>(a.t_in + ci);
      float4 pre[MAXT];
      uint32_t valid = 0;
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        const int task = tid + j * NT;
        pre[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        const int64_t g = r0 - 2 + task / QPP;
        if (task < XR * QPP && g >= 0 && g < HH) {
          if constexpr (POOL) {
            const int64_t cl = g / a.t;
            const int tt = (int)(g - cl * a.t);
            const float* src = a.x + (cl * a.t_src + 2 * tt) * CIN + ci;
            float4 v = *reinterpret_cast<const float4*>(src);
            if (2 * tt + 1 < a.t_src) {
              const float4 u = *reinterpret_cast<const float4*>(src + CIN);
              v = make_float4(fmaxf(v.x, u.x), fmaxf(v.y, u.y), fmaxf(v.z, u.z), fmaxf(v.w, u.w));
            }
            pre[j] = v;
          } else {
            pre[j] = *reinterpret_cast<const float4*>(a.x + g * C + ci);
          }
          valid |= 1u << j;
        }
      }
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        const int task = tid + j * NT;
        if (task >= XR * QPP) continue;
        float4 v = pre[j];
        if (valid & (1u << j)) {
          v.x = bn_relu(v.x, sc.x, sh.x);
          v.y = bn_relu(v.y, sc.y, sh.y);
          v.z = bn_relu(v.z, sc.z, sh.z);
          v.w = bn_relu(v.w, sc.w, sh.w);
        }
        rbad |= !(fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))) < ACT_RANGE);
        v.x *= ACT_SCALE;
        v.y *= ACT_SCALE;
        v.z *= ACT_SCALE;
        v.w *= ACT_SCALE;
        f16x4 hv, lv;
        hv[0] = (_Float16)v.x;
        hv[1] = (_Float16)v.y;
        hv[2] = (_Float16)v.z;
        hv[3] = (_Float16)v.w;
        {
          const uint2 hu_ = __builtin_bit_cast(uint2, hv);
          lv = __builtin_bit_cast(f16x4, make_uint2(split_lo2(v.x, v.y, hu_.x), split_lo2(v.z, v.w, hu_.y)));
        }
        const int row = task / QPP;
        *reinterpret_cast<f16x4*>(lhi + row * LDPX + ci) = hv;
        *reinterpret_cast<f16x4*>(llo + row * LDPX + ci) = lv;
      }
    }
  }
  __syncthreads();

  // B fragments (conv_h3_split_weights order): per tap, 16-channel k-step and 32-column tile
  constexpr size_t kstride = (size_t)(C / 32) * 512;
  const int lofs = wn * 512 + lane * 8;
  // this lane's A rows and, per tap, the LDS row it reads (the zero row where the tap leaves the clip);
  // NCHK channel chunks of A rows LDPA halfs apart
  auto gemm = [&](auto nchk_c, auto ldpa_c, const uint16_t* __restrict__ wh,
                  const uint16_t* __restrict__ wl, int64_t g_row0, f32x16 (&acc)[MT]) {
    constexpr int NCHK = decltype(nchk_c)::value, LDPA = decltype(ldpa_c)::value;
    constexpr size_t tap_stride = (size_t)C * NCHK * CK;
    int mrow[MT], trow[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      mrow[mt] = (wm * MT + mt) * 32 + (lane & 31);
      const int64_t g = g_row0 + mrow[mt];                 // the global row of this A row
      trow[mt] = (int)(((g % a.t) + a.t) % a.t);           // its position in its clip
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[mt][i] = 0.0f;
    }
#pragma unroll 1
    for (int ch = 0; ch < NCHK; ++ch) {
#pragma unroll 1
      for (int tap = 0; tap < TAPS; ++tap) {   // (unrolled, every tap's A reads were hoisted: spills)
        f16x8 bh[KS], bl[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const size_t u = tap * tap_stride + (size_t)(ch * KS + s) * kstride + lofs;
          bh[s] = *reinterpret_cast<const f16x8*>(wh + u);
          bl[s] = *reinterpret_cast<const f16x8*>(wl + u);
        }
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const int src = trow[mt] + tap - 1;
            const int off = (src < 0 || src >= a.t ? ZR : mrow[mt] + tap) * LDPA + ch * CK + 16 * s + koff;
            const f16x8 ah = *reinterpret_cast<const f16x8*>(lhi + off);
            const f16x8 al = *reinterpret_cast<const f16x8*>(llo + off);
            acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s], acc[mt], 0, 0, 0);
            acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[s], acc[mt], 0, 0, 0);
            acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], acc[mt], 0, 0, 0);
          }
      }
    }
  };

  const int co = wn * 32 + (lane & 31);
  const int hsel = 4 * (lane >> 5);
  f32x16 acc[MT];
  // ---- GEMM a: t1 rows r0 - 1 + m, m < ROWS (x LDS row of t1 row m at tap dy: m + dy) -------------
  gemm(std::integral_constant<int, NCHX>{}, std::integral_constant<int, LDPX>{}, a.wah, a.wal, r0 - 1, acc);
  __syncthreads();   // every wave has read x
  if constexpr (LDPX != LDP) {   // the zero row again, in t1's pitch
    if (tid < LDP / 8) {
      *reinterpret_cast<f16x8*>(lhi + ZR * LDP + 8 * tid) = f16x8{};
      *reinterpret_cast<f16x8*>(llo + ZR * LDP + 8 * tid) = f16x8{};
    }
  }
  {
    const float b = a.ba[co], s2 = a.s_mid[co], t2 = a.t_mid[co];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = (wm * MT + mt) * 32 + (r & 3) + 8 * (r >> 2) + hsel;
        const int64_t g = r0 - 1 + m;
        float v = 0.0f;
        if (g >= 0 && g < HH) {   // rows outside the sequence stage as zeros (conv_h3's valid mask)
          v = bn_relu(fmaf(acc[mt][r], a.ua, b), s2, t2);
          rbad |= !(fabsf(v) < ACT_RANGE);
        }
        v *= ACT_SCALE;
        const _Float16 hv = (_Float16)v;
        lhi[m * LDP + co] = hv;
        llo[m * LDP + co] = (_Float16)(v - (float)hv);
      }
  }
  __syncthreads();
  // ---- GEMM b: output rows r0 + m, m < R (t1 LDS row of output row m at tap dy: m + dy) -----------
  // EARLY: the residuals of all MT tiles loaded before GEMM b, so their latency hides under it
  // (units without pooling whose registers allow it: MT 2)
  constexpr bool EARLY = !POOL && MT <= 2;
  float ersd[EARLY ? MT : 1][16];
  if constexpr (EARLY) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = (wm * MT + mt) * 32 + (r & 3) + 8 * (r >> 2) + hsel;
        const int64_t g = r0 + m;
        ersd[mt][r] = m < R && g < HH ? a.x[g * C + co] : 0.0f;
      }
  }
  gemm(std::integral_constant<int, NCH>{}, std::integral_constant<int, LDP>{}, a.wbh, a.wbl, r0, acc);
  {
    const float b = a.bb[co];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {   // one 32-row tile at a time: 16 residuals live, not 16 MT
      float rsd[16];
      if constexpr (POOL) {
        // the shortcut Conv1D(1, stride 2) of x as conv_h3's EPI_ADD_SC: A row = the output row's
        // source row 2 tt of x (raw, x 2^4, split), 16-channel k-steps, its own accumulator
        f32x16 sacc;
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[i] = 0.0f;
        const int64_t g = r0 + (wm * MT + mt) * 32 + (lane & 31);
        const bool sok = g < HH;
        const int64_t gs = sok ? g : 0;
        const int64_t cl = gs / a.t;
        const int tt = (int)(gs - cl * a.t);
        const float* sxp = a.x + (cl * a.t_src + 2 * tt) * CIN + koff;
#pragma unroll
        for (int s = 0; s < CIN / 16; ++s) {
          const f16x8 sbh = *reinterpret_cast<const f16x8*>(a.wsh + (size_t)s * kstride + lofs);
          const f16x8 sbl = *reinterpret_cast<const f16x8*>(a.wsl + (size_t)s * kstride + lofs);
          float4 x0 = make_float4(0.f, 0.f, 0.f, 0.f), x1 = x0;
          if (sok) {
            x0 = *reinterpret_cast<const float4*>(sxp + 16 * s);
            x1 = *reinterpret_cast<const float4*>(sxp + 16 * s + 4);
          }
          const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
          f16x8 xh, xl;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            rbad |= !(fabsf(xv[k]) < ACT_RANGE);
            const float v = xv[k] * ACT_SCALE;
            xh[k] = (_Float16)v;
            xl[k] = (_Float16)(v - (float)xh[k]);
          }
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, sbl, sacc, 0, 0, 0);
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, sbh, sacc, 0, 0, 0);
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, sbh, sacc, 0, 0, 0);
        }
        const float bsc = a.bs[co];
#pragma unroll
        for (int r = 0; r < 16; ++r) rsd[r] = fmaf(sacc[r], a.us, bsc);
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = (wm * MT + mt) * 32 + (r & 3) + 8 * (r >> 2) + hsel;
          const int64_t g = r0 + m;
          rsd[r] = EARLY ? ersd[EARLY ? mt : 0][r] : (m < R && g < HH ? a.x[g * C + co] : 0.0f);
        }
      }
      if constexpr (FIN) {
        // registers 4 q .. 4 q + 3 are the rows m0 .. m0 + 3, m0 = 8 q + hsel (+ tile): with r0, R
        // and t multiples of 4 each group is one pool window of one clip
        const float fs = a.fs[co], ft = a.ft[co];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int m0 = (wm * MT + mt) * 32 + 8 * q + hsel;
          const int64_t g0 = r0 + m0;
          if (m0 < R && g0 < HH) {
            float sum = 0.0f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float val = fmaf(acc[mt][4 * q + j], a.ub, b);
              val += rsd[4 * q + j];
              sum += fmaxf(fmaf(val, fs, ft), 0.0f);
            }
            a.seq[(g0 >> 2) * C + co] = sum / 4.0f;
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = (wm * MT + mt) * 32 + (r & 3) + 8 * (r >> 2) + hsel;
          const int64_t g = r0 + m;
          if (m < R && g < HH) {
            float val = fmaf(acc[mt][r], a.ub, b);
            val += rsd[r];
            a.y[g * C + co] = val;
          }
        }
      }
    }
  }
  if (rbad && a.range_flag) *a.range_flag = 1;
}

template <int CIN, int C, int ROWS, int NW, bool POOL = false, bool FIN = false, int MINW = 2>
hipError_t launch(const SiuArgs& a, hipStream_t s) {
  constexpr int R = FIN ? (ROWS - 2) / 4 * 4 : ROWS - 2;
  const int64_t rows = (int64_t)a.n * a.t;
  const int64_t blocks = (rows + R - 1) / R;
  hipLaunchKernelGGL((siu_kernel<CIN, C, ROWS, NW, POOL, FIN, MINW>), dim3((unsigned)blocks), dim3(64 * NW), 0, s, a);
  return hipGetLastError();
}

}  // namespace

bool siu_supported(int c) { return c == 32 || c == 64 || c == 128; }

bool siu_final_supported(int c) { return c == 128; }

bool sipu_supported(int cin, int c) {
  return (cin == 32 && c == 32) || (cin == 32 && c == 64) || (cin == 64 && c == 128);
}

hipError_t sipu_launch(const SiuArgs& a, int cin, int c, hipStream_t s) {
  if ((int64_t)a.n * a.t == 0) return hipSuccess;
  if (!a.x || !a.y || a.x == a.y || a.t < 1 || a.t != (a.t_src + 1) / 2 || !a.wsh || !a.wsl || !a.bs)
    return hipErrorInvalidValue;
  // unit 4 (32 -> 64 channels): 128-row tiles at 3 waves per SIMD (112 VGPRs, 37.7 KB) instead of
  // 256-row tiles at 2 (152 VGPRs, 74.6 KB): SI +1.1 % (A/B, 2 rounds; the same choice for the other
  // units -- C 32 pool / non-pool at 128 rows and 4 waves per SIMD, C 64 at 128 rows -- was neutral)
  if (cin == 32 && c == 32) return launch<32, 32, 256, 4, true>(a, s);
  if (cin == 32 && c == 64) return launch<32, 64, 128, 4, true, false, 3>(a, s);
  // unit 7 (64 -> 128): 64-row tiles at 3 waves per SIMD (158 VGPRs) instead of 128-row tiles at 2
  // (227): SI +1.0 % (A/B, 2 rounds; 64-row tiles for units 8 / 9 at 3 waves: +0.1-0.6 % / noise)
  if (cin == 64 && c == 128) return launch<64, 128, 64, 4, true, false, 3>(a, s);
  return hipErrorInvalidValue;
}

hipError_t siu_launch(const SiuArgs& a, int c, hipStream_t s) {
  if ((int64_t)a.n * a.t == 0) return hipSuccess;
  if (a.seq) {   // the last unit with the final BN + ReLU + AveragePooling1D(4) in its epilogue
    if (!a.x || !a.fs || !a.ft || a.t % 4 != 0 || !siu_final_supported(c)) return hipErrorInvalidValue;
    return launch<128, 128, 128, 4, false, true>(a, s);
  }
  if (!a.x || !a.y || a.x == a.y || a.t < 1) return hipErrorInvalidValue;
  // Tiles (4 waves): C = 32 256 t1 rows (MT 2, 134 VGPRs, 3 workgroups per CU); C = 64 256 rows and
  // C = 128 128 rows (MT 4, 242 VGPRs once the residual epilogue went tile by tile, 2 per CU).
  // Measured per unit and SI step against the conv_h3 pair: C = 32 1.004 vs 1.033 ms, C = 64 (128-row
  // tiles) 1.061 vs 1.203 ms, C = 128 with 64-row tiles 1.672 vs 1.625 ms (B streamed per 62 output
  // rows); with the MT 4 tiles SI 2.45 -> 2.51 M clips/s (A/B, 2 rounds; the conv stage itself
  // +0.8 %).  Tried: 8-wave workgroups
  // (one per CU) and 512-row C = 32 tiles (occupancy 1): slower
  if (c == 32) return launch<32, 32, 256, 4>(a, s);
  if (c == 64) return launch<64, 64, 256, 4>(a, s);
  if (c == 128) return launch<128, 128, 128, 4>(a, s);
  return hipErrorInvalidValue;
}
