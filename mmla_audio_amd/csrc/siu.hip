// SpeakerIdentification res_unit without pooling (speaker_identification.py:168-190; units 2-3, 5-6,
// 8-9 of the nine):
//     y = x + Conv1D_b(ReLU(BN_mid(Conv1D_a(ReLU(BN_in(x))))))        Conv1D(C, 3, 'same')
// as ONE kernel per unit.  A workgroup stages ROWS + 2 rows of x (BN_in + ReLU + 3xFP16 split, as
// conv_h3's staging), computes the ROWS rows of t1 its output rows need (GEMM a), writes them back
// into the same LDS already BN_mid + ReLU'd and split, and computes ROWS - 2 output rows (GEMM b) +
// bias + residual.  t1 never leaves the CU.
//
// The pool units (1, 4, 7: MaxPool1D(2, 'same') of x into BN_in, and the residual is the shortcut
// Conv1D(C, 1, strides=2) of x) run the same way with POOL: x's two source rows are max-pooled while
// staging (conv_h3's PIN) and the epilogue computes the shortcut as a small 3xFP16 GEMM per 32-row
// tile (conv_h3's EPI_ADD_SC), so the pool unit's t1 stays on chip too.
//
// Both GEMMs run as C^T = W^T X^T (weights the A operand): a lane's accumulator quad is 4 adjacent
// channels of one row, so t1 goes back to LDS as 8-B hi / lo quads and the epilogue moves float4s.
// Row -> (clip, position) by a multiply-high division (SiuArgs::tdiv_*), 32-bit offsets, the 2^4
// operand scale folded into the BatchNorm parameters, and a running range maximum: the round-6
// counters put this kernel at ~23 VALU per MFMA before (profiles/r6_pmc_si_pipeline_summary.txt).
//
// Bit-identical to the conv_h3 pair it replaces: the same staged operands (values and 2^4 scale:
// fma(v, 16 s, 16 t) = 16 fma(v, s, t) exactly), the same MFMA sequence per output element (channel
// chunks of 32, then taps, then k-steps, the three 3xFP16 products in conv_h3's order into one
// accumulator; the transposed product sums the same terms in the same order), the same epilogue
// arithmetic, and the same zero rows for taps that leave a clip (conv_h3's TW = 1 zero row).
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
constexpr float SPLIT_MAX = 65504.0f;  // largest finite fp16 (operands are compared once scaled)

MMLA_DEV __amdgpu_buffer_rsrc_t siu_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)0xffffffff, 0x00020000);
}
MMLA_DEV float4 ld4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}
MMLA_DEV f16x8 ldw(__amdgpu_buffer_rsrc_t r, int lofs, int u) {   // 16 B of a split weight
  return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)lofs * 2u, u * 2, 0));
}
// x / t for x < 2^31 (SiuArgs::tdiv_m, tdiv_s from siu_fastdiv)
MMLA_DEV uint32_t tdiv(uint32_t x, uint32_t m, uint32_t s) { return (__umulhi(x, m) + x) >> s; }

// v' = max(fma(v, sc', sh'), 0) (the BN already x 2^4), split into hi / lo quads; rmax tracks the
// largest v' (post-ReLU: never NaN, never negative)
MMLA_DEV void bn_split4(float4 v, float4 sc, float4 sh, f16x4& h, f16x4& l, float& rmax) {
  const float a = fmaxf(fmaf(v.x, sc.x, sh.x), 0.0f), b = fmaxf(fmaf(v.y, sc.y, sh.y), 0.0f);
  const float c = fmaxf(fmaf(v.z, sc.z, sh.z), 0.0f), d = fmaxf(fmaf(v.w, sc.w, sh.w), 0.0f);
  rmax = fmaxf(rmax, fmaxf(fmaxf(a, b), fmaxf(c, d)));
  h[0] = (_Float16)a;
  h[1] = (_Float16)b;
  h[2] = (_Float16)c;
  h[3] = (_Float16)d;
  const uint2 hu = __builtin_bit_cast(uint2, h);
  l = __builtin_bit_cast(f16x4, make_uint2(split_lo2(a, b, hu.x), split_lo2(c, d, hu.y)));
}

// CIN input / C output channels; NW waves; ROWS = t1 rows per workgroup = a multiple of the waves'
// 32-row MFMA tiles; output rows per workgroup R = ROWS - 2 (t1 needs one row of halo each side, x
// two).  POOL: a pool unit (rows are pooled rows, a.t_src the unpooled rows per clip)
// FIN (the last unit): the epilogue writes BN + ReLU + AveragePooling1D(4) of the unit's output
// (speaker_identification.py:208-212, nets.hip bn_relu_avgpool4_kernel's arithmetic) instead of the
// output itself; tiles then hold a multiple of 4 output rows, so no pool window straddles two.  FIN's
// GEMM b keeps the natural C = X W form (a lane's quad = 4 rows of one channel = one pool window).
template <int CIN, int C, int ROWS, int NW, bool POOL, bool FIN, int MINW = 2>
__global__ void __launch_bounds__(64 * NW, MINW) siu_kernel(SiuArgs a) {
  constexpr int NT = 64 * NW;
  constexpr int WN = C / 32;           // waves along N (32 channels each)
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
  // per-channel parameters: [0] b_a, [1] 16 s_mid, [2] 16 t_mid, [3] b_b, [4] the shortcut bias
  __shared__ __attribute__((aligned(16))) float spar[5 * C];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int HH = a.n * a.t;                       // rows of the batch (< 2^24, siu_launch checks)
  const int r0 = (int)blockIdx.x * R;
  const int koff = (lane >> 5) * 8;
  const int h4 = 4 * (lane >> 5);
  const uint32_t tm = a.tdiv_m, ts = a.tdiv_s;
  float rmax = 0.0f;                              // the largest scaled operand this thread split
  bool rbad = false;                              // ... or a raw shortcut operand out of range / NaN
  const __amdgpu_buffer_rsrc_t rx = siu_rsrc(a.x);

  if (tid < LDPX / 8) {   // the zero row (x pitch)
    *reinterpret_cast<f16x8*>(lhi + ZR * LDPX + 8 * tid) = f16x8{};
    *reinterpret_cast<f16x8*>(llo + ZR * LDPX + 8 * tid) = f16x8{};
  }
  for (int i = tid; i < C; i += NT) {
    spar[i] = a.ba[i];
    spar[C + i] = ACT_SCALE * a.s_mid[i];
    spar[2 * C + i] = ACT_SCALE * a.t_mid[i];
    spar[3 * C + i] = a.bb[i];
    spar[4 * C + i] = POOL ? a.bs[i] : 0.0f;
  }

  // ---- stage x: rows r0 - 2 + j, BN_in + ReLU, x 2^4, split (all chunks, one barrier) ------------
  //      (POOL: row g = (clip, tt) is the max of the clip's unpooled rows 2 tt, 2 tt + 1).  Rows
  //      outside the batch load row 0 / HH - 1 instead: GEMM a reaches them only through taps that
  //      leave a clip (the zero row) or for t1 rows outside the batch, which GEMM b never reads.
  {
    const int q = tid % QPP;
#pragma unroll 1
    for (int ch = 0; ch < NCHX; ++ch) {
      const int ci = ch * CK + 4 * q;
      float4 sc = *reinterpret_cast<const float4*>(a.s_in + ci);
      float4 sh = *reinterpret_cast<const float4*>(a.t_in + ci);
      sc = make_float4(ACT_SCALE * sc.x, ACT_SCALE * sc.y, ACT_SCALE * sc.z, ACT_SCALE * sc.w);
      sh = make_float4(ACT_SCALE * sh.x, ACT_SCALE * sh.y, ACT_SCALE * sh.z, ACT_SCALE * sh.w);
      float4 pre[MAXT];
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        const int task = tid + j * NT;
        const int g = min(max(r0 - 2 + task / QPP, 0), HH - 1);
        if constexpr (POOL) {
          const uint32_t cl = tdiv((uint32_t)g, tm, ts);
          const int tt = g - (int)cl * a.t;
          const uint32_t src = ((uint32_t)cl * (uint32_t)a.t_src + 2u * tt) * (CIN * 4u) + ci * 4u;
          const float4 v = ld4(rx, src);
          const float4 u = ld4(rx, 2 * tt + 1 < a.t_src ? src + CIN * 4u : src);
          pre[j] = make_float4(fmaxf(v.x, u.x), fmaxf(v.y, u.y), fmaxf(v.z, u.z), fmaxf(v.w, u.w));
        } else {
          pre[j] = ld4(rx, (uint32_t)g * (C * 4u) + ci * 4u);
        }
      }
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        const int task = tid + j * NT;
        if (MAXT * NT > XR * QPP && task >= XR * QPP) continue;
        f16x4 hv, lv;
        bn_split4(pre[j], sc, sh, hv, lv, rmax);
        const int row = task / QPP;
        *reinterpret_cast<f16x4*>(lhi + row * LDPX + ci) = hv;
        *reinterpret_cast<f16x4*>(llo + row * LDPX + ci) = lv;
      }
    }
  }
  __syncthreads();

  // weight fragments (conv_h3_split_weights order): per tap, 16-channel k-step and 32-column tile
  constexpr int kstride = (C / 32) * 512;
  const int lofs = wn * 512 + lane * 8;
  // this lane's LDS row per tile and, per tap, that row or the zero row where the tap leaves the
  // clip; NCHK channel chunks of rows LDPA halfs apart.  CT: acc = W^T X^T (lane = row, quads of
  // channels), else acc = X W (lane = channel, quads of rows)
  auto gemm = [&](auto nchk_c, auto ldpa_c, auto ct_c, const uint16_t* wh, const uint16_t* wl, int g_row0,
                  f32x16 (&acc)[MT]) {
    constexpr int NCHK = decltype(nchk_c)::value, LDPA = decltype(ldpa_c)::value;
    constexpr bool CT = decltype(ct_c)::value;
    constexpr int tap_stride = C * NCHK * CK;
    const __amdgpu_buffer_rsrc_t rwh = siu_rsrc(wh), rwl = siu_rsrc(wl);
    int mrow[MT], trow[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      mrow[mt] = (wm * MT + mt) * 32 + (lane & 31);
      const uint32_t gp = (uint32_t)(g_row0 + mrow[mt] + a.t);            // >= 0
      trow[mt] = (int)(gp - tdiv(gp, tm, ts) * (uint32_t)a.t);            // the row's position in its clip
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
          const int u = tap * tap_stride + (ch * KS + s) * kstride;
          bh[s] = ldw(rwh, lofs, u);
          bl[s] = ldw(rwl, lofs, u);
        }
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const int src = trow[mt] + tap - 1;
            const int off = (src < 0 || src >= a.t ? ZR : mrow[mt] + tap) * LDPA + ch * CK + 16 * s + koff;
            const f16x8 ah = *reinterpret_cast<const f16x8*>(lhi + off);
            const f16x8 al = *reinterpret_cast<const f16x8*>(llo + off);
            if constexpr (CT) {
              acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bl[s], ah, acc[mt], 0, 0, 0);
              acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[s], al, acc[mt], 0, 0, 0);
              acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[s], ah, acc[mt], 0, 0, 0);
            } else {
              acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s], acc[mt], 0, 0, 0);
              acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[s], acc[mt], 0, 0, 0);
              acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], acc[mt], 0, 0, 0);
            }
          }
      }
    }
  };

  f32x16 acc[MT];
  // ---- GEMM a: t1 rows r0 - 1 + m, m < ROWS (x LDS row of t1 row m at tap dy: m + dy) -------------
  gemm(std::integral_constant<int, NCHX>{}, std::integral_constant<int, LDPX>{}, std::true_type{}, a.wah, a.wal,
       r0 - 1, acc);
  __syncthreads();   // every wave has read x
  if constexpr (LDPX != LDP) {   // the zero row again, in t1's pitch
    if (tid < LDP / 8) {
      *reinterpret_cast<f16x8*>(lhi + ZR * LDP + 8 * tid) = f16x8{};
      *reinterpret_cast<f16x8*>(llo + ZR * LDP + 8 * tid) = f16x8{};
    }
  }
  {
    // lane: t1 row m (its tile's lane & 31), channels co0 + 0..3 of each quad q
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = (wm * MT + mt) * 32 + (lane & 31);
      const int g = r0 - 1 + m;
      float tmax = 0.0f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co0 = wn * 32 + 8 * q + h4;
        const float4 b = *reinterpret_cast<const float4*>(spar + co0);
        const float4 s2 = *reinterpret_cast<const float4*>(spar + C + co0);
        const float4 t2 = *reinterpret_cast<const float4*>(spar + 2 * C + co0);
        const float4 v = make_float4(fmaf(acc[mt][4 * q], a.ua, b.x), fmaf(acc[mt][4 * q + 1], a.ua, b.y),
                                     fmaf(acc[mt][4 * q + 2], a.ua, b.z), fmaf(acc[mt][4 * q + 3], a.ua, b.w));
        f16x4 hv, lv;
        bn_split4(v, s2, t2, hv, lv, tmax);
        *reinterpret_cast<f16x4*>(lhi + m * LDP + co0) = hv;
        *reinterpret_cast<f16x4*>(llo + m * LDP + co0) = lv;
      }
      // t1 rows outside the batch are never read (see staging): kept out of the range guard
      if (g >= 0 && g < HH) rmax = fmaxf(rmax, tmax);
    }
  }
  __syncthreads();
  // ---- GEMM b: output rows r0 + m, m < R (t1 LDS row of output row m at tap dy: m + dy) -----------
  if constexpr (!FIN) {
    // EARLY: the residuals of all MT tiles loaded before GEMM b, so their latency hides under it
    // (units without pooling whose registers allow it: MT 2)
    constexpr bool EARLY = !POOL && MT <= 2;
    float4 ersd[EARLY ? MT : 1][4];
    auto rsd_off = [&](int mt, int q) {
      const int g = min(r0 + (wm * MT + mt) * 32 + (lane & 31), HH - 1);
      return (uint32_t)g * (C * 4u) + (wn * 32 + 8 * q + h4) * 4u;
    };
    if constexpr (EARLY) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int q = 0; q < 4; ++q) ersd[mt][q] = ld4(rx, rsd_off(mt, q));
    }
    gemm(std::integral_constant<int, NCH>{}, std::integral_constant<int, LDP>{}, std::true_type{}, a.wbh, a.wbl, r0,
         acc);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {   // one 32-row tile at a time: 16 residuals live, not 16 MT
      const int m = (wm * MT + mt) * 32 + (lane & 31);
      const int g = r0 + m;
      float4 rsd[4];
      if constexpr (POOL) {
        // the shortcut Conv1D(1, stride 2) of x as conv_h3's EPI_ADD_SC: the row's source row 2 tt of
        // x (raw, x 2^4, split) is the B operand, 16-channel k-steps, its own accumulator
        f32x16 sacc;
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[i] = 0.0f;
        const int gs = min(g, HH - 1);
        const uint32_t cl = tdiv((uint32_t)gs, tm, ts);
        const int tt = gs - (int)cl * a.t;
        const uint32_t sxo = ((uint32_t)cl * (uint32_t)a.t_src + 2u * tt) * (CIN * 4u) + koff * 4u;
        const __amdgpu_buffer_rsrc_t rsh = siu_rsrc(a.wsh), rsl = siu_rsrc(a.wsl);
#pragma unroll
        for (int s = 0; s < CIN / 16; ++s) {
          const f16x8 sbh = ldw(rsh, lofs, s * kstride);
          const f16x8 sbl = ldw(rsl, lofs, s * kstride);
          const float4 x0 = ld4(rx, sxo + 64u * s), x1 = ld4(rx, sxo + 64u * s + 16u);
          const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
          f16x8 xh, xl;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float v = xv[k] * ACT_SCALE;
            rbad |= !(fabsf(v) < SPLIT_MAX);
            xh[k] = (_Float16)v;
            xl[k] = (_Float16)(v - (float)xh[k]);
          }
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(sbl, xh, sacc, 0, 0, 0);
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(sbh, xl, sacc, 0, 0, 0);
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(sbh, xh, sacc, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 bs = *reinterpret_cast<const float4*>(spar + 4 * C + wn * 32 + 8 * q + h4);
          rsd[q] = make_float4(fmaf(sacc[4 * q], a.us, bs.x), fmaf(sacc[4 * q + 1], a.us, bs.y),
                               fmaf(sacc[4 * q + 2], a.us, bs.z), fmaf(sacc[4 * q + 3], a.us, bs.w));
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) rsd[q] = EARLY ? ersd[EARLY ? mt : 0][q] : ld4(rx, rsd_off(mt, q));
      }
      if (m < R && g < HH) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int co0 = wn * 32 + 8 * q + h4;
          const float4 b = *reinterpret_cast<const float4*>(spar + 3 * C + co0);
          float4 val = make_float4(fmaf(acc[mt][4 * q], a.ub, b.x), fmaf(acc[mt][4 * q + 1], a.ub, b.y),
                                   fmaf(acc[mt][4 * q + 2], a.ub, b.z), fmaf(acc[mt][4 * q + 3], a.ub, b.w));
          val.x += rsd[q].x;
          val.y += rsd[q].y;
          val.z += rsd[q].z;
          val.w += rsd[q].w;
          *reinterpret_cast<float4*>(a.y + (size_t)g * C + co0) = val;
        }
      }
    }
  } else {
    static_assert(!FIN || (!POOL && CIN == C), "the last unit keeps its width");
    gemm(std::integral_constant<int, NCH>{}, std::integral_constant<int, LDP>{}, std::false_type{}, a.wbh, a.wbl, r0,
         acc);
    const int co = wn * 32 + (lane & 31);
    const float b = spar[3 * C + co], fs = a.fs[co], ft = a.ft[co];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      // registers 4 q .. 4 q + 3 are the rows m0 .. m0 + 3, m0 = 8 q + h4 (+ tile): with r0, R and t
      // multiples of 4 each group is one pool window of one clip
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m0 = (wm * MT + mt) * 32 + 8 * q + h4;
        const int g0 = r0 + m0;
        float rs[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          rs[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                rx, (uint32_t)min(g0 + j, HH - 1) * (C * 4u) + co * 4u, 0, 0));
        if (m0 < R && g0 < HH) {
          float sum = 0.0f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float val = fmaf(acc[mt][4 * q + j], a.ub, b);
            val += rs[j];
            sum += fmaxf(fmaf(val, fs, ft), 0.0f);
          }
          a.seq[(size_t)(g0 >> 2) * C + co] = sum / 4.0f;
        }
      }
    }
  }
  if ((rbad || !(rmax < SPLIT_MAX)) && a.range_flag) *a.range_flag = 1;
}

// the chain kernel's first output row per workgroup (its halo in front) and output rows: U units
// narrow the correct rows by 2 U; FIN keeps both multiples of 4 (pool windows)
template <bool POOL, bool FIN>
constexpr int chain_front() { return POOL ? (FIN ? 8 : 6) : 4; }
template <int NR, bool POOL, bool FIN>
constexpr int chain_rows() { return FIN ? (NR - chain_front<POOL, FIN>() - (POOL ? 6 : 4)) / 4 * 4 : NR - (POOL ? 12 : 8); }

// A chain of res units as ONE kernel: two consecutive units without pooling (2-3, 5-6, 8-9), or with
// POOL the pool unit before them too (1-3, 4-6, 7-9).  Each unit's output stays in registers (the next
// unit's residual) and in LDS (BN + ReLU + split, the next unit's staged input), so only the chain's
// input and output touch HBM.  All GEMMs run over the same NR rows i <-> global (pooled) row rb + i;
// each conv narrows the rows it computes correctly by one at each end, so the last unit's output is
// right for i in [2 U, NR - 2 U), U = the chain's units: every GEMM's tile row i is the same lane,
// and the running residual of row i is where the next epilogue needs it.  Output rows per workgroup
// RO = [F, F + RO), F = 2 U (FIN: 8 with POOL, so that rb and RO are multiples of 4).  LDS row
// L = i + 1 (rows 0 and NR + 1 are zero pads, ZR the zero row of taps that leave a clip); one buffer,
// overwritten stage by stage.  FIN (unit 9 last): the AveragePooling1D(4) windows are 4 adjacent
// lanes, summed in the unfused kernel's order through DPP broadcasts.
// Bit-identical to one siu launch per unit: the same operands, MFMA sequences and epilogue arithmetic.
template <int CIN, int C, int NR, int NW, bool POOL, bool FIN, int MINW>
__global__ void __launch_bounds__(64 * NW, MINW) siu_chain_kernel(SiuArgs p, SiuArgs a, SiuArgs b) {
  constexpr int NT = 64 * NW;
  constexpr int WN = C / 32;
  constexpr int WM = NW / WN;
  constexpr int MT = NR / (WM * 32);
  constexpr int NCHX = CIN / CK, NCH = C / CK;
  constexpr int LDP = C + 8;
  constexpr int F = chain_front<POOL, FIN>(), RO = chain_rows<NR, POOL, FIN>();
  constexpr int ZR = NR + 2;
  constexpr int QPP = CK / 4;
  constexpr int MAXT = (NR * QPP + NT - 1) / NT;
  constexpr int P0 = POOL ? 2 : 0;     // rows the pool unit narrows
  static_assert(WM * WN == NW && MT * WM * 32 == NR && NT % QPP == 0, "tiling");
  static_assert(POOL || CIN == C, "units without pooling keep their width");
  static_assert(F + RO <= NR - (POOL ? 6 : 4) && (!FIN || (F % 4 == 0 && RO % 4 == 0)), "rows");
  __shared__ __attribute__((aligned(16))) _Float16 lhi[(NR + 3) * LDP];
  __shared__ __attribute__((aligned(16))) _Float16 llo[(NR + 3) * LDP];
  // per-channel parameters: unit a [0] b_a [1] 16 s_mid [2] 16 t_mid [3] b_b; unit b [4] 16 s_in
  // [5] 16 t_in [6] b_a [7] 16 s_mid [8] 16 t_mid [9] b_b; FIN [10] fs [11] ft; POOL: unit a [12]
  // 16 s_in [13] 16 t_in, the pool unit [14] b_a [15] 16 s_mid [16] 16 t_mid [17] b_b [18] b_s
  constexpr int NPAR = POOL ? 19 : 12;
  __shared__ __attribute__((aligned(16))) float spar[NPAR * C];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const SiuArgs& s0 = POOL ? p : a;                // the chain's first unit
  const int HH = a.n * a.t;
  const int rb = (int)blockIdx.x * RO - F;
  const int koff = (lane >> 5) * 8;
  const int h4 = 4 * (lane >> 5);
  const uint32_t tm = a.tdiv_m, ts = a.tdiv_s;
  float rmax = 0.0f;
  int rbad = 0;   // a raw shortcut operand out of range / NaN (an int, pinned per tile: see below)
  const __amdgpu_buffer_rsrc_t rx = siu_rsrc(s0.x);

  for (int e = tid; e < 3 * (LDP / 8); e += NT) {   // pad rows 0, NR + 1 and the zero row
    const int z = e / (LDP / 8), k8 = e - z * (LDP / 8);
    const int row = z == 0 ? 0 : z == 1 ? NR + 1 : ZR;
    *reinterpret_cast<f16x8*>(lhi + row * LDP + 8 * k8) = f16x8{};
    *reinterpret_cast<f16x8*>(llo + row * LDP + 8 * k8) = f16x8{};
  }
  for (int i = tid; i < C; i += NT) {
    spar[i] = a.ba[i];
    spar[C + i] = ACT_SCALE * a.s_mid[i];
    spar[2 * C + i] = ACT_SCALE * a.t_mid[i];
    spar[3 * C + i] = a.bb[i];
    spar[4 * C + i] = ACT_SCALE * b.s_in[i];
    spar[5 * C + i] = ACT_SCALE * b.t_in[i];
    spar[6 * C + i] = b.ba[i];
    spar[7 * C + i] = ACT_SCALE * b.s_mid[i];
    spar[8 * C + i] = ACT_SCALE * b.t_mid[i];
    spar[9 * C + i] = b.bb[i];
    if constexpr (FIN) {
      spar[10 * C + i] = b.fs[i];
      spar[11 * C + i] = b.ft[i];
    }
    if constexpr (POOL) {
      spar[12 * C + i] = ACT_SCALE * a.s_in[i];
      spar[13 * C + i] = ACT_SCALE * a.t_in[i];
      spar[14 * C + i] = p.ba[i];
      spar[15 * C + i] = ACT_SCALE * p.s_mid[i];
      spar[16 * C + i] = ACT_SCALE * p.t_mid[i];
      spar[17 * C + i] = p.bb[i];
      spar[18 * C + i] = p.bs[i];
    }
  }

  // ---- stage the chain's input rows i < NR (clamped to the batch: see siu_kernel; POOL: row g =
  //      (clip, tt) is the max of the clip's unpooled rows 2 tt, 2 tt + 1) into LDS rows 1 .. NR ------
  {
    const int q = tid % QPP;
#pragma unroll 1
    for (int ch = 0; ch < NCHX; ++ch) {
      const int ci = ch * CK + 4 * q;
      float4 sc = *reinterpret_cast<const float4*>(s0.s_in + ci);
      float4 sh = *reinterpret_cast<const float4*>(s0.t_in + ci);
      sc = make_float4(ACT_SCALE * sc.x, ACT_SCALE * sc.y, ACT_SCALE * sc.z, ACT_SCALE * sc.w);
      sh = make_float4(ACT_SCALE * sh.x, ACT_SCALE * sh.y, ACT_SCALE * sh.z, ACT_SCALE * sh.w);
      float4 pre[MAXT];
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        const int task = tid + j * NT;
        const int g = min(max(rb + task / QPP, 0), HH - 1);
        if constexpr (POOL) {
          const uint32_t cl = tdiv((uint32_t)g, tm, ts);
          const int tt = g - (int)cl * a.t;
          const uint32_t src = ((uint32_t)cl * (uint32_t)p.t_src + 2u * tt) * (CIN * 4u) + ci * 4u;
          const float4 v = ld4(rx, src);
          const float4 u = ld4(rx, 2 * tt + 1 < p.t_src ? src + CIN * 4u : src);
          pre[j] = make_float4(fmaxf(v.x, u.x), fmaxf(v.y, u.y), fmaxf(v.z, u.z), fmaxf(v.w, u.w));
        } else {
          pre[j] = ld4(rx, (uint32_t)g * (C * 4u) + ci * 4u);
        }
      }
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        const int task = tid + j * NT;
        if (MAXT * NT > NR * QPP && task >= NR * QPP) continue;
        f16x4 hv, lv;
        bn_split4(pre[j], sc, sh, hv, lv, rmax);
        const int row = task / QPP + 1;
        *reinterpret_cast<f16x4*>(lhi + row * LDP + ci) = hv;
        *reinterpret_cast<f16x4*>(llo + row * LDP + ci) = lv;
      }
    }
  }

  constexpr int kstride = (C / 32) * 512;
  const int lofs = wn * 512 + lane * 8;
  int mrow[MT], trow[MT], grow[MT];   // per tile: this lane's row i, its position in its clip, rb + i
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    mrow[mt] = (wm * MT + mt) * 32 + (lane & 31);
    grow[mt] = rb + mrow[mt];
    const uint32_t gp = (uint32_t)(grow[mt] + a.t);
    trow[mt] = (int)(gp - tdiv(gp, tm, ts) * (uint32_t)a.t);
  }
  // acc = W^T X^T over LDS rows, NCHK 32-channel chunks (row i's taps: LDS rows i .. i + 2, or the
  // zero row)
  auto gemm = [&](auto nchk_c, const uint16_t* wh, const uint16_t* wl, f32x16 (&acc)[MT]) {
    constexpr int NCHK = decltype(nchk_c)::value;
    constexpr int tap_stride = C * NCHK * CK;
    const __amdgpu_buffer_rsrc_t rwh = siu_rsrc(wh), rwl = siu_rsrc(wl);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[mt][i] = 0.0f;
#pragma unroll 1
    for (int ch = 0; ch < NCHK; ++ch) {
#pragma unroll 1
      for (int tap = 0; tap < TAPS; ++tap) {
        f16x8 bh[KS], bl[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const int u = tap * tap_stride + (ch * KS + s) * kstride;
          bh[s] = ldw(rwh, lofs, u);
          bl[s] = ldw(rwl, lofs, u);
        }
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const int src = trow[mt] + tap - 1;
            const int off = (src < 0 || src >= a.t ? ZR : mrow[mt] + tap) * LDP + ch * CK + 16 * s + koff;
            const f16x8 ah = *reinterpret_cast<const f16x8*>(lhi + off);
            const f16x8 al = *reinterpret_cast<const f16x8*>(llo + off);
            acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bl[s], ah, acc[mt], 0, 0, 0);
            acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[s], al, acc[mt], 0, 0, 0);
            acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[s], ah, acc[mt], 0, 0, 0);
          }
      }
    }
  };
  // LDS row i + 1 = split(max(fma(v, s16, t16), 0)) of each tile's row; rows outside [lo, NR - lo)
  // or the batch stay out of the range guard
  auto put = [&](const float (&v)[MT][16], int ps, int pt, int lo) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int L = mrow[mt] + 1;
      float tmax = 0.0f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co0 = wn * 32 + 8 * q + h4;
        const float4 s = *reinterpret_cast<const float4*>(spar + ps * C + co0);
        const float4 t = *reinterpret_cast<const float4*>(spar + pt * C + co0);
        f16x4 hv, lv;
        bn_split4(make_float4(v[mt][4 * q], v[mt][4 * q + 1], v[mt][4 * q + 2], v[mt][4 * q + 3]), s, t, hv, lv,
                  tmax);
        *reinterpret_cast<f16x4*>(lhi + L * LDP + co0) = hv;
        *reinterpret_cast<f16x4*>(llo + L * LDP + co0) = lv;
      }
      if (mrow[mt] >= lo && mrow[mt] < NR - lo && grow[mt] >= 0 && grow[mt] < HH) rmax = fmaxf(rmax, tmax);
    }
  };
  // v = fma(acc, u, bias[pb])
  auto unscale = [&](const f32x16 (&acc)[MT], float u, int pb, float (&v)[MT][16]) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 bq = *reinterpret_cast<const float4*>(spar + pb * C + wn * 32 + 8 * q + h4);
        v[mt][4 * q] = fmaf(acc[mt][4 * q], u, bq.x);
        v[mt][4 * q + 1] = fmaf(acc[mt][4 * q + 1], u, bq.y);
        v[mt][4 * q + 2] = fmaf(acc[mt][4 * q + 2], u, bq.z);
        v[mt][4 * q + 3] = fmaf(acc[mt][4 * q + 3], u, bq.w);
      }
  };

  // y = fma(acc, u, bias[pb]) + y (the unit's epilogue: conv + residual, in that order)
  auto unscale_add = [&](const f32x16 (&acc)[MT], float u, int pb, float (&y)[MT][16]) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 bq = *reinterpret_cast<const float4*>(spar + pb * C + wn * 32 + 8 * q + h4);
        y[mt][4 * q] = fmaf(acc[mt][4 * q], u, bq.x) + y[mt][4 * q];
        y[mt][4 * q + 1] = fmaf(acc[mt][4 * q + 1], u, bq.y) + y[mt][4 * q + 1];
        y[mt][4 * q + 2] = fmaf(acc[mt][4 * q + 2], u, bq.z) + y[mt][4 * q + 2];
        y[mt][4 * q + 3] = fmaf(acc[mt][4 * q + 3], u, bq.w) + y[mt][4 * q + 3];
      }
  };

  f32x16 acc[MT];
  float v[MT][16];
  float y[MT][16];   // the running residual: each unit's output
  __syncthreads();
  if constexpr (POOL) {
    // the pool unit: t1, then y1 = conv_b + the shortcut Conv1D(1, stride 2) of the raw x (siu_kernel's
    // arithmetic; the shortcut first, into y, while GEMM a's accumulators are dead)
    gemm(std::integral_constant<int, NCHX>{}, p.wah, p.wal, acc);
    __syncthreads();
    unscale(acc, p.ua, 14, v);
    put(v, 15, 16, 1);
    const __amdgpu_buffer_rsrc_t rsh = siu_rsrc(p.wsh), rsl = siu_rsrc(p.wsl);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      f32x16 sacc;
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[i] = 0.0f;
      const int gs = min(max(grow[mt], 0), HH - 1);
      const uint32_t cl = tdiv((uint32_t)gs, tm, ts);
      const int tt = gs - (int)cl * a.t;
      const uint32_t sxo = ((uint32_t)cl * (uint32_t)p.t_src + 2u * tt) * (CIN * 4u) + koff * 4u;
#pragma unroll
      for (int s = 0; s < CIN / 16; ++s) {
        const f16x8 sbh = ldw(rsh, lofs, s * kstride);
        const f16x8 sbl = ldw(rsl, lofs, s * kstride);
        const float4 x0 = ld4(rx, sxo + 64u * s), x1 = ld4(rx, sxo + 64u * s + 16u);
        const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        f16x8 xh, xl;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float w = xv[k] * ACT_SCALE;
          rbad |= !(fabsf(w) < SPLIT_MAX) ? 1 : 0;
          xh[k] = (_Float16)w;
          xl[k] = (_Float16)(w - (float)xh[k]);
        }
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(sbl, xh, sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(sbh, xl, sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(sbh, xh, sacc, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 bs = *reinterpret_cast<const float4*>(spar + 18 * C + wn * 32 + 8 * q + h4);
        y[mt][4 * q] = fmaf(sacc[4 * q], p.us, bs.x);
        y[mt][4 * q + 1] = fmaf(sacc[4 * q + 1], p.us, bs.y);
        y[mt][4 * q + 2] = fmaf(sacc[4 * q + 2], p.us, bs.z);
        y[mt][4 * q + 3] = fmaf(sacc[4 * q + 3], p.us, bs.w);
      }
      // evaluate this tile's range tests here: left to the compiler, they sink to the kernel's end
      // and keep every scaled shortcut operand alive across the chain (hundreds of spilled VGPRs)
      asm volatile("" : "+v"(rbad));
      __builtin_amdgcn_sched_barrier(0);   // one tile's shortcut operands live at a time
    }
    __syncthreads();
    gemm(std::integral_constant<int, NCH>{}, p.wbh, p.wbl, acc);
    unscale_add(acc, p.ub, 17, y);
    __syncthreads();   // every wave has read t1
    put(y, 12, 13, 2);
    __syncthreads();
  } else {
    // the raw x of each tile row: the first unit's residual, loaded under its GEMMs
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int g = min(max(grow[mt], 0), HH - 1);
        const float4 r = ld4(rx, (uint32_t)g * (C * 4u) + (wn * 32 + 8 * q + h4) * 4u);
        y[mt][4 * q] = r.x;
        y[mt][4 * q + 1] = r.y;
        y[mt][4 * q + 2] = r.z;
        y[mt][4 * q + 3] = r.w;
      }
  }
  // unit a
  gemm(std::integral_constant<int, NCH>{}, a.wah, a.wal, acc);
  __syncthreads();
  unscale(acc, a.ua, 0, v);
  put(v, 1, 2, P0 + 1);
  __syncthreads();
  gemm(std::integral_constant<int, NCH>{}, a.wbh, a.wbl, acc);
  unscale_add(acc, a.ub, 3, y);
  __syncthreads();   // every wave has read t1
  // unit b
  put(y, 4, 5, P0 + 2);
  __syncthreads();
  gemm(std::integral_constant<int, NCH>{}, b.wah, b.wal, acc);
  __syncthreads();
  unscale(acc, b.ua, 6, v);
  put(v, 7, 8, P0 + 3);
  __syncthreads();
  gemm(std::integral_constant<int, NCH>{}, b.wbh, b.wbl, acc);
  unscale_add(acc, b.ub, 9, y);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int i = mrow[mt], g = grow[mt];
    const bool ok = i >= F && i < F + RO && g < HH;
    if constexpr (!FIN) {
      if (ok) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 val = make_float4(y[mt][4 * q], y[mt][4 * q + 1], y[mt][4 * q + 2], y[mt][4 * q + 3]);
          *reinterpret_cast<float4*>(b.y + (size_t)g * C + wn * 32 + 8 * q + h4) = val;
        }
      }
    } else {
      // BN + ReLU of each row, then the 4-row window sum in the unfused order ((r0 + r1) + r2) + r3:
      // lanes 4k .. 4k + 3 hold rows rb + i, i = 0 .. 3 mod 4
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co0 = wn * 32 + 8 * q + h4;
        const float4 fs = *reinterpret_cast<const float4*>(spar + 10 * C + co0);
        const float4 ft = *reinterpret_cast<const float4*>(spar + 11 * C + co0);
        const float fsv[4] = {fs.x, fs.y, fs.z, fs.w}, ftv[4] = {ft.x, ft.y, ft.z, ft.w};
        float out[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = __builtin_bit_cast(int, fmaxf(fmaf(y[mt][4 * q + e], fsv[e], ftv[e]), 0.0f));
          const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(r, 0x00, 0xf, 0xf, false));
          const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(r, 0x55, 0xf, 0xf, false));
          const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(r, 0xaa, 0xf, 0xf, false));
          const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(r, 0xff, 0xf, 0xf, false));
          out[e] = (((r0 + r1) + r2) + r3) / 4.0f;
        }
        if (ok && (i & 3) == 0)
          *reinterpret_cast<float4*>(b.seq + (size_t)(g >> 2) * C + co0) = make_float4(out[0], out[1], out[2], out[3]);
      }
    }
  }
  if ((rbad || !(rmax < SPLIT_MAX)) && a.range_flag) *a.range_flag = 1;
}

// q = x / d for x < 2^31 as (umulhi(x, m) + x) >> s: s = ceil(log2 d), m = floor(2^(32+s) / d) + 1 - 2^32
void siu_fastdiv(uint32_t d, uint32_t& m, uint32_t& s) {
  s = 0;
  while ((1u << s) < d) ++s;
  m = (uint32_t)(((uint64_t)1 << (32 + s)) / d + 1 - ((uint64_t)1 << 32));
}

template <int CIN, int C, int ROWS, int NW, bool POOL = false, bool FIN = false, int MINW = 2>
hipError_t launch(const SiuArgs& a0, hipStream_t s) {
  constexpr int R = FIN ? (ROWS - 2) / 4 * 4 : ROWS - 2;
  SiuArgs a = a0;
  siu_fastdiv((uint32_t)a.t, a.tdiv_m, a.tdiv_s);
  const int64_t rows = (int64_t)a.n * a.t;
  // 32-bit row indices and byte offsets: x (pool units: [n t_src, CIN]) and y below 4 GiB
  const int64_t xbytes = (int64_t)a.n * (POOL ? a.t_src : a.t) * CIN * 4;
  if (rows >= (1 << 24) || xbytes > 0xffffff00ll || rows * C * 4 > 0xffffff00ll) return hipErrorInvalidValue;
  const int64_t blocks = (rows + R - 1) / R;
  hipLaunchKernelGGL((siu_kernel<CIN, C, ROWS, NW, POOL, FIN, MINW>), dim3((unsigned)blocks), dim3(64 * NW), 0, s, a);
  return hipGetLastError();
}

template <int CIN, int C, int NR, int NW, bool POOL, bool FIN, int MINW>
hipError_t launch_chain(const SiuArgs& p, const SiuArgs& a0, const SiuArgs& b, hipStream_t s) {
  constexpr int RO = chain_rows<NR, POOL, FIN>();
  SiuArgs a = a0;
  siu_fastdiv((uint32_t)a.t, a.tdiv_m, a.tdiv_s);
  const int64_t rows = (int64_t)a.n * a.t;
  const int64_t xbytes = (int64_t)a.n * (POOL ? p.t_src : a.t) * CIN * 4;
  if (rows >= (1 << 24) || xbytes > 0xffffff00ll || rows * C * 4 > 0xffffff00ll) return hipErrorInvalidValue;
  const int64_t blocks = (rows + RO - 1) / RO;
  hipLaunchKernelGGL((siu_chain_kernel<CIN, C, NR, NW, POOL, FIN, MINW>), dim3((unsigned)blocks), dim3(64 * NW), 0,
                     s, p, a, b);
  return hipGetLastError();
}

}  // namespace

bool siu_pair_supported(int c) { return c == 32 || c == 64 || c == 128; }

hipError_t siu_pair_launch(const SiuArgs& a, const SiuArgs& b, int c, hipStream_t s) {
  if ((int64_t)a.n * a.t == 0) return hipSuccess;
  if (!a.x || a.n != b.n || a.t != b.t || a.t < 1) return hipErrorInvalidValue;
  if (b.seq) {   // units 8-9 with the final BN + ReLU + AveragePooling1D(4)
    if (!b.fs || !b.ft || a.t % 4 != 0 || c != 128) return hipErrorInvalidValue;
    return launch_chain<128, 128, 128, 4, false, true, 2>(a, a, b, s);
  }
  if (!b.y || b.y == a.x) return hipErrorInvalidValue;
  if (c == 32) return launch_chain<32, 32, 256, 4, false, false, 3>(a, a, b, s);
  if (c == 64) return launch_chain<64, 64, 256, 4, false, false, 2>(a, a, b, s);
  if (c == 128) return launch_chain<128, 128, 128, 4, false, false, 2>(a, a, b, s);
  return hipErrorInvalidValue;
}

bool siu_triple_supported(int cin, int c) { return sipu_supported(cin, c); }

hipError_t siu_triple_launch(const SiuArgs& p, const SiuArgs& a, const SiuArgs& b, int cin, int c,
                             hipStream_t s) {
  if ((int64_t)a.n * a.t == 0) return hipSuccess;
  if (!p.x || !p.wsh || !p.wsl || !p.bs || p.n != a.n || a.n != b.n || p.t != a.t || a.t != b.t || a.t < 1 ||
      a.t != (p.t_src + 1) / 2)
    return hipErrorInvalidValue;
  if (b.seq) {
    if (!b.fs || !b.ft || a.t % 4 != 0 || cin != 64 || c != 128) return hipErrorInvalidValue;
    return launch_chain<64, 128, 128, 4, true, true, 2>(p, a, b, s);
  }
  if (!b.y || b.y == p.x) return hipErrorInvalidValue;
  if (cin == 32 && c == 32) return launch_chain<32, 32, 256, 4, true, false, 3>(p, a, b, s);
  if (cin == 32 && c == 64) return launch_chain<32, 64, 256, 4, true, false, 2>(p, a, b, s);
  if (cin == 64 && c == 128) return launch_chain<64, 128, 128, 4, true, false, 2>(p, a, b, s);
  return hipErrorInvalidValue;
}

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
  // Tiles (4 waves): C = 32 256 t1 rows (MT 2, 3 workgroups per CU); C = 64 256 rows and C = 128
  // 128 rows (MT 4, 2 per CU).  Measured per unit and SI step against the conv_h3 pair (round 4):
  // C = 32 1.004 vs 1.033 ms, C = 64 (128-row tiles) 1.061 vs 1.203 ms, C = 128 with 64-row tiles
  // 1.672 vs 1.625 ms (B streamed per 62 output rows).  Tried: 8-wave workgroups (one per CU) and
  // 512-row C = 32 tiles (occupancy 1): slower
  if (c == 32) return launch<32, 32, 256, 4>(a, s);
  if (c == 64) return launch<64, 64, 256, 4>(a, s);
  if (c == 128) return launch<128, 128, 128, 4>(a, s);
  return hipErrorInvalidValue;
}
