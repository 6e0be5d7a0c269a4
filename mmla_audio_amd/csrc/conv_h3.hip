// Halo-tiled implicit-GEMM convolution on gfx950 f16 MFMA with error-compensated 3xFP16 products.
//
// Each float32 operand is first scaled by an exact power of two (activations x 2^4 while staging,
// weights x 2^8 on the host) and split into v' = hi + lo with hi = fp16(v'), lo = fp16(v' - hi)
// (|error| <= 2^-22 |v'|, or the fp16 subnormal step 2^-25 once |v'| < 2^-3).  A product is
// accumulated in ONE f32 accumulator per tile:
//     acc += hi(a) hi(w) + hi(a) lo(w) + lo(a) hi(w)      (three v_mfma_f32_32x32x16_f16)
//     y    = acc * 2^-12                                   (dropped term lo*lo <= 2^-22 |a w|)
// i.e. ~22-bit products with float32 accumulation -- float32-class accuracy (the reference's Keras
// layers run float32) at 16/3 = 5.3x the f32-MFMA rate.  The scales keep the lo halves out of the
// subnormals for all but tiny operands (whose absolute error, <= 2^-29 for activations and 2^-33
// for weights, is far below the f32 rounding of the sums they join) and cost fp16 range: staged
// activations must stay below 65504 / 2^4 = 4094 (range guard) and weights below 255.
// One accumulator instead of separate hi*hi / correction accumulators halves the accumulator
// registers (the occupancy limiter of the 32x32 tiles).  Layer-wise parity vs the float64 oracle:
// tests/test_gpu_parity.py::test_od_layerwise_trace / test_precision_modes_vs_oracle.
//
// One workgroup (256 threads = 4 waves) computes a TH x TW = 128-pixel output tile of one clip for
// BN output channels; TW is a compile-time 16 (wide images), 8 (narrow) or 1 (the SI Conv1D), so
// every pixel <-> (row, col) map is a shift.  Per chunk of CK input channels the
// (TH+KH-1) x (TW+KW-1) input halo is staged ONCE into LDS -- BatchNorm + ELU/ReLU prologue applied
// once per input element (not once per tap), split into fp16 hi/lo -- and all KH*KW taps read their
// A fragments from it (ds_read_b128, pixel rows padded by 16 B).  B fragments (pre-split weights
// [tap][cout][cin]: a lane's 8 k-values are one 16-B load) come from L2, next tap prefetched under
// the current tap's MFMAs.  Waves split the tile 4 x 1 / 2 x 2 / 1 x 4 (BN = 32 / 64 / 128): every
// wave owns its own 32 output channels, so no B fragment is fetched twice per workgroup.
// Epilogue: bias, optional in-place residual, or (pool blocks) MaxPool2D(2,'same') written at half
// resolution: the 2x2 window is rows r, r+1, r+TW, r+TW+1 of one lane's 32-row accumulator tile,
// so no data leaves the registers.
#include "common.h"
#include "conv.h"
#include "conv_h3.h"

#include <cstring>


namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 256;
constexpr int BM = 128;
constexpr float ACT_SCALE = 16.0f;      // 2^4: staged activations
// weights are split at a per-tensor power-of-two scale (conv_h3_split_weights, capi.cpp pick_wscale:
// 2^8 for the usual |w| in [1/16, 255.9)); the epilogue multiplies by a.unscale = 2^-4 / that scale
constexpr float ACT_RANGE = 65504.0f / ACT_SCALE;   // largest finite fp16 / the activation scale
// The B fragments by raw buffer loads from a wave-uniform descriptor (voffset = the
// lane's 32-bit offset, soffset = the uniform (tap, k-step) offset): no per-load 64-bit address VALU
MMLA_DEV __amdgpu_buffer_rsrc_t h3_rsrc(const void* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)0x7fffffff, 0x00020000);
}
// 16 B of a split weight at half index uoff (wave-uniform) + lofs (this lane's)
MMLA_DEV f16x8 h3_frag(const uint16_t* base, __amdgpu_buffer_rsrc_t r, size_t uoff, int lofs) {
  (void)base;
  return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)lofs * 2u,
                                                                         (int)(uoff * 2), 0));
}


template <int PRO>
MMLA_DEV float pro_fn(float v, float sc, float sh) {
  if constexpr (PRO == PRO_NONE) {
    return v;
  } else {
    v = fmaf(v, sc, sh);
    // Keras/TF Elu: exp(x) - 1 for x < 0 (Eigen: (x < 0).select(x.exp() - 1, x)), as elu16 (exact
    // power-of-two scalings) so odu / rbs reproduce these operands bit for bit
    if constexpr (PRO == PRO_BN_ELU) return elu16(16.0f * v) * 0.0625f;
    return fmaxf(v, 0.0f);
  }
}

// Pixels per tile.  BN 64 tiles of 256 pixels stage B once per 256 pixels and cut the halo share
// (measured: <3,3,64,8> 1.88 -> 1.51 ms, <4,1,64,16,pool> 4.01 -> 3.62, <4,1,64,8,res> 1.27 -> 1.20)
// at occupancy 2; the 3x3 TW 16 variant is slower with them (3.31 -> 3.54) and keeps 128.  BN 128
// halved to 64 pixels (occupancy 4) was 25-33 % slower: per-tile costs dominate, not latency.
template <int KH, int BN, int TW>
// the SI Conv1D layers with BN <= 64 (K = 3 x 32 or 3 x 64: little work per row) take 256-row tiles:
// the per-tile fixed costs (B fragments, bias, setup) over twice the rows -- SI conv 41.05 -> 40.51 ms
// per 3 steps, outputs bit-identical (A/B, round 4)
constexpr int tile_px() {
  return BN == 64 && TW > 1 && !(KH == 3 && TW == 16) ? 256 : (TW == 1 && BN <= 64 ? 256 : BM);
}

// TW == 0 (LIN): a tile is 128 consecutive pixels of the whole batch in NHWC order (rows of all
// clips back to back), so the 19-wide images do not pad 19 -> 24 columns.  The rows the tile touches
// plus the halo rows are staged with a padded pitch of w + kw - 1 pixels (<= LIN_WP) into at most
// LIN_SLOTS row slots; a tap whose source row lies outside the output pixel's clip reads row slot
// LIN_SLOTS, which stays zero.
constexpr int LIN_SLOTS = 11, LIN_WP = 21;

// kernel-internal epilogue: EPI_ADD whose residual is the pool unit's shortcut Conv1D(1, stride 2),
// computed in the epilogue (ConvH3Args::sc_x); its own instantiation, with the 2-wave register
// budget (inside the 3-wave one of the plain residual tiles it spilled)
constexpr int EPI_ADD_SC = 3;

// register estimate (accumulators + staged halo + one tap of B) up to which tap 0's B fragments are
// loaded before the staging instead of after its barrier (above it the variants spilled)
constexpr int EARLY_B_VGPRS = 168;

// V4: channels loaded as float4 (cin % 4 == 0); else per element (the SI stem, cin = 39).
// PIN (Conv1D): the input rows are MaxPool1D(2, 'same') of x, taken while staging (SI pool units)
// Shape: the layer geometry, compile-time for the fixed OD-NET / SI-NET layers (every bound,
// division and address offset folds) or read from the arguments (Shape<0, 0, 0, 0>)
template <int SH, int SW, int SCI, int SCO>
struct Shape {
  static constexpr bool FIXED = SH > 0;
};

template <class S> struct ShapeOf;
template <int SH, int SW, int SCI, int SCO>
struct ShapeOf<Shape<SH, SW, SCI, SCO>> {
  static constexpr int h = SH, w = SW, ci = SCI, co = SCO;
};
template <class S> MMLA_DEV constexpr int shp_h() { return ShapeOf<S>::h; }
template <class S> MMLA_DEV constexpr int shp_w() { return ShapeOf<S>::w; }
template <class S> MMLA_DEV constexpr int shp_ci() { return ShapeOf<S>::ci; }
template <class S> MMLA_DEV constexpr int shp_co() { return ShapeOf<S>::co; }

// Waves per SIMD the register budget is sized for: 3 (<= 168 VGPRs) for the SI Conv1D BN 128 tiles
// (the residual variant needed 169 and ran at 2; now 168 + 2 spilled dwords) and for the fixed-shape
// 64-channel residual conv(4,1) of OD blocks 5-6 (172 -> 166 VGPRs, 44.8 KB LDS: 3 workgroups per
// CU); conv -0.4 % (OD) / -0.5 % (SI) per step in an A/B.  2 elsewhere: forced to 3, the block-4
// conv(4,1) + pool and the 19-wide BN 128 layers spill 64-152 B per lane.
template <int KH, int BN, int TW, int EPI, bool FIXED>
constexpr int conv_minw() {
  return EPI == EPI_ADD_SC                                            ? 2
         : TW == 1 && BN == 128                                       ? 3
         : (FIXED && KH == 4 && BN == 64 && TW == 8 && EPI == EPI_ADD) ? 3
                                                                     : 2;
}

template <int KH, int KW, int CK, int BN, int TW, int PRO, int EPI, bool POOL, bool V4 = true,
          bool PIN = false, class SHP = Shape<0, 0, 0, 0>>
__global__ void __launch_bounds__(NT, (conv_minw<KH, BN, TW, EPI, SHP::FIXED>())) conv_h3_kernel(ConvH3Args a) {
  constexpr bool ADD = EPI == EPI_ADD || EPI == EPI_ADD_SC;   // the output adds a residual
  constexpr bool SCR = EPI == EPI_ADD_SC;                     // ... the fused shortcut's
  // each wave owns ONE 32-column slice of B (no B fragment is loaded by two waves) and
  // 128 / WM rows: BN 32 -> 4 x 1, BN 64 -> 2 x 2, BN 128 -> 1 x 4 (waves along N)
  constexpr int WN = BN / 32;
  constexpr int WM = 4 / WN;
  constexpr int BMK = tile_px<KH, BN, TW>();
  constexpr int MT = BMK / (WM * 32);     // 32-row tiles per wave
  constexpr int NTL = BN / (WN * 32);     // 32-col tiles per wave
  constexpr int LDP = CK + 8;             // fp16 per staged pixel (16-B pad)
  constexpr int KS = CK / 16;             // MFMA k-steps per chunk
  constexpr int TAPS = KH * KW;
  constexpr bool LIN = TW == 0;
  constexpr int TH = LIN ? 0 : BMK / (LIN ? 1 : TW);
  constexpr int WP = LIN ? LIN_WP : TW + KW - 1;
  constexpr int HP = LIN ? LIN_SLOTS + 1 : TH + KH - 1;   // LIN: + the zero row
  constexpr int NPIX = HP * WP;
  constexpr int NSTG = LIN ? LIN_SLOTS * LIN_WP : NPIX;   // staged pixels (upper bound)
  constexpr int QPP = CK / 4;             // float4 per staged pixel
  constexpr int MAXT = (NSTG * QPP + NT - 1) / NT;     // staged float4 per thread and chunk
  // registers allow the early loads (tap 0's B, prologue and epilogue parameters): EARLY_B_VGPRS
  constexpr bool EARLY_B = MT * NTL * 16 + MAXT * 4 + NTL * KS * 8 <= EARLY_B_VGPRS;
  // CIL (channels in lane): the MFMA computes the transposed tile, so a lane holds 4 consecutive
  // output channels of one pixel per register quad and the epilogue reads residuals and writes
  // outputs as 16-B vectors (4x fewer memory instructions than one dword per (pixel, channel), but
  // each instruction touches 32 pixels' 32-B pieces instead of two 128-B rows).  Measured per
  // variant (rocprof A/B): only the 8-wide residual conv(4,1) gains (blocks 5-6: 4.43 -> 4.13 ms);
  // the 3x3 and linear-pixel variants lose 2.5-6.6 % and the SI Conv1D stack 5 %.  The pooled
  // epilogue needs the pixel-row layout (its 2x2 windows inside one lane's registers).
  constexpr bool CIL = !POOL && ADD && TW == 8;
  // Conv1D (TW == 1): one more staged row that stays zero -- a tap whose source row leaves the output
  // row's clip reads it (one select of the row offset per tap and row tile, instead of zeroing the
  // 2 x 8 halves of every A fragment read)
  constexpr int ZROW = TW == 1 && KH > 1 ? 1 : 0;
  __shared__ __attribute__((aligned(16))) _Float16 lds_hi[(NPIX + ZROW) * LDP];
  __shared__ __attribute__((aligned(16))) _Float16 lds_lo[(NPIX + ZROW) * LDP];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if constexpr (ZROW) {   // read only after the first chunk's staging barrier
    static_assert(LDP % 8 == 0 && LDP / 8 <= NT, "zero row");
    if (tid < LDP / 8) {
      *reinterpret_cast<f16x8*>(lds_hi + NPIX * LDP + 8 * tid) = f16x8{};
      *reinterpret_cast<f16x8*>(lds_lo + NPIX * LDP + 8 * tid) = f16x8{};
    }
  }
  // layer geometry (compile-time when SHP is a fixed shape: cin, cout are then their padded sizes)
  constexpr bool FX = SHP::FIXED;
  const int A_H = FX ? shp_h<SHP>() : a.h, A_W = FX ? shp_w<SHP>() : a.w;
  const int A_CIN = FX ? shp_ci<SHP>() : a.cin, A_COUT = FX ? shp_co<SHP>() : a.cout;
  const int A_CINP = FX ? shp_ci<SHP>() : a.cin_pad, A_COUTP = FX ? shp_co<SHP>() : a.cout_pad;
  const int A_PH = FX ? (KH - 1) / 2 : a.pad_h, A_PW = FX ? (KW - 1) / 2 : a.pad_w;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  // TW == 1 (Conv1D): the clips' rows form ONE sequence of n * h rows tiled 128 at a time, so a
  // short sequence (t = 64, 32) does not pad a tile; taps that cross a clip boundary read zeros
  const int HH = TW <= 1 ? a.n * A_H : A_H;
  // tiles per clip (TW > 1) / in total (LIN, Conv1D: tiles_w = 1)
  const int TLW = TW <= 1 ? 1 : (FX ? (A_W + TW - 1) / (TW > 1 ? TW : 1) : a.tiles_w);
  const int TLH = FX && TW > 1 ? (A_H + TH - 1) / (TH > 0 ? TH : 1) : a.tiles_h;
  const int tiles = TLH * TLW;
  const int64_t clip = TW <= 1 ? 0 : blockIdx.x / tiles;
  const int tile = blockIdx.x - (int)(clip * tiles);
  const int th_i = tile / TLW;
  const int h0 = th_i * TH;
  const int w0 = (tile - th_i * TLW) * TW;
  const int n0 = blockIdx.y * BN;

  int apix[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = (wm * MT + mt) * 32 + (lane & 31);
    apix[mt] = LIN ? 0 : ((m / (LIN ? 1 : TW)) * WP + (m % (LIN ? 1 : TW))) * LDP;
  }
  int trow[MT];   // TW == 1: the A row's position inside its clip
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) trow[mt] = TW == 1 ? (h0 + (wm * MT + mt) * 32 + (lane & 31)) % A_H : 0;
  // LIN: p0 = first pixel of the tile (flattened over n * h * w), r0 = its row; per A row and
  // kernel row dy the LDS pixel of tap (dy, 0), or the zero row when the source row leaves the clip
  const int wpad = A_W + KW - 1;
  const int64_t npx = (int64_t)a.n * A_H * A_W;
  const int64_t p0 = LIN ? (int64_t)tile * BMK : 0;
  const int r0 = LIN ? (int)(p0 / A_W) : 0;
  int abase[MT][LIN ? KH : 1];
  if constexpr (LIN) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int64_t P = p0 + (wm * MT + mt) * 32 + (lane & 31);
      const int r = (int)(P / A_W), c = (int)(P - (int64_t)r * A_W), cr = r % A_H;
#pragma unroll
      for (int dy = 0; dy < KH; ++dy) {
        const int sr = cr + dy - A_PH;
        abase[mt][dy] = ((sr >= 0 && sr < A_H ? (r - r0 + dy) * wpad : LIN_SLOTS * wpad) + c) * LDP;
      }
    }
    // the zero row (never staged)
    for (int i = tid; i < LIN_WP * QPP; i += NT) {
      *reinterpret_cast<f16x4*>(lds_hi + (LIN_SLOTS * wpad + i / QPP) * LDP + (i % QPP) * 4) = f16x4{};
      *reinterpret_cast<f16x4*>(lds_lo + (LIN_SLOTS * wpad + i / QPP) * LDP + (i % QPP) * 4) = f16x4{};
    }
  }
  const int koff = (lane >> 5) * 8;

  f32x16 acc[MT][NTL];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[mt][nt][i] = 0.0f;

  // B in MFMA fragment order (conv_h3_split_weights): per tap, 16-channel k-step and 32-channel
  // output tile the 64 lanes' 16-B fragments are 1 KB contiguous, so one load instruction covers 8
  // whole 128-B lines (the [co][ci] rows had put a wave's 64 lanes on 32 lines, 32 B used of each)
  // (address = wave-uniform base + a 32-bit lane offset, so the loads take the scalar-base form)
  int lofs[NTL];
#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) lofs[nt] = (n0 / 32 + wn * NTL + nt) * 512 + lane * 8;
  const __amdgpu_buffer_rsrc_t rwh = h3_rsrc(a.wh), rwl = h3_rsrc(a.wl);
  const size_t tap_stride = (size_t)A_COUTP * A_CINP;
  const size_t kstride = (size_t)(A_COUTP / 32) * 512;   // one 16-channel k-step
  // the epilogue's bias, loaded now: after the MFMA loop it cost a memory round trip of its own
  float bias_r[NTL];
#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) {
    const int co = n0 + (wn * NTL + nt) * 32 + (lane & 31);
    if (EARLY_B && !CIL) bias_r[nt] = co < A_COUT ? a.bias[co] : 0.0f;
  }
  const float* xclip = a.x + clip * HH * A_W * A_CIN;

  bool rbad = false;   // 3xFP16 range guard: a staged operand left the fp16 range
  const int nchunks = A_CINP / CK;
  for (int ch = 0; ch < nchunks; ++ch) {
    const int ci0 = ch * CK;
    __syncthreads();   // every wave is done reading the previous chunk's halo
    // ---- stage the input halo of this channel chunk: prologue once per element, split hi/lo ----
    // all of this thread's halo loads are issued before the first is consumed (one HBM latency
    // per chunk, not one per element group)
    const int nstg = LIN ? LIN_SLOTS * wpad : NPIX;
    // this thread's channel quad is the same for every task (NT % QPP == 0): its prologue scale /
    // shift are loaded once, ahead of the halo, instead of once per task behind it
    // (the register-tight variants, !EARLY_B below, load them after the halo instead)
    static_assert(NT % QPP == 0, "a thread's channel quad is fixed");
    float4 psc = make_float4(0.f, 0.f, 0.f, 0.f), psh = psc;
    auto load_pro = [&]() {
      const int ci = ci0 + (tid % QPP) * 4;
      if (PRO != PRO_NONE && ci < A_CIN) {
        psc = *reinterpret_cast<const float4*>(a.scale + ci);
        psh = *reinterpret_cast<const float4*>(a.shift + ci);
      }
    };
    if constexpr (EARLY_B) load_pro();
    float4 pre[MAXT];
    uint32_t valid = 0;
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
      const int task = tid + j * NT;
      pre[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (task < nstg * QPP) {
        const int px = task / QPP, q = task % QPP;
        const int py = LIN ? px / wpad : px / WP, pxx = LIN ? px - py * wpad : px % WP;
        const int ih = (LIN ? r0 : h0) - A_PH + py, iw = w0 - A_PW + pxx;
        const int ci = ci0 + q * 4;
        if (ih >= 0 && ih < HH && iw >= 0 && iw < A_W && ci < A_CIN) {
          const float* src = xclip + (ih * A_W + iw) * A_CIN + ci;
          if constexpr (PIN) {
            // pooled row ih = (clip, tt) <- unpooled rows 2 tt, 2 tt + 1 of that clip
            const int cl = ih / A_H, tt = ih - cl * A_H;
            src = a.x + ((int64_t)cl * a.h_in + 2 * tt) * A_CIN + ci;
            float4 v = *reinterpret_cast<const float4*>(src);
            if (2 * tt + 1 < a.h_in) {
              const float4 u = *reinterpret_cast<const float4*>(src + A_CIN);
              v = make_float4(fmaxf(v.x, u.x), fmaxf(v.y, u.y), fmaxf(v.z, u.z), fmaxf(v.w, u.w));
            }
            pre[j] = v;
          } else if constexpr (V4) {
            pre[j] = *reinterpret_cast<const float4*>(src);
          } else {
            pre[j].x = src[0];
            pre[j].y = ci + 1 < A_CIN ? src[1] : 0.0f;
            pre[j].z = ci + 2 < A_CIN ? src[2] : 0.0f;
            pre[j].w = ci + 3 < A_CIN ? src[3] : 0.0f;
          }
          valid |= 1u << j;
        }
      }
    }
    // tap 0's B fragments: issued here they are in flight across the staging and its barrier --
    // where the registers allow it (accumulators + halo + fragments within EARLY_B_VGPRS; the
    // variants above it spill), else after the barrier
    f16x8 bh[NTL][KS], bl[NTL][KS];
    auto load_b0 = [&]() {
#pragma unroll
      for (int nt = 0; nt < NTL; ++nt)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const size_t u = (size_t)(ch * KS + s) * kstride;
          bh[nt][s] = h3_frag(a.wh, rwh, u, lofs[nt]);
          bl[nt][s] = h3_frag(a.wl, rwl, u, lofs[nt]);
        }
    };
    if constexpr (EARLY_B) load_b0();
    else load_pro();
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
      const int task = tid + j * NT;
      if (task >= nstg * QPP) continue;
      const int px = task / QPP, q = task % QPP;
      float4 v = pre[j];
      if constexpr (PRO != PRO_NONE) {
        if (valid & (1u << j)) {
          const float4 sc = psc, sh = psh;
          v.x = pro_fn<PRO>(v.x, sc.x, sh.x);
          v.y = pro_fn<PRO>(v.y, sc.y, sh.y);
          v.z = pro_fn<PRO>(v.z, sc.z, sh.z);
          v.w = pro_fn<PRO>(v.w, sc.w, sh.w);
        }
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
      *reinterpret_cast<f16x4*>(lds_hi + px * LDP + q * 4) = hv;
      *reinterpret_cast<f16x4*>(lds_lo + px * LDP + q * 4) = lv;
    }
    __syncthreads();

    // ---- all taps of this chunk ------------------------------------------------------------------
    if constexpr (!EARLY_B) load_b0();
#pragma unroll
    for (int tap = 0; tap < TAPS; ++tap) {
      constexpr int dummy = 0;
      (void)dummy;
      const int dy = tap / KW, dx = tap % KW;
      const int toff = (dy * WP + dx) * LDP;
      f16x8 nbh[NTL][KS], nbl[NTL][KS];
      if (tap + 1 < TAPS) {   // prefetch the next tap's B fragments under this tap's MFMAs
#pragma unroll
        for (int nt = 0; nt < NTL; ++nt)
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const size_t u = (tap + 1) * tap_stride + (size_t)(ch * KS + s) * kstride;
            nbh[nt][s] = h3_frag(a.wh, rwh, u, lofs[nt]);
            nbl[nt][s] = h3_frag(a.wl, rwl, u, lofs[nt]);
          }
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          int roff = LIN ? abase[mt][LIN ? dy : 0] + dx * LDP : apix[mt] + toff;
          if constexpr (ZROW) {
            const int src = trow[mt] + dy - A_PH;
            if (src < 0 || src >= A_H) roff = NPIX * LDP;
          }
          const int off = roff + 16 * s + koff;
          const f16x8 ah = *reinterpret_cast<const f16x8*>(lds_hi + off);
          const f16x8 al = *reinterpret_cast<const f16x8*>(lds_lo + off);
#pragma unroll
          for (int nt = 0; nt < NTL; ++nt) {
            if constexpr (CIL) {   // C^T: rows = channels, columns = pixels
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bl[nt][s], ah, acc[mt][nt], 0, 0, 0);
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[nt][s], al, acc[mt][nt], 0, 0, 0);
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[nt][s], ah, acc[mt][nt], 0, 0, 0);
            } else {
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[nt][s], acc[mt][nt], 0, 0, 0);
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[nt][s], acc[mt][nt], 0, 0, 0);
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[nt][s], acc[mt][nt], 0, 0, 0);
            }
          }
        }
      }
      if (tap + 1 < TAPS) {
#pragma unroll
        for (int nt = 0; nt < NTL; ++nt)
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            bh[nt][s] = nbh[nt][s];
            bl[nt][s] = nbl[nt][s];
          }
      }
    }
  }

  // ---- epilogue ----------------------------------------------------------------------------------
  if constexpr (CIL) {
    // lane's register quad g holds channels 8 g + 4 (lane >> 5) + 0..3 of tile pixel
    // mbase + (lane & 31); the pixel's output address for every (layout) case
    auto pix_off = [&](int m, bool& ok) -> int64_t {
      if constexpr (LIN) {
        ok = p0 + m < npx;
        return (p0 + m) * A_COUT;
      } else {
        const int oh = h0 + m / (TW > 1 ? TW : 1), ow = w0 + m % (TW > 1 ? TW : 1);
        ok = oh < HH && ow < A_W;
        return ((clip * HH + oh) * A_W + ow) * A_COUT;
      }
    };
    const int cq = 4 * (lane >> 5);
    // the in-place residual: every load issued before the first store (see the pixel-row path)
    float4 rsd4[NTL][MT][4];
    if constexpr (ADD) {
#pragma unroll
      for (int nt = 0; nt < NTL; ++nt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          bool ok;
          const int64_t o = pix_off((wm * MT + mt) * 32 + (lane & 31), ok);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int co = n0 + (wn * NTL + nt) * 32 + 8 * g + cq;
            rsd4[nt][mt][g] = ok && co < A_COUT ? *reinterpret_cast<const float4*>(a.res + o + co)
                                                 : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
    }
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt) {
      float4 b4[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int co = n0 + (wn * NTL + nt) * 32 + 8 * g + cq;
        b4[g] = co < A_COUT ? *reinterpret_cast<const float4*>(a.bias + co) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        bool ok;
        const int64_t o = pix_off((wm * MT + mt) * 32 + (lane & 31), ok);
        if (!ok) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co = n0 + (wn * NTL + nt) * 32 + 8 * g + cq;
          if (co >= A_COUT) continue;
          float4 v = make_float4(fmaf(acc[mt][nt][4 * g], a.unscale, b4[g].x),
                                 fmaf(acc[mt][nt][4 * g + 1], a.unscale, b4[g].y),
                                 fmaf(acc[mt][nt][4 * g + 2], a.unscale, b4[g].z),
                                 fmaf(acc[mt][nt][4 * g + 3], a.unscale, b4[g].w));
          if constexpr (ADD) {
            const float4 r = rsd4[nt][mt][g];
            v = make_float4(v.x + r.x, v.y + r.y, v.z + r.z, v.w + r.w);
          }
          *reinterpret_cast<float4*>(a.y + o + co) = v;
        }
      }
    }
  } else {
  // lane's accumulator register r holds tile row m = mbase + (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  const int hsel = 4 * (lane >> 5);
  // pooled blocks: the shortcut Conv2D(1x1, stride 2) as a 3xFP16 GEMM whose accumulator layout is
  // the pooled one.  A lane's pooled outputs are (m-tile mt, window j) = 4 per m-tile, 16 in all --
  // one 32x32 MFMA tile: register r = 4 mt + j of lane-half h is row (r & 3) + 8 (r >> 2) + 4 h, so A
  // row rho holds the input pixel of window (mt = rho >> 3, j = rho & 3, h = (rho >> 2) & 1), i.e. the
  // window's top-left pixel (oh, ow) -- exactly the pixel the stride-2 1x1 conv samples
  f32x16 sacc[NTL];
  bool has_sc = false;
  if constexpr (POOL && MT == 4) {   // other tilings: the launcher refuses a shortcut
    has_sc = a.sc_x != nullptr;
    if (has_sc) {
      constexpr int TWP = TW == 16 ? 16 : 8;
      const int rho = lane & 31;
      const int smt = rho >> 3, sj = rho & 3, sh = (rho >> 2) & 1;
      // the j-th (q, e) window of the pooled loop below: TW 16 -> q = j >> 1; TW 8 -> q = 2 (j >> 1)
      const int sq = TW == 16 ? (sj >> 1) : 2 * (sj >> 1), se = 2 * (sj & 1);
      const int sm_ = (wm * MT + smt) * 32 + 8 * sq + 4 * sh + se;
      const int soh = h0 + sm_ / TWP, sow = w0 + sm_ % TWP;
      const bool sok = soh < A_H && sow < A_W;
      const float* sx = a.sc_x + ((clip * A_H + (sok ? soh : 0)) * A_W + (sok ? sow : 0)) * a.sc_cin + koff;
      const size_t sks = (size_t)(A_COUTP / 32) * 512;
#pragma unroll
      for (int nt = 0; nt < NTL; ++nt)
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[nt][i] = 0.0f;
      for (int s = 0; s < a.sc_cin / 16; ++s) {
        float4 x0 = make_float4(0.f, 0.f, 0.f, 0.f), x1 = x0;
        if (sok) {
          x0 = *reinterpret_cast<const float4*>(sx + 16 * s);
          x1 = *reinterpret_cast<const float4*>(sx + 16 * s + 4);
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
#pragma unroll
        for (int nt = 0; nt < NTL; ++nt) {
          const size_t u = (size_t)s * sks + lofs[nt];
          const f16x8 wh = *reinterpret_cast<const f16x8*>(a.sc_wh + u);
          const f16x8 wl = *reinterpret_cast<const f16x8*>(a.sc_wl + u);
          sacc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wl, sacc[nt], 0, 0, 0);
          sacc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, wh, sacc[nt], 0, 0, 0);
          sacc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wh, sacc[nt], 0, 0, 0);
        }
      }
    }
  }
  // the residual is added in place (res == y): all of the lane's residual loads are issued before
  // its first store, otherwise every load waits behind the previous (possibly aliasing) store
  float rsd[NTL][MT][16];
  bool sc_res = false;
  if constexpr (SCR && !POOL && TW == 1) {
    // the pool unit's shortcut Conv1D(1, stride 2) computed here as the residual: a 3xFP16 GEMM whose
    // A row is the output row's source row 2 tt of sc_x, accumulated in the main tile's layout
    sc_res = true;
    {
      const size_t sks = (size_t)(A_COUTP / 32) * 512;
      f32x16 sacc[NTL][MT];
#pragma unroll
      for (int nt = 0; nt < NTL; ++nt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int i = 0; i < 16; ++i) sacc[nt][mt][i] = 0.0f;
      const float* sxp[MT];
      bool sok[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int rg = h0 + (wm * MT + mt) * 32 + (lane & 31);   // global output row (clip, tt)
        sok[mt] = rg < HH;
        const int cl = (sok[mt] ? rg : 0) / A_H, tt = (sok[mt] ? rg : 0) - ((sok[mt] ? rg : 0) / A_H) * A_H;
        sxp[mt] = a.sc_x + ((int64_t)cl * a.sc_h + 2 * tt) * a.sc_cin + koff;
      }
      for (int s = 0; s < a.sc_cin / 16; ++s) {
        f16x8 bh_[NTL], bl_[NTL];
#pragma unroll
        for (int nt = 0; nt < NTL; ++nt) {
          bh_[nt] = h3_frag(a.sc_wh, h3_rsrc(a.sc_wh), (size_t)s * sks, lofs[nt]);
          bl_[nt] = h3_frag(a.sc_wl, h3_rsrc(a.sc_wl), (size_t)s * sks, lofs[nt]);
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          float4 x0 = make_float4(0.f, 0.f, 0.f, 0.f), x1 = x0;
          if (sok[mt]) {
            x0 = *reinterpret_cast<const float4*>(sxp[mt] + 16 * s);
            x1 = *reinterpret_cast<const float4*>(sxp[mt] + 16 * s + 4);
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
#pragma unroll
          for (int nt = 0; nt < NTL; ++nt) {
            sacc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, bl_[nt], sacc[nt][mt], 0, 0, 0);
            sacc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, bh_[nt], sacc[nt][mt], 0, 0, 0);
            sacc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, bh_[nt], sacc[nt][mt], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int nt = 0; nt < NTL; ++nt) {
        const int co = n0 + (wn * NTL + nt) * 32 + (lane & 31);
        const float bsc = co < A_COUT ? a.sc_bias[co] : 0.0f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int i = 0; i < 16; ++i) rsd[nt][mt][i] = fmaf(sacc[nt][mt][i], a.sc_unscale, bsc);
      }
    }
  }
  if constexpr (ADD && !POOL) {
    if (!sc_res)
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt) {
      const int co = n0 + (wn * NTL + nt) * 32 + (lane & 31);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int mbase = (wm * MT + mt) * 32;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int m0 = mbase + 8 * g + hsel;
          if constexpr (LIN) {
            const float* rp = a.res + (p0 + m0) * A_COUT + co;
#pragma unroll
            for (int j = 0; j < 4; ++j)
              rsd[nt][mt][4 * g + j] = co < A_COUT && p0 + m0 + j < npx ? rp[j * A_COUT] : 0.0f;
            continue;
          }
          const int oh = h0 + m0 / (LIN ? 1 : TW), ow0 = w0 + m0 % (LIN ? 1 : TW);
          const float* rp = a.res + ((clip * HH + oh) * A_W + ow0) * A_COUT + co;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int step = TW == 1 ? A_W * A_COUT : A_COUT;
            const bool ok = co < A_COUT && oh < HH && (TW == 1 ? (oh + j < HH) : (ow0 + j < A_W));
            rsd[nt][mt][4 * g + j] = ok ? rp[j * step] : 0.0f;
          }
        }
      }
    }
  }
#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) {
    const int co = n0 + (wn * NTL + nt) * 32 + (lane & 31);
    if (co >= A_COUT) continue;
    const float b = EARLY_B ? bias_r[nt] : a.bias[co];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = fmaf(acc[mt][nt][r], a.unscale, b);
      const int mbase = (wm * MT + mt) * 32;
      if constexpr (POOL) {
        // windows: top-left rows i = 8q + hsel + e (i % TW even, (i / TW) even) -> registers
        // {4q+e, 4q+e+1, 4q+e+TW/2, 4q+e+TW/2+1}  (row + TW = register + TW/2)
        static_assert(TW == 16 || TW == 8, "pooled epilogue needs TW 8 or 16");
        constexpr int TWP = TW == 16 ? 16 : 8;
        const int hp = (A_H + 1) >> 1, wp = (A_W + 1) >> 1;
        const float bsc = has_sc ? a.sc_bias[co] : 0.0f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            constexpr int R = TW / 2;
            const int i = 8 * q + hsel + e;
            if ((i / TWP) & 1) continue;                   // only top rows of window pairs
            if (4 * q + e + R + 1 > 15) continue;
            // window index j of this m-tile (the shortcut accumulator's register 4 mt + j): the rows
            // kept above depend on q only (hsel + e < 8), so j is compile-time
            const int jr = TW == 16 ? 2 * q + e / 2 : (q >> 1) * 2 + e / 2;
            const int m = mbase + i;
            const int oh = h0 + m / TWP, ow = w0 + m % TWP;
            if (oh >= A_H || ow >= A_W) continue;
            float mx = v[4 * q + e];
            if (ow + 1 < A_W) mx = fmaxf(mx, v[4 * q + e + 1]);
            if (oh + 1 < A_H) {
              mx = fmaxf(mx, v[4 * q + e + R]);
              if (ow + 1 < A_W) mx = fmaxf(mx, v[4 * q + e + R + 1]);
            }
            // Add()([MaxPool2D(t2), shortcut]): the shortcut's bias added in its own rounding step
            if (has_sc) mx += fmaf(sacc[nt][4 * mt + jr], a.sc_unscale, bsc);
            a.y[((clip * hp + (oh >> 1)) * wp + (ow >> 1)) * A_COUT + co] = mx;
          }
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) {        // 4 groups of 4 consecutive tile rows
          const int m0 = mbase + 8 * g + hsel;
          if constexpr (LIN) {               // 4 consecutive pixels of the flattened batch
            float* yp = a.y + (p0 + m0) * A_COUT + co;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              if (p0 + m0 + j >= npx) continue;
              float val = v[4 * g + j];
              if constexpr (ADD) val += rsd[nt][mt][4 * g + j];
              yp[j * A_COUT] = val;
            }
            continue;
          }
          const int oh = h0 + m0 / (LIN ? 1 : TW);
          if (oh >= HH) continue;
          const int ow0 = w0 + m0 % (LIN ? 1 : TW);
          float* yp = a.y + ((clip * HH + oh) * A_W + ow0) * A_COUT + co;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            // TW >= 4 keeps the 4 rows in one image row; TW == 1 walks image rows instead
            const int step = TW == 1 ? A_W * A_COUT : A_COUT;
            const bool ok = TW == 1 ? (oh + j < HH) : (ow0 + j < A_W);
            if (!ok) continue;
            float val = v[4 * g + j];
            if constexpr (ADD) val += rsd[nt][mt][4 * g + j];
            yp[j * step] = val;
          }
        }
      }
    }
  }
  }   // CIL
  if (rbad && a.range_flag) *a.range_flag = 1;
}

template <int KH, int KW, int CK, int BN, int TW, int PRO, int EPI, bool POOL, bool V4 = true,
          bool PIN = false, class SHP = Shape<0, 0, 0, 0>>
hipError_t launch(ConvH3Args a, hipStream_t s) {
  constexpr int BMK = tile_px<KH, BN, TW>();
  // the fused pooled shortcut needs 4 m-tiles per wave (16 pooled outputs per lane) and 16-channel steps
  constexpr int WN_ = BN / 32, MT_ = BMK / ((4 / WN_) * 32);
  if ((EPI == EPI_ADD_SC) != (a.sc_x && !POOL)) return hipErrorInvalidValue;
  if (a.sc_x && ((POOL ? MT_ != 4 : !(EPI == EPI_ADD_SC && TW == 1 && a.sc_h > 0)) || a.sc_cin % 16 != 0 ||
                 a.sc_cin <= 0))
    return hipErrorInvalidValue;
  if constexpr (TW == 0) {
    a.th = 0;
    a.tiles_w = 1;
    a.tiles_h = (int)(((int64_t)a.n * a.h * a.w + BMK - 1) / BMK);
  } else {
    a.th = BMK / TW;
    a.tiles_h = TW == 1 ? (int)(((int64_t)a.n * a.h + a.th - 1) / a.th) : (a.h + a.th - 1) / a.th;
  }
  const int64_t tiles = (int64_t)a.tiles_h * a.tiles_w * (TW <= 1 ? 1 : a.n);
  dim3 grid((unsigned)tiles, (unsigned)(a.cout_pad / BN));
  hipLaunchKernelGGL((conv_h3_kernel<KH, KW, CK, BN, TW, PRO, EPI, POOL, V4, PIN, SHP>), grid,
                     dim3(NT), 0, s, a);
  return hipGetLastError();
}

template <int KH, int KW, int CK, int TW, int PRO, int EPI, bool POOL, bool PIN = false,
          class SHP = Shape<0, 0, 0, 0>>
hipError_t by_bn(const ConvH3Args& a, hipStream_t s) {
  if (a.cout_pad % 128 == 0) return launch<KH, KW, CK, 128, TW, PRO, EPI, POOL, true, PIN, SHP>(a, s);
  if (a.cout_pad % 64 == 0) return launch<KH, KW, CK, 64, TW, PRO, EPI, POOL, true, PIN, SHP>(a, s);
  return launch<KH, KW, CK, 32, TW, PRO, EPI, POOL, true, PIN, SHP>(a, s);
}

}  // namespace

hipError_t conv_h3_launch(ConvH3Args a, hipStream_t s) {
  if ((int64_t)a.n * a.h * a.w == 0) return hipSuccess;
  if (a.cout_pad % 32 != 0) return hipErrorInvalidValue;
  // SI stem Conv1D(32, 4, same) on the [t, 39] features: element-wise staging, cin_pad 48
  if (a.cin % 4 != 0) {
    if (a.kh == 4 && a.kw == 1 && a.w == 1 && a.cin_pad % 16 == 0 && a.cout_pad == 32 &&
        a.pro == PRO_NONE && a.epi == EPI_BIAS && !a.pool_out) {
      a.tw = 1;
      a.tiles_w = 1;
      return launch<4, 1, 16, 32, 1, PRO_NONE, EPI_BIAS, false, false>(a, s);
    }
    return hipErrorInvalidValue;
  }
  // tile: 16 wide for wide images, 8 for narrow ones (W = 38, 19), 1 for Conv1D
  // (th, tiles_h follow from the variant's tile size in launch<>; Conv1D is one row sequence
  // over all clips, conv_h3_kernel TW == 1)
  a.tw = a.w == 1 ? 1 : (a.w >= 48 ? 16 : 8);
  // narrow images whose 128-pixel tiles span few rows: linear-pixel tiles (TW = 0), no padding
  // columns (W = 19: 8-wide tiles compute 24 columns for 19)
  if (a.w > 1 && a.w < 24 && !a.pool_out && a.w + a.kw - 1 <= LIN_WP &&
      (a.w - 1 + BM - 1) / a.w + a.kh <= LIN_SLOTS)
    a.tw = 0;
  a.tiles_w = a.tw == 0 ? 1 : (a.w + a.tw - 1) / a.tw;
  const int ck = a.cin_pad % 32 == 0 ? 32 : 16;
  if (a.sc_x && !a.pool_out && a.epi == EPI_ADD) a.epi = EPI_ADD_SC;   // Conv1D + fused shortcut
  if (a.cin_pad % ck != 0) return hipErrorInvalidValue;
  if (a.pool_in) {   // SI pool unit: MaxPool1D(2) -> BN -> ReLU -> Conv1D(3)
    if (a.kh == 3 && a.kw == 1 && ck == 32 && a.tw == 1 && a.pro == PRO_BN_RELU &&
        a.epi == EPI_BIAS && !a.pool_out && a.h_in >= 2 * a.h - 1 && a.h_in <= 2 * a.h)
      return by_bn<3, 1, 32, 1, PRO_BN_RELU, EPI_BIAS, false, true>(a, s);
    return hipErrorInvalidValue;
  }
  // the fixed OD-NET layers (blocks 4-9 on the 128 x 151 image): compile-time geometry
  const bool std_pad = a.pad_h == (a.kh - 1) / 2 && a.pad_w == (a.kw - 1) / 2 &&
                       a.cin == a.cin_pad && a.cout == a.cout_pad;
#define H3F(KH, KW, TW, E, PL, H, W, CI, CO)                                                     \
  if (std_pad && a.kh == KH && a.kw == KW && ck == 32 && a.tw == TW && a.pro == PRO_BN_ELU &&   \
      a.epi == E && (a.pool_out != 0) == PL && a.h == H && a.w == W && a.cin == CI &&          \
      a.cout == CO)                                                                            \
    return by_bn<KH, KW, 32, TW, PRO_BN_ELU, E, PL, false, Shape<H, W, CI, CO>>(a, s);
  H3F(3, 3, 16, EPI_BIAS, false, 64, 76, 32, 64)     // block 4
  H3F(4, 1, 16, EPI_BIAS, true, 64, 76, 64, 64)
  H3F(3, 3, 8, EPI_BIAS, false, 32, 38, 64, 64)      // blocks 5-6
  H3F(4, 1, 8, EPI_ADD, false, 32, 38, 64, 64)
  H3F(3, 3, 8, EPI_BIAS, false, 32, 38, 64, 128)     // block 7
  H3F(4, 1, 8, EPI_BIAS, true, 32, 38, 128, 128)
  H3F(3, 3, 0, EPI_BIAS, false, 16, 19, 128, 128)    // blocks 8-9
  // (blocks 8-9 conv(4,1) + residual: the fixed-shape build was slower, 3.0 -> 3.3 ms)
#undef H3F
  // (the SI Conv1D layers gained nothing from a fixed geometry: 48.3 vs 48.1 ms per step, A/B)
#define H3(KH, KW, CK, TW, P, E, PL)                                                           \
  if (a.kh == KH && a.kw == KW && ck == CK && a.tw == TW && a.pro == P && a.epi == E &&        \
      (a.pool_out != 0) == PL)                                                                 \
    return by_bn<KH, KW, CK, TW, P, E, PL>(a, s);
  // OD-NET res_block convs (overlap_detector_temp.py:258-274)
  H3(3, 3, 16, 16, PRO_BN_ELU, EPI_BIAS, false)
  H3(3, 3, 32, 16, PRO_BN_ELU, EPI_BIAS, false)
  H3(3, 3, 32, 8, PRO_BN_ELU, EPI_BIAS, false)
  H3(3, 3, 32, 0, PRO_BN_ELU, EPI_BIAS, false)
  H3(4, 1, 32, 16, PRO_BN_ELU, EPI_BIAS, true)
  H3(4, 1, 32, 8, PRO_BN_ELU, EPI_BIAS, true)
  H3(4, 1, 32, 16, PRO_BN_ELU, EPI_ADD, false)
  H3(4, 1, 32, 8, PRO_BN_ELU, EPI_ADD, false)
  H3(4, 1, 32, 0, PRO_BN_ELU, EPI_ADD, false)
  // SI-NET res_unit convs (speaker_identification.py:173-188)
  H3(3, 1, 32, 1, PRO_BN_RELU, EPI_BIAS, false)
  H3(3, 1, 32, 1, PRO_BN_RELU, EPI_ADD, false)
  H3(3, 1, 32, 1, PRO_BN_RELU, EPI_ADD_SC, false)
  // SI stem Conv1D(32, 4) on 40-float feature rows (si_fe's padded layout; speaker_identification.py:195)
  H3(4, 1, 16, 1, PRO_NONE, EPI_BIAS, false)
  // SI-NET Dense head as a 1x1 conv over the clips (speaker_identification.py:216)
  H3(1, 1, 32, 1, PRO_NONE, EPI_BIAS, false)
#undef H3
  return hipErrorInvalidValue;
}

static uint16_t f32_to_f16_bits(float f) {
  _Float16 h = (_Float16)f;
  uint16_t b;
  memcpy(&b, &h, 2);
  return b;
}

void conv_h3_split_weights(const float* w, int kh, int kw, int cin, int cout, int cin_pad,
                           int cout_pad, uint16_t* hi, uint16_t* lo, float wscale) {
  const size_t n = (size_t)kh * kw * cout_pad * cin_pad;
  for (size_t i = 0; i < n; ++i) hi[i] = lo[i] = 0;
  for (int t = 0; t < kh * kw; ++t)
    for (int ci = 0; ci < cin; ++ci)
      for (int co = 0; co < cout; ++co) {
        const float v = w[((size_t)t * cin + ci) * cout + co] * wscale;   // exact (power of two)
        const _Float16 h = (_Float16)v;
        // MFMA fragment order: [tap][ci / 16][co / 32][lane = co % 32 + 32 (ci % 16 / 8)][ci % 8]
        const size_t o = (size_t)t * cout_pad * cin_pad +
                         (((size_t)(ci / 16) * (cout_pad / 32) + co / 32) * 64 + co % 32 +
                          32 * ((ci % 16) / 8)) * 8 + ci % 8;
        hi[o] = f32_to_f16_bits(v);
        lo[o] = f32_to_f16_bits(v - (float)h);
      }
}

