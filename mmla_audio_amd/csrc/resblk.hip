// Fused OD-NET res_block (overlap_detector_temp.py:253-277) on gfx950 f16 MFMA, 3xFP16 products.
//
//   t1 = Conv2D(C, 3x3, same)(ELU(BN1(x)))              -- GEMM 1, K = 9 * CIN
//   t2 = Conv2D(C, (4,1), same)(ELU(BN2(t1)))           -- GEMM 2, K = 4 * C
//   y  = x + t2                       (non-pool blocks)
//   y  = MaxPool2D(2, same)(t2)       (pool blocks; the Conv2D(1x1, stride 2) shortcut is added by
//                                      the next launch, conv.hip EPI_ADD)
//
// One workgroup (4 waves) owns a 16 x 16 output tile of one clip and ALL C channels.  The
// intermediate t1 never touches HBM: its 19 x 16 tile (one row above, two below: the (4,1) 'same'
// padding) is computed from a 21 x 18 input halo staged in LDS, BN2 + ELU + the hi/lo split are applied
// once per element, and the result is re-staged in the SAME LDS bytes for GEMM 2.  HBM traffic per
// block is the input halo (21*18 / 16*16 = 1.48 x the input) plus the output, instead of
// in + t1 + t1 + out (+ residual) for the two-launch form; the price is recomputing 3 of every 19 t1
// rows.
//
// MFMA v_mfma_f32_16x16x32_f16: one 16-row M tile = one 16-pixel image row segment of the tile, so
// the pixel <-> (row, col) map is the tile row index and the lane's column.  Lane l holds
// A[row l & 15][k 8 (l >> 4) .. +7] (one ds_read_b128 per operand half), B[k 8 (l >> 4) .. +7][col
// l & 15] (one 16-B global load from the [C][K] weight image) and C[rows 4 (l >> 4) .. +3][col l & 15].
// K runs over (tap, channel) with the channel fastest, so CIN = 16 packs two taps per k-step.
// 3xFP16 as in conv_h3.hip: activations x 2^4 and weights x 2^8 split into hi + lo (lo unscaled),
// ONE accumulator per tile: acc += hi*hi + hi*lo + lo*hi; value = acc * 2^-12.
#include "common.h"
#include "resblk.h"

#define RB_MARK(k)

#include <algorithm>
#include <cstring>

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 256;
constexpr int TW = 16;
constexpr int TH = 16;                 // output rows per tile (block 1; blocks 2-3: TH_NP)
constexpr int TH_NP = 16;          // output rows per tile of the non-pool blocks 2-3
constexpr float ACT_SCALE = 16.0f;     // 2^4: every split activation
// weights: split at a per-tensor power-of-two scale (resblk_split_weights; the a.u1 / a.u2 / a.us
// epilogue factors are 2^-4 / that scale)
constexpr float ACT_RANGE = 65504.0f / ACT_SCALE;

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
constexpr float LOG2E = 1.4426950408889634f;

// TF Elu on a pair (v_pk_* for the arithmetic): x > 0 ? x : exp(x) - 1
__device__ __forceinline__ f32x2 elu2(f32x2 u) {
  const f32x2 t = u * LOG2E;
  f32x2 e = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  e = e - 1.0f;
  return f32x2{u.x > 0.0f ? u.x : e.x, u.y > 0.0f ? u.y : e.y};
}

// v * 2^4 = hi + lo, both fp16 (RNE).  lo = f16(v' - hi) by v_fma_mix: the exact difference rounded
// once, as cvt(v' - f32(hi)) rounds it (v' - hi is exact in f32) -- bit-identical, 4 VALU per pair
// instead of 6 (two v_cvt_f32_f16 and a v_pk_add gone); clang keeps the cvt + sub + cvt form itself
__device__ __forceinline__ void split2(f32x2 v, f16x2& h, f16x2& l) {
  v = v * ACT_SCALE;
  h = __builtin_convertvector(v, f16x2);
  uint32_t lu;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %3, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(lu) : "v"(v.x), "v"(__builtin_bit_cast(uint32_t, h)), "v"(v.y));
  l = __builtin_bit_cast(f16x2, lu);
}

// GEMM 1 / GEMM 2 B fragments by raw buffer loads from a wave-uniform descriptor
// (voffset = the lane's offset, soffset = the uniform (k-step, tile) offset): no per-load 64-bit
// address VALU (as conv_h3.hip h3_frag)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rb_rsrc(const void* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)0x7fffffff, 0x00020000);
}
// 16 B of a split weight at half index uoff (wave-uniform) + lofs (this lane's)
__device__ __forceinline__ f16x8 rb_frag(const uint16_t* base, __amdgpu_buffer_rsrc_t r, int uoff,
                                         int lofs) {
  (void)base;
  return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)lofs * 2u, uoff * 2, 0));
}

// the 3 channels of image pixel `pix` (uint8 decoded PNG or float NHWC), as floats
// 3xFP16 range guard: false when a value about to be split leaves the fp16 range once scaled
// (|v| >= 65504 / 2^4) or is not finite
__device__ __forceinline__ bool in_f16_range(f32x2 a, f32x2 b) {
  return fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(b.x), fabsf(b.y))) < ACT_RANGE;
}

__device__ __forceinline__ float4 image_px(const ResBlkArgs& a, int64_t pix) {
  if (a.img8) {
    const uint8_t* p = a.img8 + pix * 3;
    return make_float4((float)p[0], (float)p[1], (float)p[2], 0.f);
  }
  const float* p = a.imgf + pix * 3;
  return make_float4(p[0], p[1], p[2], 0.f);
}
template <int CIN, int C, bool POOL>
struct Geo {
  static constexpr int WN = 1;                     // waves along N: each wave owns all C columns,
                                                   // so every A fragment read feeds C/16 N tiles
  static constexpr int WM = 4 / WN;                // waves along M (tile rows)
  static constexpr int NTW = C / 16 / WN;          // N tiles per wave
  static constexpr int TH = POOL ? ::TH : TH_NP;   // output rows per tile
  static constexpr int TR = TH + 3;                // t1 rows needed: image rows h0-1 .. h0+TH+1
  static constexpr int TRP = (TR + WM - 1) / WM * WM;   // computed (padded: no per-row branches)
  // input halo rows h0-2 .. h0+TH+2 (the padded t1 row reads one row past it: finite LDS data,
  // discarded result), cols w0-1 .. w0+TW
  static constexpr int XR = TR + 2, XC = TW + 2, XNP = XR * XC;
  // LDS pixel layouts.  ds_read_b128 of a 16 x 32 fragment (lanes = 16 consecutive pixels x 4
  // 16-B k-groups) is conflict-free when the pixel stride is 32 mod 64 bytes
  // (MI355X_MICROARCH.md LDS lane groups): 16 channels -> separate hi / lo planes of 32-B pixels;
  // 32 channels -> hi and lo interleaved in one 160-B pixel (64 + 64 + 32 pad).
  static constexpr int XPS = CIN == 16 ? 16 : (2 * CIN + 16 + 31) / 32 * 32 - 16;   // halfs
  static constexpr int XLO = CIN == 16 ? XNP * 16 : CIN;     // lo offset from hi (halfs)
  static constexpr int XREG = CIN == 16 ? 2 * XNP * 16 : XNP * XPS;
  static constexpr int TPS = (2 * C + 16 + 31) / 32 * 32 - 16;   // t1: interleaved hi | lo | pad
  static constexpr int TLO = C;
  static constexpr int TREG = TRP * TW * TPS;
  static constexpr int SM = XREG > TREG ? XREG : TREG;
  static constexpr int MT1 = TRP / WM;             // t1 rows per wave (GEMM 1)
  static constexpr int MT2 = TH / WM;              // output rows per wave (GEMM 2)
  static constexpr int KS1 = (9 * CIN + 31) / 32;  // GEMM 1 k-steps
  static constexpr int K1PAD = KS1 * 32;
  static constexpr int KS2 = 4 * C / 32;           // GEMM 2 k-steps
  static constexpr int KSC = (CIN + 31) / 32;      // shortcut (1x1) k-steps
  static constexpr int LW2 = 4 * C + 16;           // halfs per LDS row of GEMM 2's weights (288 B)
  // GEMM 2's weights: block 1 reads them from L2 in fragment order, one k-step ahead, so that its
  // LDS (51 KB) admits a third workgroup per CU: conv 1432 -> 1386 ms per OD step (A/B).  (With
  // the [co][k] rows and no prefetch the same move had been 7.5 % slower.)  Blocks 2-3 keep them in
  // LDS: without them they still need 60 KB, two workgroups per CU.
  static constexpr bool W2LDS = CIN != 16 && TH == 16;
  static constexpr int W2 = W2LDS ? C * LW2 : 0;
  static constexpr int MINB = W2LDS ? 2 : 3;   // resident workgroups per CU
  static constexpr int PF = 3;                     // GEMM 1 B fragments in flight (k-steps)
  static constexpr int QPP = CIN / 4;              // float4 per halo pixel
  static constexpr int MAXT = (XNP * QPP + NT - 1) / NT;
  static_assert(CIN % 16 == 0 && C % 16 == 0, "channel tiles");
  static_assert(!POOL || MT2 % 4 == 0, "pooled shortcut tiles need 4 output rows per wave");
  static_assert(NT % QPP == 0, "a thread's channel quad is fixed");
};

// STEM: the block input is the stem Conv2D(16, 1x1) of the image, computed while staging (block 1)
template <int CIN, int C, bool POOL, bool STEM>
__global__ void __launch_bounds__(NT, (Geo<CIN, C, POOL>::MINB)) resblk_kernel(ResBlkArgs a) {
  using G = Geo<CIN, C, POOL>;
  constexpr int XC = G::XC, XPS = G::XPS, TPS = G::TPS, MT1 = G::MT1, MT2 = G::MT2, NTW = G::NTW;
  constexpr int KS1 = G::KS1, KS2 = G::KS2, PF = G::PF, QPP = G::QPP;
  constexpr int MAXT = G::MAXT, WN = G::WN;
  // [halo | t1] (hi and lo, layouts in Geo), then GEMM 2's weights hi, lo
  __shared__ __attribute__((aligned(16))) _Float16 smem[G::SM + 2 * G::W2];
  _Float16* const s_w2h = smem + G::SM;
  _Float16* const s_w2l = s_w2h + G::W2;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // SGPR: per-wave values are scalar
  const int wn = wave % WN, wm = wave / WN;
  const int col = lane & 15, grp = lane >> 4;
  const int tiles = a.tiles_h * a.tiles_w;
  const int bid = (int)xcd_block_id();
  const int clip = bid / tiles;
  const int tile = bid - clip * tiles;
  const int th_i = tile / a.tiles_w;
  constexpr int TH = G::TH;
  const int h0 = th_i * TH, w0 = (tile - th_i * a.tiles_w) * TW;

  RB_MARK(0);
  bool rbad = false;   // 3xFP16 range guard (ResBlkArgs::range_flag)
  // ---- per-thread parameters first: BN1 (+ stem) for the staging, BN2 / bias for the t1 re-staging
  //      and the epilogue.  Issued here they share the halo's memory latency; issued where they are
  //      used (after a barrier or a dependent wait) each group cost a round trip of its own --------
  const int q = tid % QPP;
  const float4 sc4 = *reinterpret_cast<const float4*>(a.s1 + 4 * q);
  const float4 sh4 = *reinterpret_cast<const float4*>(a.t1 + 4 * q);
  // STEM: the image halo is loaded ONCE per pixel (not once per channel quad) into LDS as float4
  // {r, g, b, inside-image}, the stem weights as [co] float4 {w_r, w_g, w_b, bias}; the staging and
  // the shortcut operands read both from LDS behind one extra barrier.  Both live past the halo's
  // hi/lo planes, inside bytes that t1 only takes after GEMM 1 (GEMM 1's padded rows may read them:
  // finite fp16 patterns).  Per thread this issues <= 7 loads where the per-task image and per-channel
  // weight loads were ~50 (a phase timeline: the halo phase was the longest of block 1).
  float4* const s_img = reinterpret_cast<float4*>(smem + G::XREG);
  float4* const s_wst = s_img + G::XNP;
  static_assert(!STEM || (G::XREG % 8 == 0 && G::XREG * 2 + (G::XNP + 16) * 16 <= G::SM * 2),
                "stem staging buffers fit behind the halo planes");
  float stw[3][4], stb[4];   // STEM: this thread's stem weights (channels 4q .. 4q+3), from s_wst
  if constexpr (STEM) {
    constexpr int PPT = (G::XNP + NT - 1) / NT;   // pixels per thread
    float4 im[PPT];
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int p = tid + k * NT;
      im[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      const int py = p / XC, pxx = p - (p / XC) * XC;
      const int ih = h0 - 2 + py, iw = w0 - 1 + pxx;
      if (p < G::XNP && ih >= 0 && ih < a.h && iw >= 0 && iw < a.w) {
        im[k] = image_px(a, ((int64_t)clip * a.h + ih) * a.w + iw);
        im[k].w = 1.0f;
      }
    }
    if (tid < 64) {   // [co][k]: k < 3 weights of the r, g, b inputs, k = 3 the bias
      const int co = tid >> 2, k = tid & 3;
      reinterpret_cast<float*>(s_wst)[tid] = k < 3 ? a.wst[k * a.ldst + co] : a.bst[co];
    }
#pragma unroll
    for (int k = 0; k < PPT; ++k)
      if (tid + k * NT < G::XNP) s_img[tid + k * NT] = im[k];
  }
  float ps2[NTW], pb1[NTW], pt2[NTW], pbo[NTW];   // BN2 scale / conv-1 bias / BN2 shift, out bias
#pragma unroll
  for (int nt = 0; nt < NTW; ++nt) {
    const int n = (wn * NTW + nt) * 16 + col;
    ps2[nt] = a.s2[n];
    pb1[nt] = a.b1[n];
    pt2[nt] = a.t2[n];
    pbo[nt] = POOL ? a.b2[n] + a.bs[n] : a.b2[n];
  }

  // ---- issue the halo loads (all in flight at once) ----------------------------------------------
  float4 pre[MAXT];
  uint32_t valid = 0;
  {
    const float* xc = STEM ? nullptr : a.x + (int64_t)clip * a.h * a.w * CIN + 4 * q;
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
      const int px = (tid + j * NT) / QPP;
      pre[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (px < G::XNP) {
        const int py = px / XC, pxx = px - (px / XC) * XC;
        const int ih = h0 - 2 + py, iw = w0 - 1 + pxx;
        if (ih >= 0 && ih < a.h && iw >= 0 && iw < a.w) {
          if constexpr (!STEM) {   // (STEM: from s_img after the barrier below)
            pre[j] = *reinterpret_cast<const float4*>(xc + (ih * a.w + iw) * CIN);
          }
          valid |= 1u << j;
        }
      }
    }
  }
  // pool blocks: the Conv2D(1x1, stride 2) shortcut on the raw input is a small 3xFP16 GEMM whose M
  // rows are ordered so that its accumulator layout equals the pooled epilogue's: tile j of this
  // wave, element i of lane (grp, col) = pooled row wm*MT2/2 + 2j + (i >> 1), pooled column
  // 2 grp + (i & 1), channel col.  Its operands are loaded here, beside the halo.
  constexpr int MSC = POOL ? MT2 / 4 : 1;
  constexpr int KSC = POOL ? G::KSC : 1;
  float4 scx[KSC][MSC][2];
  f16x8 scbh[KSC][NTW], scbl[KSC][NTW];
  f32x4 e1[MSC][NTW];
  if constexpr (POOL) {
    const int p = col;                            // this lane's A row (pooled pixel of the tile)
    const int pr = (p & 3) >> 1, pc = 2 * (p >> 2) + (p & 1);
    const float* xc = STEM ? nullptr : a.x + (int64_t)clip * a.h * a.w * CIN;
#pragma unroll
    for (int s = 0; s < KSC; ++s) {
      const int ci = 32 * s + 8 * grp;
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int co = (wn * NTW + nt) * 16 + col;
        scbh[s][nt] = *reinterpret_cast<const f16x8*>(a.wsh + co * (KSC * 32) + ci);
        scbl[s][nt] = *reinterpret_cast<const f16x8*>(a.wsl + co * (KSC * 32) + ci);
      }
#pragma unroll
      for (int j = 0; j < MSC; ++j) {
        const int ih = h0 + 2 * (wm * (MT2 / 2) + 2 * j + pr), iw = w0 + 2 * pc;
        scx[s][j][0] = scx[s][j][1] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!STEM && ci < CIN && ih < a.h && iw < a.w) {   // (STEM: from LDS after the barrier)
          const float* src = xc + (ih * a.w + iw) * CIN + ci;
          scx[s][j][0] = *reinterpret_cast<const float4*>(src);
          scx[s][j][1] = *reinterpret_cast<const float4*>(src + 4);
        }
      }
    }
  }
  if constexpr (G::W2LDS) {
  // GEMM 2's weights -> LDS (16-B pieces; rows padded to spread the banks)
    // (the global copy is in fragment order: k = 8 k8 + e of channel co sits at piece
    //  ((k / 32) (C / 16) + co / 16) 64 + co % 16 + 16 ((k % 32) / 8))
    for (int i = tid; i < C * (4 * C / 8); i += NT) {
      const int co = i / (4 * C / 8), k8 = i - co * (4 * C / 8);
      const int src = (((k8 / 4) * (C / 16) + co / 16) * 64 + co % 16 + 16 * (k8 % 4)) * 8;
      *reinterpret_cast<f16x8*>(s_w2h + co * G::LW2 + 8 * k8) =
          *reinterpret_cast<const f16x8*>(a.w2h + src);
      *reinterpret_cast<f16x8*>(s_w2l + co * G::LW2 + 8 * k8) =
          *reinterpret_cast<const f16x8*>(a.w2l + src);
    }
  }

  // GEMM 1's first PF k-steps of B: in flight across the staging and its barrier
  // GEMM 1's B in MFMA fragment order (resblk_split_weights, frag): per 32-deep k-step and 16-channel
  // tile the 64 lanes' 16-B fragments are 1 KB contiguous (8 whole 128-B lines per load instead of
  // 16 rows at 64 B each)
  const int b1o = (wn * NTW) * 512 + lane * 8;   // + nt * 512 + s * B1KS
  constexpr int B1KS = (C / 16) * 512;
  const __amdgpu_buffer_rsrc_t rw1h = rb_rsrc(a.w1h), rw1l = rb_rsrc(a.w1l);
  f16x8 bh[PF][NTW], bl[PF][NTW];   // ring of B fragments, PF k-steps ahead
#pragma unroll
  for (int s = 0; s < PF && s < KS1; ++s)
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      bh[s][nt] = rb_frag(a.w1h, rw1h, nt * 512 + B1KS * s, b1o);
      bl[s][nt] = rb_frag(a.w1l, rw1l, nt * 512 + B1KS * s, b1o);
    }

  if constexpr (STEM) {
    __syncthreads();   // s_img / s_wst staged
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float4 wv = s_wst[4 * q + c];
      stw[0][c] = wv.x;
      stw[1][c] = wv.y;
      stw[2][c] = wv.z;
      stb[c] = wv.w;
    }
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
      const int px = (tid + j * NT) / QPP;
      if (px < G::XNP) pre[j] = s_img[px];   // .w = 1 inside the image, matching `valid`
    }
    if constexpr (POOL) {   // the shortcut's raw stem channels ci .. ci + 7 of its pixel
      const int p = col;
      const int pr = (p & 3) >> 1, pc = 2 * (p >> 2) + (p & 1);
#pragma unroll
      for (int s = 0; s < KSC; ++s) {
        const int ci = 32 * s + 8 * grp;
#pragma unroll
        for (int j = 0; j < MSC; ++j) {
          // tile pixel (2 (wm MT2/2 + 2j + pr), 2 pc) = halo pixel (+2 rows, +1 column)
          const float4 x = s_img[(2 * (wm * (MT2 / 2) + 2 * j + pr) + 2) * XC + 2 * pc + 1];
          if (ci < CIN && x.w != 0.0f) {
            float o[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) {   // od_stem_kernel's order
              const float4 wv = s_wst[ci + c];
              float acc = x.x * wv.x;
              acc = fmaf(x.y, wv.y, acc);
              acc = fmaf(x.z, wv.z, acc);
              o[c] = acc + wv.w;
            }
            scx[s][j][0] = make_float4(o[0], o[1], o[2], o[3]);
            scx[s][j][1] = make_float4(o[4], o[5], o[6], o[7]);
          }
        }
      }
    }
  }

  RB_MARK(1);
  // ---- stage: BN1 + ELU once per element, split hi/lo; zero outside the image (conv padding) ----
  {
    const f32x2 sc01 = {sc4.x, sc4.y}, sc23 = {sc4.z, sc4.w};
    const f32x2 sh01 = {sh4.x, sh4.y}, sh23 = {sh4.z, sh4.w};
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
      const int px = (tid + j * NT) / QPP;
      if (px >= G::XNP) continue;
      float4 xv = pre[j];
      if constexpr (STEM) {   // stem channels 4q .. 4q+3, in od_stem_kernel's order
        float o[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float acc = pre[j].x * stw[0][c];
          acc = fmaf(pre[j].y, stw[1][c], acc);
          acc = fmaf(pre[j].z, stw[2][c], acc);
          o[c] = acc + stb[c];
        }
        xv = make_float4(o[0], o[1], o[2], o[3]);
      }
      f32x2 v01 = {xv.x, xv.y}, v23 = {xv.z, xv.w};
      const bool ok = (valid >> j) & 1u;
      const f32x2 u01 = elu2(v01 * sc01 + sh01), u23 = elu2(v23 * sc23 + sh23);
      v01 = ok ? u01 : f32x2{0.f, 0.f};
      v23 = ok ? u23 : f32x2{0.f, 0.f};
      rbad |= !in_f16_range(v01, v23);
      f16x2 h01, l01, h23, l23;
      split2(v01, h01, l01);
      split2(v23, h23, l23);
      const f16x4 hv = {h01.x, h01.y, h23.x, h23.y};
      const f16x4 lv = {l01.x, l01.y, l23.x, l23.y};
      *reinterpret_cast<f16x4*>(smem + px * XPS + 4 * q) = hv;
      *reinterpret_cast<f16x4*>(smem + px * XPS + G::XLO + 4 * q) = lv;
    }
  }
  __syncthreads();

  if constexpr (POOL) {
#pragma unroll
    for (int j = 0; j < MSC; ++j)
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        e1[j][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int s = 0; s < KSC; ++s)
#pragma unroll
      for (int j = 0; j < MSC; ++j) {
        const float4 u0 = scx[s][j][0], u1 = scx[s][j][1];
        rbad |= !in_f16_range(f32x2{u0.x, u0.y}, f32x2{u0.z, u0.w}) ||
                !in_f16_range(f32x2{u1.x, u1.y}, f32x2{u1.z, u1.w});
        f16x2 h0_, l0_, h1_, l1_, h2_, l2_, h3_, l3_;
        split2(f32x2{u0.x, u0.y}, h0_, l0_);
        split2(f32x2{u0.z, u0.w}, h1_, l1_);
        split2(f32x2{u1.x, u1.y}, h2_, l2_);
        split2(f32x2{u1.z, u1.w}, h3_, l3_);
        const f16x8 ah = {h0_.x, h0_.y, h1_.x, h1_.y, h2_.x, h2_.y, h3_.x, h3_.y};
        const f16x8 al = {l0_.x, l0_.y, l1_.x, l1_.y, l2_.x, l2_.y, l3_.x, l3_.y};
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          e1[j][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, scbl[s][nt], e1[j][nt], 0, 0, 0);
          e1[j][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, scbh[s][nt], e1[j][nt], 0, 0, 0);
          e1[j][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, scbh[s][nt], e1[j][nt], 0, 0, 0);
        }
      }
  }
  RB_MARK(2);
  // ---- GEMM 1: t1 rows [wm * MT1, +MT1) x this wave's N tiles, K = (tap, ci) ----------------------
  f32x4 acc1[MT1][NTW];
#pragma unroll
  for (int m = 0; m < MT1; ++m)
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) acc1[m][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    const _Float16* ahb = smem + (wm * MT1 * XC + col) * XPS;   // + m * XC * XPS (immediate)
    const _Float16* alb = ahb + G::XLO;
#pragma unroll
    for (int s = 0; s < KS1; ++s) {
      const int kk = 32 * s + 8 * grp;
      int tap = kk / CIN;
      const int ci = kk - tap * CIN;
      tap = tap > 8 ? 8 : tap;                 // k >= 9 * CIN: zero weights, any finite A
      const int dy = tap / 3, dx = tap - (tap / 3) * 3;
      const int koff = (dy * XC + dx) * XPS + ci;
      f16x8 ch[NTW], cl[NTW];
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        ch[nt] = bh[s % PF][nt];
        cl[nt] = bl[s % PF][nt];
      }
      if (s + PF < KS1) {
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          bh[s % PF][nt] = rb_frag(a.w1h, rw1h, nt * 512 + B1KS * (s + PF), b1o);
          bl[s % PF][nt] = rb_frag(a.w1l, rw1l, nt * 512 + B1KS * (s + PF), b1o);
        }
      }
#pragma unroll
      for (int m = 0; m < MT1; ++m) {
        const f16x8 ah = *reinterpret_cast<const f16x8*>(ahb + koff + m * XC * XPS);
        const f16x8 al = *reinterpret_cast<const f16x8*>(alb + koff + m * XC * XPS);
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          acc1[m][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, cl[nt], acc1[m][nt], 0, 0, 0);
          acc1[m][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, ch[nt], acc1[m][nt], 0, 0, 0);
          acc1[m][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, ch[nt], acc1[m][nt], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the scheduler's LDS-read hoisting within a k-step
    }
  }
  RB_MARK(3);
  __syncthreads();   // every wave is done with the input halo: its LDS now takes t1
  RB_MARK(4);

  // ---- t1 -> LDS: BN2(acc + b1) + ELU; rows outside the image are the (4,1) conv's zero padding ----
  // BN2(v + b1) = acc * (2^-12 s2) + (b1 s2 + t2): one v_pk_fma_f32 per pixel pair
  {
    _Float16* const thb = smem + wm * MT1 * TW * TPS + 4 * grp * TPS;   // + (m * TW + i) * TPS + n
    _Float16* const tlb = thb + G::TLO;
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      const int n = (wn * NTW + nt) * 16 + col;
      const float s2 = ps2[nt];
      const float c2 = fmaf(pb1[nt], s2, pt2[nt]);
      const f32x2 s2v = {s2 * a.u1, s2 * a.u1}, c2v = {c2, c2};
#pragma unroll
      for (int m = 0; m < MT1; ++m) {
        const int ih = h0 - 1 + wm * MT1 + m;   // scalar
        // branch-free (a branch per row serialises the 2 x MT1 x NTW independent chains)
        const float rm = (ih >= 0 && ih < a.h) ? 1.0f : 0.0f;
        const f32x2 rmask = {rm, rm};
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const f32x2 x1 = {acc1[m][nt][i], acc1[m][nt][i + 1]};
          const f32x2 u = elu2(x1 * s2v + c2v);
          // guard only the live t1 rows: the padding rows (>= TR, and outside the image) hold
          // whatever GEMM 1 made of unstaged LDS and are multiplied by 0 / never read
          rbad |= rm != 0.0f && wm * MT1 + m < G::TR && !in_f16_range(u, u);
          const f32x2 v = u * rmask;
          f16x2 hv, lv;
          split2(v, hv, lv);
          thb[(m * TW + i) * TPS + n] = hv.x;
          tlb[(m * TW + i) * TPS + n] = lv.x;
          thb[(m * TW + i + 1) * TPS + n] = hv.y;
          tlb[(m * TW + i + 1) * TPS + n] = lv.y;
        }
      }
    }
  }
  __syncthreads();

  RB_MARK(5);
  // ---- GEMM 2: output rows [wm * MT2, +MT2), K = (dy, ci) over t1 rows r + dy --------------------
  f32x4 d1[MT2][NTW];
#pragma unroll
  for (int m = 0; m < MT2; ++m)
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) d1[m][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    const _Float16* ahb = smem + (wm * MT2 * TW + col) * TPS;
    const _Float16* alb = ahb + G::TLO;
    const int b2o = ((wn * NTW) * 16 + col) * G::LW2 + 8 * grp;
    // !W2LDS: GEMM 2's B from L2 in fragment order (resblk_split_weights, frag), one k-step ahead
    const int b2g = (wn * NTW) * 512 + lane * 8;   // + nt * 512 + s * (C / 16) * 512
    const __amdgpu_buffer_rsrc_t rw2h = rb_rsrc(a.w2h), rw2l = rb_rsrc(a.w2l);
    f16x8 ph[NTW], pl[NTW];
    if constexpr (!G::W2LDS) {
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        ph[nt] = rb_frag(a.w2h, rw2h, nt * 512, b2g);
        pl[nt] = rb_frag(a.w2l, rw2l, nt * 512, b2g);
      }
    }
#pragma unroll
    for (int s = 0; s < KS2; ++s) {
      const int kk = 32 * s + 8 * grp;
      const int dy = kk / C, ci = kk - (kk / C) * C;
      const int koff = dy * TW * TPS + ci;
      f16x8 gh[NTW], gl[NTW];
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        if constexpr (G::W2LDS) {
          gh[nt] = *reinterpret_cast<const f16x8*>(s_w2h + b2o + nt * 16 * G::LW2 + 32 * s);
          gl[nt] = *reinterpret_cast<const f16x8*>(s_w2l + b2o + nt * 16 * G::LW2 + 32 * s);
        } else {
          gh[nt] = ph[nt];
          gl[nt] = pl[nt];
          if (s + 1 < KS2) {
            ph[nt] = rb_frag(a.w2h, rw2h, nt * 512 + (s + 1) * (C / 16) * 512, b2g);
            pl[nt] = rb_frag(a.w2l, rw2l, nt * 512 + (s + 1) * (C / 16) * 512, b2g);
          }
        }
      }
#pragma unroll
      for (int m = 0; m < MT2; ++m) {
        const f16x8 ah = *reinterpret_cast<const f16x8*>(ahb + koff + m * TW * TPS);
        const f16x8 al = *reinterpret_cast<const f16x8*>(alb + koff + m * TW * TPS);
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          d1[m][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, gl[nt], d1[m][nt], 0, 0, 0);
          d1[m][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, gh[nt], d1[m][nt], 0, 0, 0);
          d1[m][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, gh[nt], d1[m][nt], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  RB_MARK(6);
  // ---- epilogue through LDS: the tile's outputs go to LDS as f32 [pixel][C + 4] (the 4-dword pad
  //      puts the four lane groups of a ds_write_b32 on distinct banks), then every thread writes
  //      whole 16-B channel quads of consecutive pixels: 2 (pool) / 8 fully coalesced dwordx4 stores
  //      per thread instead of 8 / 32 dword stores per lane (and, non-pool, no residual loads: the
  //      residual is the raw halo interior this thread staged, still in pre[]) --------------------
  constexpr int OPS = C + 4;
  float* const so = reinterpret_cast<float*>(smem);
  static_assert(TH * TW * OPS * 2 <= G::SM, "the output tile fits the halo / t1 bytes");
  const bool interior = h0 + TH <= a.h && w0 + TW <= a.w;   // scalar: no per-element bounds checks
  __syncthreads();   // every wave is done reading t1 (GEMM 2)
  if constexpr (POOL) {
    constexpr int MSC = MT2 / 4;
    constexpr int PW = TW / 2;                                   // pooled tile: PW x PW pixels
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      const int n = (wn * NTW + nt) * 16 + col;
      const float b = pbo[nt];
#pragma unroll
      for (int j = 0; j < MSC; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = 4 * j + 2 * (i >> 1);        // t2 row pair (m, m + 1) of this wave
          const int e = 2 * (i & 1);                  // column pair (e, e + 1) of the lane's 4
          const int oh = h0 + wm * MT2 + m, ow = w0 + 4 * grp + e;   // even
          float mx = d1[m][nt][e] * a.u2;
          float v01 = d1[m][nt][e + 1] * a.u2;
          float v10 = d1[m + 1][nt][e] * a.u2;
          float v11 = d1[m + 1][nt][e + 1] * a.u2;
          if (!interior) {   // MaxPool2D 'same' on odd sizes: the window is cut at the edge
            if (oh >= a.h || ow >= a.w) continue;
            if (ow + 1 >= a.w) { v01 = mx; v11 = v10; }
            if (oh + 1 >= a.h) { v10 = mx; v11 = v01; }
          }
          mx = fmaxf(fmaxf(mx, v01), fmaxf(v10, v11));
          const float sc = e1[j][nt][i] * a.us;
          so[(((wm * MT2 + m) >> 1) * PW + ((4 * grp + e) >> 1)) * OPS + n] = mx + sc + b;
        }
    }
    __syncthreads();
    const int hp = (a.h + 1) >> 1, wp = (a.w + 1) >> 1;
    constexpr int QO = C / 4;                                    // float4 per output pixel
#pragma unroll
    for (int k = 0; k < (PW * PW * QO + NT - 1) / NT; ++k) {
      const int idx = tid + k * NT;
      if (idx >= PW * PW * QO) continue;
      const int p = idx / QO, qq = idx - (idx / QO) * QO;
      const int ph = (h0 >> 1) + p / PW, pw = (w0 >> 1) + p % PW;
      if (!interior && (ph >= hp || pw >= wp)) continue;
      *reinterpret_cast<float4*>(a.y + (((int64_t)clip * hp + ph) * wp + pw) * C + 4 * qq) =
          *reinterpret_cast<const float4*>(so + p * OPS + 4 * qq);
    }
  } else {
    static_assert(CIN == C, "the residual is the block input");
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      const int n = (wn * NTW + nt) * 16 + col;
      const float b = pbo[nt];
#pragma unroll
      for (int m = 0; m < MT2; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          so[((wm * MT2 + m) * TW + 4 * grp + i) * OPS + n] = fmaf(d1[m][nt][i], a.u2, b);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
      const int px = (tid + j * NT) / QPP;
      if (px >= G::XNP) continue;
      const int py = px / XC, pxx = px - (px / XC) * XC;
      const int r = py - 2, c = pxx - 1;                         // the halo pixel's output pixel
      if (r < 0 || r >= TH || c < 0 || c >= TW) continue;
      const int oh = h0 + r, ow = w0 + c;
      if (!interior && (oh >= a.h || ow >= a.w)) continue;
      const float4 v = *reinterpret_cast<const float4*>(so + (r * TW + c) * OPS + 4 * q);
      const float4 x = pre[j];
      *reinterpret_cast<float4*>(a.y + (((int64_t)clip * a.h + oh) * a.w + ow) * C + 4 * q) =
          make_float4(v.x + x.x, v.y + x.y, v.z + x.z, v.w + x.w);
    }
  }
  RB_MARK(7);
  if (rbad && a.range_flag) *a.range_flag = 1;
}

template <int CIN, int C, bool POOL, bool STEM = false>
hipError_t launch(const ResBlkArgs& a, hipStream_t s) {
  const int total = a.n * a.tiles_h * a.tiles_w;
  hipLaunchKernelGGL((resblk_kernel<CIN, C, POOL, STEM>), dim3(total), dim3(NT), 0, s, a);
  return hipGetLastError();
}

}  // namespace


int resblk_k1pad(int cin) { return (9 * cin + 31) / 32 * 32; }

bool resblk_supported(int cin, int c, bool pool) {
  return c == 32 && ((cin == 16 && pool) || (cin == 32 && !pool));
}

hipError_t resblk_launch(ResBlkArgs a, int cin, int c, bool pool, hipStream_t s) {
  if ((int64_t)a.n * a.h * a.w == 0) return hipSuccess;
  if (!resblk_supported(cin, c, pool)) return hipErrorInvalidValue;
  const int th = pool ? TH : TH_NP;
  a.tiles_h = (a.h + th - 1) / th;
  a.tiles_w = (a.w + TW - 1) / TW;
  if ((int64_t)a.n * a.tiles_h * a.tiles_w > 0x7fffffffLL) return hipErrorInvalidValue;
  if (cin == 16) {
    if (a.img8 || a.imgf) return launch<16, 32, true, true>(a, s);
    return launch<16, 32, true>(a, s);
  }
  return launch<32, 32, false>(a, s);
}

static uint16_t f16_bits(float f) {
  _Float16 h = (_Float16)f;
  uint16_t b;
  memcpy(&b, &h, 2);
  return b;
}

void resblk_split_weights(const float* w, int taps, int cin, int cout, int kpad, uint16_t* hi,
                          uint16_t* lo, bool frag, float wscale) {
  for (size_t i = 0; i < (size_t)cout * kpad; ++i) hi[i] = lo[i] = 0;
  for (int t = 0; t < taps; ++t)
    for (int ci = 0; ci < cin; ++ci)
      for (int co = 0; co < cout; ++co) {
        const float v = w[((size_t)t * cin + ci) * cout + co] * wscale;   // exact (power of two)
        const _Float16 h = (_Float16)v;
        const size_t k = (size_t)t * cin + ci;
        // frag: [k / 32][co / 16][lane = co % 16 + 16 (k % 32 / 8)][k % 8] (GEMM 1's B fragments)
        const size_t o = frag ? (((k / 32) * (cout / 16) + co / 16) * 64 + co % 16 + 16 * ((k % 32) / 8)) * 8 + k % 8
                              : (size_t)co * kpad + k;
        hi[o] = f16_bits(v);
        lo[o] = f16_bits(v - (float)h);
      }
}
