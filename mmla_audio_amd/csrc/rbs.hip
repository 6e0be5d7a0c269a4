// OD-NET res_blocks 1-3 (overlap_detector_temp.py:253-277) as rolling column strips on gfx950
// 32x32x16 f16 MFMA, 3xFP16 products:
//
//   t1 = Conv2D(32, 3x3, same)(ELU(BN1(x)))                GEMM 1, K = 9 * CIN
//   t2 = Conv2D(32, (4,1), same)(ELU(BN2(t1)))             GEMM 2, K = 4 * 32
//   y  = x + t2                          (blocks 2-3: 64 x 76 x 32)
//   y  = MaxPool2D(2, same)(t2) + Conv2D(32, 1x1, stride 2)(x)
//                                        (block 1, whose x is the stem Conv2D(16, 1x1) of the image,
//                                         computed while staging: 128 x 151 x 3 -> 64 x 76 x 32)
//
// One workgroup (4 waves) owns a 16-column strip of one clip and walks down it in chunks of R = 8
// output rows.  The conv(4,1) is vertical and the 3x3 reaches one row up and down, so a chunk needs
// only R new input rows and R new t1 rows: the rows it shares with the previous chunk stay in two
// LDS rings (x: R + 2 rows of the 18-column halo, t1: R + 3 rows), so no t1 row is computed twice
// and the input is staged 18/16 times instead of the 21 x 18 / 16 x 16 of a 16 x 16 tile.  Per
// chunk: stage the R new x rows (BN1 + ELU + the 2^4 scale + fp16 hi / lo split, from registers
// loaded during the previous chunk) -> barrier -> GEMM 1 (wave w: t1 rows 2w, 2w + 1 of the chunk =
// one 32-pixel tile, as t1^T = W1^T X^T so a lane holds 4-channel quads of one pixel) -> BN2 + ELU
// + split into the t1 ring as 8-byte channel quads -> barrier -> GEMM 2 (wave w: output rows 2w,
// 2w + 1) -> epilogue straight from the accumulators:
//   * blocks 2-3: y^T again (a lane: 16 channels of one pixel), + bias + the raw residual (float4
//     loads issued under GEMM 2's last k-steps);
//   * block 1: y in pixel rows ordered so that a lane's register quad IS one 2x2 pool window;
//     max-pool in registers, + the 1x1 / 2 shortcut as a 3xFP16 MFMA whose A rows are the windows'
//     top-left stem pixels (replicated 4x so its accumulator layout equals the pooled one).
// 32x32x16 MFMAs hold the SIMD's issue port for 8 of their 32 cycles (16x16x32: 8 of 16), which
// leaves the staging / t1 VALU work room beside the matrix pipe.
//
// LDS (hi and lo planes): 16-B channel groups of a pixel XOR-swizzled by column (and, for block 1's
// t1 read in pool-window order, by row parity), rows padded to a multiple of 256 B, so every
// ds_read_b128 of the GEMMs is conflict-free (model: the MI355X guide's lane groups).  Blocks 2-3:
// 47 KB -> three workgroups per CU; block 1: 38 KB -> four.
//
// 3xFP16 as conv_h3.hip: activations x 2^4 and weights x their power-of-two scale split into hi + lo,
// ONE f32 accumulator per tile (hi*lo + lo*hi + hi*hi); the 2^4 is folded into the BN coefficients
// (exact power-of-two scaling), ELU(u) * 16 = u16 > 0 ? u16 : 16 exp(u) - 16.
#include "common.h"
#include "resblk.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 256;            // 4 waves
constexpr int TW = 16;             // strip width (output columns)
constexpr int R = 8;               // output rows per chunk (4 waves x 2 rows)
constexpr int C = 32;              // output channels of blocks 1-3
constexpr float SPLIT_MAX = 65504.0f;                    // largest finite fp16
#ifndef RBS_TRACE
#define RBS_TRACE 0
#endif
#if RBS_TRACE
// dev timeline (RBS_TRACE builds only): s_memtime at 8 phase points of chunks 2..5, waves 0-3, of the
// first 2048 workgroups of each launch (the last launch wins)
__device__ unsigned long long rbs_trace_buf[2048 * 4 * 4 * 8];
#define RBS_T(i) do { if (bid < 2048 && k >= 2 && k < 6) tt[i] = __builtin_amdgcn_s_memtime(); } while (0)
#define RBS_TFLUSH() do { if (bid < 2048 && k >= 2 && k < 6 && lane == 0) { for (int i_ = 0; i_ < 8; ++i_) rbs_trace_buf[(((size_t)bid * 4 + wave) * 4 + (k - 2)) * 8 + i_] = tt[i_]; } } while (0)
#else
#define RBS_T(i) do { } while (0)
#define RBS_TFLUSH() do { } while (0)
#endif

MMLA_DEV __amdgpu_buffer_rsrc_t rbs_rsrc(const void* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)0x7fffffff, 0x00020000);
}
// 16 B of a split weight (conv_h3_split_weights order): wave-uniform half index u + this lane's lofs
MMLA_DEV f16x8 rbs_frag(__amdgpu_buffer_rsrc_t r, int u, int lofs) {
  return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)lofs * 2u, u * 2, 0));
}

// v' (already x 2^4) = hi + lo, both fp16 (RNE); lo = f16(v' - hi) exactly rounded once (v_fma_mix)
MMLA_DEV void split4(float a, float b, float c, float d, f16x4& h, f16x4& l) {
  h[0] = (_Float16)a;
  h[1] = (_Float16)b;
  h[2] = (_Float16)c;
  h[3] = (_Float16)d;
  const uint2 hu = __builtin_bit_cast(uint2, h);
  l = __builtin_bit_cast(f16x4, make_uint2(split_lo2(a, b, hu.x), split_lo2(c, d, hu.y)));
}

MMLA_DEV float amax4(float a, float b, float c, float d) {
  return fmaxf(fmaxf(fabsf(a), fabsf(b)), fmaxf(fabsf(c), fabsf(d)));
}

template <int H, int W, int CIN, bool POOL>
struct SG {
  static constexpr int XW = TW + 2;                     // halo columns w0 - 1 .. w0 + 16
  static constexpr int XRING = R + 2, TRING = R + 3;    // ring rows
  static constexpr int XROW = XW * CIN;                 // halfs per x ring row: 1152 / 576 B
  static constexpr int XPLANE = XRING * XROW;
  static constexpr int TROW = TW * C;                   // 512 halfs = 1024 B
  static constexpr int TPLANE = TRING * TROW;
  static constexpr int NCHUNK = H / R;
  static constexpr int STRIPS = (W + TW - 1) / TW;
  static constexpr int QPP = CIN / 4;                   // channel quads per pixel
  static constexpr int MAXT = (R * XW * QPP + NT - 1) / NT;      // staging tasks per thread, chunk
  static constexpr int MAXT0 = (4 * XW * QPP + NT - 1) / NT;     // the prologue's 4 rows
  static constexpr int KPT = CIN / 16;                  // 16-deep k-steps per tap
  static constexpr int KS1 = 9 * KPT, KS2 = 8;
  // block 1 keeps GEMM 2's weights in LDS to fit 3 workgroups per CU; blocks 2-3 keep them in
  // registers at 2 (measured: deeper weight prefetch or LDS-resident GEMM 1 weights do not pay)
  static constexpr bool W2L = CIN == 16;                // GEMM 2's weights in LDS
  static constexpr int MINB = CIN == 16 ? 3 : 2;        // resident workgroups per CU
  static constexpr int PF = 3;                          // GEMM 1 weight k-steps in flight
  static constexpr int PD = CIN == 16 ? 1 : 2;                      // input prefetch distance (chunks)
  static_assert(H % R == 0, "geometry");
  static_assert(NT % QPP == 0, "a thread's channel quad is fixed");
  static_assert(XROW <= 1024 && W * CIN * 4 < 65536 && W * 12 < 65536, "staging task fields");
};

// the x ring: pixel (row r, halo column x), 16-B channel group g -> half offset in a plane
// (rows unpadded: 72 / 36 16-B units; the swizzle keeps GEMM 1's ds_read_b128 conflict-free for
// every tap, both lane halves and either row parity -- searched against the guide's lane groups)
template <int CIN>
MMLA_DEV int xoff(int slot, int x, int g) {
  constexpr int XROW = (TW + 2) * CIN;
  const int f = CIN == 32 ? ((x >> 1) & 3) : ((x >> 1) & 1);
  return slot * XROW + x * CIN + 8 * (g ^ f);
}
// the t1 ring: pixel (row j, column c), channel group g (4 per pixel)
template <bool POOL>
MMLA_DEV int toff(int slot, int j, int c, int g) {
  const int f = POOL ? (((c >> 2) ^ (2 * (j & 1))) & 3) : ((c >> 2) & 3);
  return slot * (TW * C) + c * C + 8 * (g ^ f);
}

template <int H, int W, int CIN, bool POOL, bool STEM>
__global__ void __launch_bounds__(NT, (SG<H, W, CIN, POOL>::MINB)) rbs_kernel(ResBlkArgs a) {
  using G = SG<H, W, CIN, POOL>;
  static_assert(!STEM || (CIN == 16 && POOL), "the stem feeds block 1");
  static_assert(POOL || CIN == C, "residual blocks keep their width");
  __shared__ __attribute__((aligned(16))) _Float16 sx[2 * G::XPLANE];   // x ring: hi plane, lo plane
  __shared__ __attribute__((aligned(16))) _Float16 st[2 * G::TPLANE];   // t1 ring: hi plane, lo plane
  // per-channel parameters: [0] 16 s2 u1, [1] 16 (b1 s2 + t2), [2] b2 (+ stem {w_r, w_g, w_b, b} rows)
  __shared__ float4 spar[3 * C / 4 + (STEM ? 16 : 0)];
  // GEMM 2's weights in fragment order (W2L): [k-step][lane][8] hi, then lo
  __shared__ __attribute__((aligned(16))) _Float16 sw2[G::W2L ? 2 * G::KS2 * 512 : 8];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;                       // lane half: k group / channel group
  const uint32_t bid = xcd_block_id();
  const int clip = (int)(bid / G::STRIPS);
  const int w0 = (int)(bid - (uint32_t)clip * G::STRIPS) * TW;
  const int lofs = lane * 8;
  float rmax = 0.0f;   // 3xFP16 range guard: the largest |operand| this thread split (ResBlkArgs::range_flag)

  // ---- parameters -------------------------------------------------------------------------------
  float* const sp = reinterpret_cast<float*>(spar);
  if (tid < C) {
    const float s2 = a.s2[tid];
    sp[tid] = 16.0f * (s2 * a.u1);
    sp[C + tid] = 16.0f * fmaf(a.b1[tid], s2, a.t2[tid]);
    sp[2 * C + tid] = a.b2[tid];
  }
  if constexpr (STEM) {
    if (tid < 64) {   // [co][k]: k < 3 the r, g, b weights, k = 3 the bias (od_stem_kernel's operands)
      const int co = tid >> 2, k = tid & 3;
      sp[3 * C + tid] = k < 3 ? a.wst[k * a.ldst + co] : a.bst[co];
    }
  }
  // GEMM 2's weights (8 k-steps, hi / lo) stay in registers for the whole strip: GEMM 2 then issues no
  // vector loads, so the next chunk's input loads can be in flight across it (vector loads complete
  // in issue order: a weight load behind them would wait for HBM)
  const __amdgpu_buffer_rsrc_t rw1h = rbs_rsrc(a.w1h), rw1l = rbs_rsrc(a.w1l);
  f16x8 w2h[G::W2L ? 1 : G::KS2], w2l[G::W2L ? 1 : G::KS2];
  if constexpr (G::W2L) {
    for (int e = tid; e < 2 * G::KS2 * 64; e += NT) {   // 16-B pieces
      const int pl = e / (G::KS2 * 64), i = e - pl * (G::KS2 * 64);
      *reinterpret_cast<f16x8*>(sw2 + 8 * e) = *reinterpret_cast<const f16x8*>((pl ? a.w2l : a.w2h) + 8 * i);
    }
  } else {
    const __amdgpu_buffer_rsrc_t rw2h = rbs_rsrc(a.w2h), rw2l = rbs_rsrc(a.w2l);
#pragma unroll
    for (int s = 0; s < G::KS2; ++s) {
      w2h[s] = rbs_frag(rw2h, s * 512, lofs);
      w2l[s] = rbs_frag(rw2l, s * 512, lofs);
    }
  }
  f16x8 wsh_, wsl_;   // block 1's shortcut weights
  if constexpr (POOL) {
    wsh_ = rbs_frag(rbs_rsrc(a.wsh), 0, lofs);
    wsl_ = rbs_frag(rbs_rsrc(a.wsl), 0, lofs);
  }
  // this thread's staging quad: BN1 x 2^4 (exact); block 1: folded into the stem weights
  const int q = tid % G::QPP;
  float bnw[4][4];   // blocks 2-3: [c] = {16 s1, 16 t1}; block 1: [c] = 16 s1 {w_r, w_g, w_b} , 16 (s1 b + t1)
  __syncthreads();   // spar
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float s16 = 16.0f * a.s1[4 * q + c], t16 = 16.0f * a.t1[4 * q + c];
    if constexpr (STEM) {
      const float4 v = spar[3 * C / 4 + 4 * q + c];
      bnw[c][0] = s16 * v.x;
      bnw[c][1] = s16 * v.y;
      bnw[c][2] = s16 * v.z;
      bnw[c][3] = fmaf(s16, v.w, t16);
    } else {
      bnw[c][0] = s16;
      bnw[c][1] = t16;
    }
  }

  // ---- staging: task j of this thread = (pixel, quad) of the chunk's R x 18 new halo pixels --------
  // source: a per-clip buffer, so rows / columns outside the image read zeros with no branches
  // (offsets past the clip or negative, wrapped, are out of range)
  constexpr uint32_t ROWB = STEM ? 0u : (uint32_t)W * CIN * 4;
  const __amdgpu_buffer_rsrc_t rx = STEM ? rbs_rsrc(nullptr) :
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x) + (int64_t)clip * H * W * CIN, (short)0,
                                        (int)(H * ROWB), 0x00020000);
  // block 1: the clip's image (u8 or float NHWC) through a buffer descriptor as well
  const bool im8 = STEM && a.img8 != nullptr;
  const __amdgpu_buffer_rsrc_t rimg = !STEM ? rbs_rsrc(nullptr) :
      __builtin_amdgcn_make_buffer_rsrc(im8 ? (void*)(a.img8 + (int64_t)clip * H * W * 3)
                                            : (void*)(a.imgf + (int64_t)clip * H * W * 3),
                                        (short)0, (int)(H * W * 3 * (im8 ? 1 : 4)), 0x00020000);
  // per task: LDS column offset (bits 0-9), tile row (10-13), column inside the image (14), task exists
  // (15), its source byte offset within a row (16-31)
  uint32_t tinfo[G::MAXT];
#pragma unroll
  for (int j = 0; j < G::MAXT; ++j) {
    const int t = tid + j * NT;
    const int px = t / G::QPP;
    const int rr = px / G::XW, x = px - rr * G::XW;
    const int iw = w0 - 1 + x;
    const bool col_ok = iw >= 0 && iw < W;
    const uint32_t tc = !col_ok ? 0u : STEM ? (uint32_t)iw * (a.img8 ? 3u : 12u) : (uint32_t)(iw * CIN + 4 * q) * 4u;
    tinfo[j] = (uint32_t)(xoff<CIN>(0, x, q >> 1) + 4 * (q & 1)) | ((uint32_t)(rr & 15) << 10) |
               ((uint32_t)col_ok << 14) | ((uint32_t)(rr < R) << 15) | (tc << 16);
  }
  // the image pixel {r, g, b, 1} (1: inside the image), or x channels 4q .. 4q+3
  // (no branch around a load: a load inside a divergent branch is waited for inside it; the raw image
  // bytes are converted where they are used)
  auto load_src = [&](int ih, int iw, bool col_ok) -> float4 {
    if constexpr (STEM) {
      const int pix = ih * W + iw;
      const bool ok = col_ok && ih >= 0 && ih < H;
      if (im8) {
        const uint32_t off = ok ? (uint32_t)pix * 3u : 0x80000000u;
        const uint32_t r = __builtin_amdgcn_raw_buffer_load_b8(rimg, off, 0, 0);
        const uint32_t g = __builtin_amdgcn_raw_buffer_load_b8(rimg, off + 1u, 0, 0);
        const uint32_t b = __builtin_amdgcn_raw_buffer_load_b8(rimg, off + 2u, 0, 0);
        return make_float4(__builtin_bit_cast(float, r), __builtin_bit_cast(float, g), __builtin_bit_cast(float, b), 0.f);
      }
      const uint32_t off = ok ? (uint32_t)pix * 12u : 0x80000000u;
      return make_float4(__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rimg, off, 0, 0)),
                         __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rimg, off + 4u, 0, 0)),
                         __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rimg, off + 8u, 0, 0)), 0.f);
    } else {
      const uint32_t off = col_ok ? (uint32_t)ih * ROWB + (uint32_t)(iw * CIN + 4 * q) * 4u : 0x80000000u;
      return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
    }
  };
  // a loaded image pixel as floats
  auto img_px = [&](float4 v) -> float4 {
    if (im8)
      return make_float4((float)__builtin_bit_cast(uint32_t, v.x), (float)__builtin_bit_cast(uint32_t, v.y),
                         (float)__builtin_bit_cast(uint32_t, v.z), 0.f);
    return v;
  };
  // task j's 4 channels at x row r0 + its tile row (rows outside the image: the wrapped or past-the-end
  // row offset is out of range, as in load_src)
  auto load_task = [&](int r0, int j) -> float4 {
    const uint32_t ti = tinfo[j];
    const uint32_t off = (ti >> 14) & 1u ? (uint32_t)((r0 + (int)((ti >> 10) & 15)) * (STEM ? W * 3 * (im8 ? 1 : 4) : (int)ROWB)) + (ti >> 16)
                                         : 0x80000000u;
    if constexpr (STEM) {
      if (im8) {
        const uint32_t r = __builtin_amdgcn_raw_buffer_load_b8(rimg, off, 0, 0);
        const uint32_t g = __builtin_amdgcn_raw_buffer_load_b8(rimg, off + 1u, 0, 0);
        const uint32_t b = __builtin_amdgcn_raw_buffer_load_b8(rimg, off + 2u, 0, 0);
        return make_float4(__builtin_bit_cast(float, r), __builtin_bit_cast(float, g), __builtin_bit_cast(float, b), 0.f);
      }
      return make_float4(__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rimg, off, 0, 0)),
                         __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rimg, off + 4u, 0, 0)),
                         __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rimg, off + 8u, 0, 0)), 0.f);
    } else {
      return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
    }
  };
  // BN1 + ELU (+ the stem) + split of one task's 4 channels at x row ih, into the x ring at lds
  // BN1 + ELU (+ the stem) + split of one task's 4 channels into the x ring at half offset o; MASK:
  // zero unless `in` (the 3x3 conv's padding rows; padding columns are zeroed once, see below)
  auto stage4 = [&](int o, bool in, float4 v, auto MASK_) {
    constexpr bool MASK = decltype(MASK_)::value;
    if constexpr (STEM) v = img_px(v);
    float u[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if constexpr (STEM) {   // 16 BN1(stem(x)) with the BN folded into the stem weights
        float acc = v.x * bnw[c][0];
        acc = fmaf(v.y, bnw[c][1], acc);
        acc = fmaf(v.z, bnw[c][2], acc);
        u[c] = acc + bnw[c][3];
      } else {
        u[c] = fmaf((&v.x)[c], bnw[c][0], bnw[c][1]);
      }
    }
    float e[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) e[c] = (!MASK || in) ? elu16(u[c]) : 0.0f;
    rmax = fmaxf(rmax, amax4(e[0], e[1], e[2], e[3]));
    f16x4 hv, lv;
    split4(e[0], e[1], e[2], e[3], hv, lv);
    *reinterpret_cast<f16x4*>(sx + o) = hv;
    *reinterpret_cast<f16x4*>(sx + G::XPLANE + o) = lv;
  };
  // a chunk's task j: rows r0 .. r0 + 7; tasks on a column outside the image do nothing (their ring
  // column stays zero); rows past the image only occur in the last chunk (MASK)
  auto stage_task = [&](int r0, int j, float4 v, auto MASK_) {
    const uint32_t ti = tinfo[j];
    if (((ti >> 14) & 3u) != 3u) return;   // task exists and its column is inside the image
    const int rr = (int)((ti >> 10) & 15);
    uint32_t slot = (uint32_t)((r0 + 1) % G::XRING) + (uint32_t)rr;   // (r0 + 1) % XRING: scalar
    slot = min(slot, slot - (uint32_t)G::XRING);
    stage4((int)slot * G::XROW + (int)(ti & 1023), r0 + rr < H, v, MASK_);
  };
  // the ring's columns outside the image (strip 0: image column -1; the last strip: columns >= W),
  // zeroed once in every slot and both planes: no task writes them
  for (int e = tid; e < 2 * G::XRING * G::XW * G::QPP; e += NT) {
    const int pl = e / (G::XRING * G::XW * G::QPP), r = e - pl * (G::XRING * G::XW * G::QPP);
    const int slot = r / (G::XW * G::QPP), x = (r / G::QPP) % G::XW, qq = r % G::QPP;
    const int iw = w0 - 1 + x;
    if (iw < 0 || iw >= W)
      *reinterpret_cast<f16x4*>(sx + pl * G::XPLANE + xoff<CIN>(slot, x, qq >> 1) + 4 * (qq & 1)) = f16x4{};
  }
  // ---- GEMM 1 for t1 rows j0, j0 + 1 (one 32-pixel tile, natural order: pixel n = lane & 31 is row
  //      j0 + (n >> 4), column n & 15) as t1^T: acc[4 jj + i] = channel 8 jj + 4 h + i of pixel n ----
  const int n = lane & 31, nr = n >> 4, nc = n & 15;
  // this lane's x column offsets for dx = 0..2 and its k groups (ks)
  int xco[3][G::KPT];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx)
#pragma unroll
    for (int ks = 0; ks < G::KPT; ++ks) xco[dx][ks] = xoff<CIN>(0, nc + dx, G::KPT == 2 ? 2 * ks + h : h);

  f16x8 w1h[G::PF], w1l[G::PF];   // GEMM 1's weight ring (PF k-steps ahead), first steps issued early
  auto gemm1_issue = [&]() {
#pragma unroll
    for (int s = 0; s < G::PF; ++s) {
      w1h[s] = rbs_frag(rw1h, s * 512, lofs);
      w1l[s] = rbs_frag(rw1l, s * 512, lofs);
    }
  };
  auto gemm1 = [&](int j0) -> f32x16 {
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
    int xr[3];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {   // x row j - 1 + dy: ring slot (j0 % XRING: scalar) + nr + dy, wrapped
      const uint32_t sl = (uint32_t)(j0 % G::XRING) + (uint32_t)(nr + dy);
      xr[dy] = (int)min(sl, sl - (uint32_t)G::XRING) * G::XROW;
    }
    // the x fragments one k-step ahead (an LDS read's latency would otherwise sit before every
    // step's MFMAs)
    auto xo = [&](int s) {
      const int tap = s / G::KPT, ks = s % G::KPT;
      return xr[tap / 3] + xco[tap % 3][ks];
    };
    f16x8 nxh = *reinterpret_cast<const f16x8*>(sx + xo(0));
    f16x8 nxl = *reinterpret_cast<const f16x8*>(sx + G::XPLANE + xo(0));
#pragma unroll
    for (int s = 0; s < G::KS1; ++s) {
      const f16x8 bh = w1h[s % G::PF], bl = w1l[s % G::PF];
      if (s + G::PF < G::KS1) {
        w1h[s % G::PF] = rbs_frag(rw1h, (s + G::PF) * 512, lofs);
        w1l[s % G::PF] = rbs_frag(rw1l, (s + G::PF) * 512, lofs);
      }
      const f16x8 xh = nxh, xl = nxl;
      if (s + 1 < G::KS1) {
        nxh = *reinterpret_cast<const f16x8*>(sx + xo(s + 1));
        nxl = *reinterpret_cast<const f16x8*>(sx + G::XPLANE + xo(s + 1));
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bl, xh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh, xl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh, xh, acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);   // keep the register footprint: no deeper hoisting
    }
    return acc;
  };
  // BN2(acc u1 + b1) + ELU + split -> t1 ring rows j0 + nr; rows past the image are the (4,1) conv's
  // zero padding (j0 is even and so is H: both rows of a wave are inside or both outside)
  auto t1_write = [&](int j0, const f32x16& acc) {
    const int j = j0 + nr;
    const uint32_t sl = (uint32_t)((j0 + 1) % G::TRING) + (uint32_t)nr;   // (j + 1) % TRING
    const int slot = (int)min(sl, sl - (uint32_t)G::TRING);
    if (j0 < H) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int c0 = 8 * jj + 4 * h;
        const float4 sv = spar[c0 / 4], cv = spar[C / 4 + c0 / 4];
        float e[4];
        e[0] = elu16(fmaf(acc[4 * jj + 0], sv.x, cv.x));
        e[1] = elu16(fmaf(acc[4 * jj + 1], sv.y, cv.y));
        e[2] = elu16(fmaf(acc[4 * jj + 2], sv.z, cv.z));
        e[3] = elu16(fmaf(acc[4 * jj + 3], sv.w, cv.w));
        rmax = fmaxf(rmax, amax4(e[0], e[1], e[2], e[3]));
        f16x4 hv, lv;
        split4(e[0], e[1], e[2], e[3], hv, lv);
        const int o = toff<POOL>(slot, j, nc, jj) + 4 * h;
        *reinterpret_cast<f16x4*>(st + o) = hv;
        *reinterpret_cast<f16x4*>(st + G::TPLANE + o) = lv;
      }
    } else {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int o = toff<POOL>(slot, j, nc, jj) + 4 * h;
        *reinterpret_cast<f16x4*>(st + o) = f16x4{};
        *reinterpret_cast<f16x4*>(st + G::TPLANE + o) = f16x4{};
      }
    }
  };

  // ---- prologue: x rows -1 .. 2, t1 rows 0, 1 (wave 0) and the zero t1 row -1 --------------------
  {
    constexpr int T0 = 4 * G::XW * G::QPP;
#pragma unroll
    for (int j = 0; j < G::MAXT0; ++j) {
      const int t = tid + j * NT;
      const int px = t / G::QPP;
      const int rr = px / G::XW, x = px - rr * G::XW;
      const int ih = rr - 1, iw = w0 - 1 + x;
      const bool col_ok = iw >= 0 && iw < W;
      const float4 v = load_src(ih, iw, col_ok);
      if (t < T0 && col_ok)
        stage4(xoff<CIN>((ih + 1) % G::XRING, x, q >> 1) + 4 * (q & 1), ih >= 0, v, std::true_type{});
    }
    for (int e = tid; e < 2 * G::TROW / 8; e += NT)   // t1 row -1 (slot 0), both planes
      *reinterpret_cast<f16x8*>(st + (e >= G::TROW / 8 ? G::TPLANE - G::TROW : 0) + 8 * e) = f16x8{};
  }
  __syncthreads();
  if (wave == 0) {
    gemm1_issue();
    const f32x16 acc = gemm1(0);
    t1_write(0, acc);
  }
  // the new rows of chunk k, loaded G::PD chunks ahead (blocks 2-3: two, in preA for even k and preB
  // for odd k, so a whole chunk of work stands between a load and its use; block 1, whose register
  // budget is three workgroups per CU: one)
  float4 preA[G::MAXT], preB[G::PD == 2 ? G::MAXT : 1];
#pragma unroll
  for (int j = 0; j < G::MAXT; ++j) preA[j] = load_task(3, j);
  if constexpr (G::PD == 2) {
#pragma unroll
    for (int j = 0; j < G::MAXT; ++j) preB[j] = load_task(3 + R, j);
  }
  __syncthreads();   // wave 0 is done with x rows -1, 0 (the first chunk overwrites their slots)

  // block 1's shortcut pixel of a chunk: this lane's pool window's top-left, conv row 8 k + 2 wave
  const int win = n >> 2;
  const int sc_col = w0 + 2 * win;

#if RBS_TRACE
  unsigned long long tt[8];
#endif
  static_assert(G::NCHUNK % 2 == 0, "chunk pairs");
  auto chunk = [&](const int k, float4* pre) {
    RBS_T(0);
    const int rx0 = R * k + 3;            // the chunk's new x rows rx0 .. rx0 + 7
    const int j0 = R * k + 2 + 2 * wave;  // this wave's t1 rows (GEMM 1)
    const int o0 = R * k + 2 * wave;      // this wave's output rows (GEMM 2)
    // ---- stage the new x rows, start GEMM 1's weight stream ------------------------------------
    if (k + 1 < G::NCHUNK) {
#pragma unroll
      for (int j = 0; j < G::MAXT; ++j) stage_task(rx0, j, pre[j], std::false_type{});
    } else {
#pragma unroll
      for (int j = 0; j < G::MAXT; ++j) stage_task(rx0, j, pre[j], std::true_type{});
    }
    gemm1_issue();
    RBS_T(1);
    __syncthreads();
    RBS_T(2);
    // ---- GEMM 1 -> t1 ring ------------------------------------------------------------------------
    {
      const f32x16 acc = gemm1(j0);
      RBS_T(3);
      t1_write(j0, acc);
    }
    RBS_T(4);
    // ---- the epilogue's operands, then the next chunk's rows (issue order = completion order) -----
    const int pr = POOL ? (n & 3) >> 1 : nr;
    const int pc = POOL ? 2 * (n >> 2) + (n & 1) : nc;
    float4 rsd[POOL ? 1 : 4];
    float4 scpx = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (!POOL) {
      const uint32_t off = w0 + pc < W ? (uint32_t)(o0 + pr) * ROWB + (uint32_t)((w0 + pc) * C + 4 * h) * 4u : 0x80000000u;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        rsd[jj] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, jj * 32, 0));
    } else {
      scpx = load_src(o0, sc_col, sc_col < W);
    }
    if (k + G::PD < G::NCHUNK) {
#pragma unroll
      for (int j = 0; j < G::MAXT; ++j) pre[j] = load_task(rx0 + G::PD * R, j);
    }
    __syncthreads();
    RBS_T(5);
    // ---- GEMM 2 (weights in registers) -----------------------------------------------------------
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
    {
      int tr[4], tj[4];
#pragma unroll
      for (int dy = 0; dy < 4; ++dy) {
        tj[dy] = o0 + pr - 1 + dy;
        const uint32_t sl = (uint32_t)(o0 % G::TRING) + (uint32_t)(pr + dy);   // (tj + 1) % TRING
        tr[dy] = (int)min(sl, sl - (uint32_t)G::TRING);
      }
      auto to = [&](int s) { return toff<POOL>(tr[s >> 1], tj[s >> 1], pc, 2 * (s & 1) + h); };
      f16x8 nxh = *reinterpret_cast<const f16x8*>(st + to(0));
      f16x8 nxl = *reinterpret_cast<const f16x8*>(st + G::TPLANE + to(0));
      f16x8 ngh, ngl;
      if constexpr (G::W2L) {
        ngh = *reinterpret_cast<const f16x8*>(sw2 + lofs);
        ngl = *reinterpret_cast<const f16x8*>(sw2 + G::KS2 * 512 + lofs);
      }
#pragma unroll
      for (int s = 0; s < G::KS2; ++s) {
        const f16x8 xh = nxh, xl = nxl;
        f16x8 gh, gl;
        if constexpr (G::W2L) {
          gh = ngh;
          gl = ngl;
        } else {
          gh = w2h[s];
          gl = w2l[s];
        }
        if (s + 1 < G::KS2) {   // the next step's fragments under this step's MFMAs
          nxh = *reinterpret_cast<const f16x8*>(st + to(s + 1));
          nxl = *reinterpret_cast<const f16x8*>(st + G::TPLANE + to(s + 1));
          if constexpr (G::W2L) {
            ngh = *reinterpret_cast<const f16x8*>(sw2 + (s + 1) * 512 + lofs);
            ngl = *reinterpret_cast<const f16x8*>(sw2 + (G::KS2 + s + 1) * 512 + lofs);
          }
        }
        if constexpr (POOL) {   // y: pixel rows (a register quad = one 2x2 window), channel = lane
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, gl, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, gh, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, gh, acc, 0, 0, 0);
        } else {                // y^T: a register quad = 4 channels of this lane's pixel
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(gl, xh, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(gh, xl, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(gh, xh, acc, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    RBS_T(6);
    // ---- epilogue ---------------------------------------------------------------------------------
    if constexpr (!POOL) {
      const int ow = w0 + pc, oh = o0 + pr;
      if (ow < W) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int c0 = 8 * jj + 4 * h;
          const float4 b = spar[2 * C / 4 + c0 / 4];
          const float4 r = rsd[jj];
          const float4 v = make_float4(fmaf(acc[4 * jj + 0], a.u2, b.x) + r.x, fmaf(acc[4 * jj + 1], a.u2, b.y) + r.y,
                                       fmaf(acc[4 * jj + 2], a.u2, b.z) + r.z, fmaf(acc[4 * jj + 3], a.u2, b.w) + r.w);
          *reinterpret_cast<float4*>(a.y + (((int64_t)clip * H + oh) * W + ow) * C + c0) = v;
        }
      }
    } else {
      // the shortcut Conv2D(1x1, stride 2) of the raw stem output: A row m = window m >> 2 (x4),
      // k = stem channels 8 h .. 8 h + 7; accumulator register 4 jj + i then holds window 2 jj + h
      f32x16 sacc;
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[i] = 0.0f;
      {
        float o8[8];
        const float4 px = img_px(scpx);
#pragma unroll
        for (int c = 0; c < 8; ++c) {   // od_stem_kernel's order
          const float4 wv = spar[3 * C / 4 + 8 * h + c];
          float s = px.x * wv.x;
          s = fmaf(px.y, wv.y, s);
          s = fmaf(px.z, wv.z, s);
          o8[c] = sc_col < W ? 16.0f * (s + wv.w) : 0.0f;
        }
        rmax = fmaxf(rmax, fmaxf(amax4(o8[0], o8[1], o8[2], o8[3]), amax4(o8[4], o8[5], o8[6], o8[7])));
        f16x4 h0, l0, h1, l1;
        split4(o8[0], o8[1], o8[2], o8[3], h0, l0);
        split4(o8[4], o8[5], o8[6], o8[7], h1, l1);
        const f16x8 ah = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        const f16x8 al = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, wsl_, sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, wsh_, sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, wsh_, sacc, 0, 0, 0);
      }
      constexpr int HP = H / 2, WP = (W + 1) / 2;
      const int co = n;
      const float b2 = sp[2 * C + co], bs = a.bs[co];
      const int prow = (R / 2) * k + wave;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int wdw = 2 * jj + h;                  // window: conv columns w0 + 2 wdw, + 1
        const int cc = w0 + 2 * wdw;
        if (cc >= W) continue;
        float m0 = fmaf(acc[4 * jj + 0], a.u2, b2);  // (row 0, col 0)
        float m1 = fmaf(acc[4 * jj + 1], a.u2, b2);  // (row 0, col 1)
        float m2 = fmaf(acc[4 * jj + 2], a.u2, b2);  // (row 1, col 0)
        float m3 = fmaf(acc[4 * jj + 3], a.u2, b2);  // (row 1, col 1)
        if (cc + 1 >= W) {                           // MaxPool 'same' on the odd width: window cut
          m1 = m0;
          m3 = m2;
        }
        const float mx = fmaxf(fmaxf(m0, m1), fmaxf(m2, m3)) + fmaf(sacc[4 * jj], a.us, bs);
        a.y[(((int64_t)clip * HP + prow) * WP + (w0 >> 1) + wdw) * C + co] = mx;
      }
    }
    RBS_T(7);
    RBS_TFLUSH();
  };
  if constexpr (G::PD == 2) {
#pragma unroll 1
    for (int k = 0; k < G::NCHUNK; k += 2) {
      chunk(k, preA);
      chunk(k + 1, preB);
    }
  } else {
#pragma unroll 1
    for (int k = 0; k < G::NCHUNK; ++k) chunk(k, preA);
  }
  if (!(rmax < SPLIT_MAX) && a.range_flag) *a.range_flag = 1;
}

template <int H, int W, int CIN, bool POOL, bool STEM>
hipError_t launch(const ResBlkArgs& a, hipStream_t s) {
  using G = SG<H, W, CIN, POOL>;
  const int64_t blocks = (int64_t)a.n * G::STRIPS;
  if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
  hipLaunchKernelGGL((rbs_kernel<H, W, CIN, POOL, STEM>), dim3((unsigned)blocks), dim3(NT), 0, s, a);
  return hipGetLastError();
}

}  // namespace

#if RBS_TRACE
extern "C" int mmla_debug_rbs_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(rbs_trace_buf), sizeof(rbs_trace_buf)) == hipSuccess ? 0 : -2;
}
#endif

bool rbs_supported(int h, int w, int cin, int c, bool pool) {
  return c == 32 && ((h == 128 && w == 151 && cin == 16 && pool) || (h == 64 && w == 76 && cin == 32 && !pool));
}

hipError_t rbs_launch(const ResBlkArgs& a, int cin, int c, bool pool, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  if (!rbs_supported(a.h, a.w, cin, c, pool) || !a.y || !a.w1h || !a.w1l || !a.w2h || !a.w2l)
    return hipErrorInvalidValue;
  if (pool) {
    if (!a.wsh || !a.wsl || !a.bs) return hipErrorInvalidValue;
    if (a.img8 || a.imgf) return launch<128, 151, 16, true, true>(a, s);
    return hipErrorInvalidValue;   // block 1 runs with the stem fused
  }
  if (!a.x || a.x == a.y) return hipErrorInvalidValue;
  return launch<64, 76, 32, false, false>(a, s);
}
