// OverlapDetection res_block (overlap_detector_temp.py:253-277) of the 64- and 128-channel stages as
// ONE kernel per block (blocks 1-3 run fused in resblk.hip):
//     t1 = Conv3x3(ELU(BN_in(x)))                      (GEMM a, K = 9 * cin)
//     t2 = Conv(4,1)(ELU(BN_mid(t1)))                  (GEMM b, K = 4 * c)
//     y  = x + t2                                      (blocks 5-6, 8-9)
//     y  = MaxPool2D(2, 'same')(t2) + Conv1x1/2(x)     (blocks 4, 7)
// The two conv_h3 launches it replaces write t1 to HBM (float32) and read it back with a halo, and the
// second re-reads x for the residual / shortcut.  Here a workgroup owns a FULL-HEIGHT strip of TW output
// columns of one clip: the conv(4,1) is vertical, so the strip's t1 is exactly its own H x TW pixels
// (no recomputed rows; Keras 'same' pads t1 with one zero row above and two below), held in LDS as
// BN_mid + ELU'd fp16 hi / lo next to nothing else -- it overlays the x halo GEMM a has finished with.
//
// Per strip: x halo (H + 2) x (TW + 2) staged in 32-channel chunks (BN_in + ELU + 2^4 + split, as
// conv_h3's staging), GEMM a as C^T = W^T X^T (a lane's accumulator quad = 4 consecutive channels of
// one pixel, so t1 goes back to LDS as 8-byte channel quads), t1 staged, GEMM b, epilogue:
//   * residual blocks: C^T again, bias + the raw x residual as float4 loads / stores;
//   * pool blocks (TW = 2): pixel rows in the accumulator, so a lane's register quad IS one 2x2 pool
//     window (rows i, i + 1 x columns 0, 1), and the shortcut Conv2D(1x1, stride 2) is a small 3xFP16
//     GEMM whose accumulator register 4 mt + q holds the window of main register quad (mt, q) --
//     its A row is that window's top-left input pixel (conv_h3's fused-shortcut trick).
//
// Bit-identical to the conv_h3 pair: the same staged operands (values, 2^4 scale, split), the same MFMA
// sequence per output element (32-channel chunks, then taps, then 16-channel k-steps; hi*lo, lo*hi,
// hi*hi into one accumulator -- C^T computes each element from the same products), the same epilogue
// arithmetic (fmaf(acc, unscale, bias), then + residual / max-pool + shortcut).  env MMLA_NO_ODU=1 at
// mmla_create runs the pair instead (tests/test_gpu_odu.py checks every block both ways).
#include "common.h"
#include "conv.h"
#include "odu.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

constexpr int CK = 32;                 // channel chunk (conv_h3's k order)
constexpr int KS = CK / 16;            // MFMA k-steps per chunk
constexpr float ACT_SCALE = 16.0f;     // 2^4, as conv_h3
constexpr float SPLIT_MAX = 65504.0f;  // largest finite fp16 (operands are compared once scaled)

MMLA_DEV __amdgpu_buffer_rsrc_t odu_rsrc(const void* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)0x7fffffff, 0x00020000);
}
// 16 B of a split weight: wave-uniform half offset uoff + this lane's lofs
MMLA_DEV f16x8 odu_frag(__amdgpu_buffer_rsrc_t r, size_t uoff, int lofs) {
  return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)lofs * 2u, (int)(uoff * 2), 0));
}

// conv_h3's PRO_BN_ELU prologue x 2^4 (sc16, sh16 = 2^4 x the folded BatchNorm: exact)
MMLA_DEV float bn_elu16(float v, float sc16, float sh16) { return elu16(fmaf(v, sc16, sh16)); }
MMLA_DEV float4 x16(float4 v) { return make_float4(ACT_SCALE * v.x, ACT_SCALE * v.y, ACT_SCALE * v.z, ACT_SCALE * v.w); }

// v (already x 2^4) = hi + lo, both fp16
MMLA_DEV void split4(float4 v, f16x4& h, f16x4& l) {
  h[0] = (_Float16)v.x;
  h[1] = (_Float16)v.y;
  h[2] = (_Float16)v.z;
  h[3] = (_Float16)v.w;
  const uint2 hu = __builtin_bit_cast(uint2, h);
  l = __builtin_bit_cast(f16x4, make_uint2(split_lo2(v.x, v.y, hu.x), split_lo2(v.z, v.w, hu.y)));
}

// the running range maximum of split operands (ResBlkArgs / OduArgs::range_flag)
MMLA_DEV float amax4(float r, float4 v) {
  return fmaxf(r, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
}

// H x W image, CIN -> C channels, strips of TW columns, 4 waves: WN = C / 32 waves along the output
// channels (one 32-channel tile each, so no weight fragment is fetched twice per workgroup), WM along
// the strip's H * TW pixels, MT 32-pixel tiles per wave
template <int H, int W, int CIN, int C, int TW, bool POOL, int NW, int MINW>
__global__ void __launch_bounds__(64 * NW, MINW) odu_kernel(OduArgs a) {
  constexpr int NT = 64 * NW;
  constexpr int WN = C / 32, WM = NW / WN;
  constexpr int M = H * TW;
  constexpr int MT = M / (WM * 32);
  static_assert(MT * WM * 32 == M && WN * WM == NW, "tiling");
  static_assert(!POOL || (TW == 2 && H % 2 == 0 && W % 2 == 0 && MT <= 4), "pool strips");
  static_assert(POOL || CIN == C, "residual blocks keep their width");
  constexpr int TLW = (W + TW - 1) / TW;
  constexpr int XP = TW + 2, XH = H + 2, NXP = XH * XP;   // x halo: rows -1 .. H, columns -1 .. TW
  // x halo layout, chosen so GEMM a's 16-lane ds_read_b128 groups (8 rows x 2 columns at TW 2, 4 x 4
  // at TW 4) hit 64 distinct banks (tools: the guide's lane groups, MI355X_MICROARCH.md section LDS):
  //   TW 2: 64-B pixels (no pad), 288-B rows, the two 16-B halves of each 32-B k-step swapped in odd
  //         halo columns -- conflict-free reads AND staging stores at 38 KB for block 4's halo, so its
  //         LDS plane (t1, 38.6 KB) admits four workgroups per CU (42.2 KB with 80-B pixels: three);
  //   TW 4: 80-B pixels (16-B pad), 576-B rows instead of 480 (2-way conflicts), same plane size.
  constexpr int LDX = TW == 2 ? CK : CK + 8;              // fp16 per staged x pixel
  constexpr int XRP = TW == 2 ? 144 : TW == 4 ? 288 : XP * LDX;   // fp16 per halo row
  constexpr bool XSW = TW == 2;                           // odd-column half swap
  constexpr int T1R = H + 3, NT1 = T1R * TW;              // t1 rows -1 .. H + 1 (three zero rows)
  constexpr int LDT = C + 8;                              // fp16 per t1 pixel
  constexpr int NCHX = CIN / CK, NCH = C / CK;
  // DB: two halo buffers, so chunk ch + 1 is loaded and staged right behind chunk ch's MFMAs (which
  // run on in the matrix pipe) instead of after a barrier; only where the second buffer fits inside
  // the t1 plane the LDS already holds (blocks 7, 8-9; blocks 5-6 would drop to two workgroups per CU)
  constexpr bool DB = NCHX > 1 && C == 128;
  constexpr int XBUF = XH * XRP;                          // fp16 per halo buffer and plane
  constexpr int XTOT = DB ? 2 * XBUF : XBUF;
  constexpr int PLANE = XTOT > NT1 * LDT ? XTOT : NT1 * LDT;
  constexpr int QPP = CK / 4;                             // float4 per pixel and chunk
  constexpr int MAXT = (NXP * QPP + NT - 1) / NT;
  static_assert(NT % QPP == 0, "a thread's channel quad is fixed");
  __shared__ __attribute__((aligned(16))) _Float16 lhi[PLANE];
  __shared__ __attribute__((aligned(16))) _Float16 llo[PLANE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const uint32_t bid = xcd_block_id();
  const int64_t clip = bid / TLW;
  const int w0 = (int)(bid - clip * TLW) * TW;
  const float* __restrict__ xc = a.x + clip * ((int64_t)H * W * CIN);
  // the clip's input through a buffer descriptor: out-of-image halo pixels read zeros with no branch
  // around the load (a load inside a divergent branch is waited for inside it)
  const __amdgpu_buffer_rsrc_t rxc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xc), (short)0,
                                                                       (int)(H * W * CIN * 4), 0x00020000);
  const int koff = (lane >> 5) * 8;
  const int hsel = 4 * (lane >> 5);
  const int cob = wn * 32;                    // this wave's output-channel tile
  const int lofs = wn * 512 + lane * 8;       // its B fragment inside a (tap, k-step) 1 KB block
  constexpr size_t kstr = (size_t)(C / 32) * 512;
  float rmax = 0.0f;   // the largest |operand| this thread split (x 2^4)

  int mpix[MT];   // the wave's pixels (C^T columns / pixel rows): strip pixel m = i * TW + c
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) mpix[mt] = (wm * MT + mt) * 32 + (lane & 31);

  f32x16 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[mt][i] = 0.0f;

  // ---- GEMM a: t1^T = Wa^T X^T over the halo, chunk by chunk --------------------------------------
  {
    const __amdgpu_buffer_rsrc_t rh = odu_rsrc(a.wah), rl = odu_rsrc(a.wal);
    constexpr size_t tap_stride = (size_t)C * CIN;
    const int q = tid % QPP;
    // XSW: this lane's k-half offset in an even / odd halo column (m % TW = lane & 1 at TW 2)
    const int kx0 = XSW ? 8 * ((lane >> 5) ^ (lane & 1)) : koff;
    const int kx1 = XSW ? 8 * ((lane >> 5) ^ (lane & 1) ^ 1) : koff;
    // global loads of chunk ch's halo quads, then BN_in + ELU + 2^4 + split into halo buffer buf
    auto load_stage = [&](int ch, int buf) {
      const int ci = ch * CK + 4 * q;
      const float4 sc = x16(*reinterpret_cast<const float4*>(a.s_in + ci));
      const float4 sh = x16(*reinterpret_cast<const float4*>(a.t_in + ci));
      float4 pre[MAXT];
      uint32_t valid = 0;
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        const int task = tid + j * NT;
        const int px = task / QPP;
        const int ih = px / XP - 1, iw = w0 + px % XP - 1;
        const bool ok = task < NXP * QPP && ih >= 0 && ih < H && iw >= 0 && iw < W;
        pre[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                rxc, ok ? (uint32_t)((ih * W + iw) * CIN + ci) * 4u : 0x80000000u, 0, 0));
        valid |= (uint32_t)ok << j;
      }
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        const int task = tid + j * NT;
        if (task >= NXP * QPP) continue;
        float4 v = pre[j];
        if (valid & (1u << j)) {
          v.x = bn_elu16(v.x, sc.x, sh.x);
          v.y = bn_elu16(v.y, sc.y, sh.y);
          v.z = bn_elu16(v.z, sc.z, sh.z);
          v.w = bn_elu16(v.w, sc.w, sh.w);
        }
        rmax = amax4(rmax, v);
        f16x4 hv, lv;
        split4(v, hv, lv);
        const int px = task / QPP;
        const int cx = px % XP;
        const int xo = (px / XP) * XRP + cx * LDX + (XSW ? 8 * ((q >> 1) ^ (cx & 1)) + 4 * (q & 1) : 4 * q);
        *reinterpret_cast<f16x4*>(lhi + buf * XBUF + xo) = hv;
        *reinterpret_cast<f16x4*>(llo + buf * XBUF + xo) = lv;
      }
    };
    if constexpr (DB) {
      load_stage(0, 0);
      __syncthreads();
    }
#pragma unroll 1
    for (int ch = 0; ch < NCHX; ++ch) {
      const int buf = DB ? (ch & 1) : 0;
      // tap 0's B fragments, in flight across the staging
      f16x8 bh[KS], bl[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bh[s] = odu_frag(rh, (size_t)(ch * KS + s) * kstr, lofs);
        bl[s] = odu_frag(rl, (size_t)(ch * KS + s) * kstr, lofs);
      }
      if constexpr (!DB) {
        if (ch > 0) __syncthreads();   // every wave is done reading the previous chunk
        load_stage(ch, 0);
        __syncthreads();
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int dy = tap / 3, dx = tap - (tap / 3) * 3;
        f16x8 nbh[KS], nbl[KS];
        if (tap + 1 < 9) {   // the next tap's fragments under this tap's MFMAs
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const size_t u = (tap + 1) * tap_stride + (size_t)(ch * KS + s) * kstr;
            nbh[s] = odu_frag(rh, u, lofs);
            nbl[s] = odu_frag(rl, u, lofs);
          }
        }
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const int m = mpix[mt];
            const int off = buf * XBUF + (m / TW + dy) * XRP + (m % TW + dx) * LDX + 16 * s + (dx & 1 ? kx1 : kx0);
            const f16x8 ah = *reinterpret_cast<const f16x8*>(lhi + off);
            const f16x8 al = *reinterpret_cast<const f16x8*>(llo + off);
            acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bl[s], ah, acc[mt], 0, 0, 0);
            acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[s], al, acc[mt], 0, 0, 0);
            acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[s], ah, acc[mt], 0, 0, 0);
          }
        if (tap + 1 < 9) {
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            bh[s] = nbh[s];
            bl[s] = nbl[s];
          }
        }
      }
      if constexpr (DB) {
        if (ch + 1 < NCHX) {
          // buffer (ch + 1) & 1 was last read in chunk ch - 1, whose readers all passed the barrier
          // that ended that chunk; this chunk's MFMAs are issued and run on meanwhile
          load_stage(ch + 1, buf ^ 1);
          __syncthreads();
        }
      }
    }
  }
  __syncthreads();   // every wave has read the x halo: t1 overlays it

  // ---- t1 = ELU(BN_mid(acc * ua + ba)), x 2^4, split, into LDS rows 1 .. H (row 0 = image row -1) ---
  // (conv_h3 writes fmaf(acc, unscale, bias) to HBM and the next launch stages BN + ELU + split of it;
  // columns past the image stage as zeros there, as here)
#pragma unroll
  for (int qd = 0; qd < 4; ++qd) {
    const int c0 = cob + 8 * qd + hsel;   // the accumulator quad's 4 consecutive channels
    const float4 b4 = *reinterpret_cast<const float4*>(a.ba + c0);
    const float4 s4 = x16(*reinterpret_cast<const float4*>(a.s_mid + c0));
    const float4 t4 = x16(*reinterpret_cast<const float4*>(a.t_mid + c0));
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mpix[mt];
      const int i = m / TW, c = m % TW;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (w0 + c < W) {
        v.x = bn_elu16(fmaf(acc[mt][4 * qd + 0], a.ua, b4.x), s4.x, t4.x);
        v.y = bn_elu16(fmaf(acc[mt][4 * qd + 1], a.ua, b4.y), s4.y, t4.y);
        v.z = bn_elu16(fmaf(acc[mt][4 * qd + 2], a.ua, b4.z), s4.z, t4.z);
        v.w = bn_elu16(fmaf(acc[mt][4 * qd + 3], a.ua, b4.w), s4.w, t4.w);
      }
      rmax = amax4(rmax, v);
      f16x4 hv, lv;
      split4(v, hv, lv);
      const int px = (i + 1) * TW + c;
      *reinterpret_cast<f16x4*>(lhi + px * LDT + c0) = hv;
      *reinterpret_cast<f16x4*>(llo + px * LDT + c0) = lv;
    }
  }
  // the zero rows: image rows -1, H, H + 1 of the strip
  for (int e = tid; e < 3 * TW * (LDT / 8); e += NT) {
    const int z = e / (LDT / 8), k8 = e - z * (LDT / 8);
    const int px = z < TW ? z : (H + 1) * TW + (z - TW);
    *reinterpret_cast<f16x8*>(lhi + px * LDT + 8 * k8) = f16x8{};
    *reinterpret_cast<f16x8*>(llo + px * LDT + 8 * k8) = f16x8{};
  }

  // residual blocks: the raw x at the wave's output pixels, loaded now so GEMM b hides the latency
  float4 rsd[POOL ? 1 : MT][4];
  if constexpr (!POOL) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mpix[mt];
      const int i = m / TW, c = m % TW;
      const bool ok = w0 + c < W;
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        rsd[mt][qd] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                          rxc, ok ? (uint32_t)((i * W + w0 + c) * C + cob + 8 * qd + hsel) * 4u : 0x80000000u, 0, 0));
    }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[mt][i] = 0.0f;
  __syncthreads();

  // ---- GEMM b: conv(4,1) over t1 (output row i, tap dy reads t1 LDS row i + dy) ---------------------
  {
    const __amdgpu_buffer_rsrc_t rh = odu_rsrc(a.wbh), rl = odu_rsrc(a.wbl);
    constexpr size_t tap_stride = (size_t)C * C;
#pragma unroll 1
    for (int ch = 0; ch < NCH; ++ch) {
      f16x8 bh[KS], bl[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bh[s] = odu_frag(rh, (size_t)(ch * KS + s) * kstr, lofs);
        bl[s] = odu_frag(rl, (size_t)(ch * KS + s) * kstr, lofs);
      }
#pragma unroll
      for (int tap = 0; tap < 4; ++tap) {
        f16x8 nbh[KS], nbl[KS];
        if (tap + 1 < 4) {
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const size_t u = (tap + 1) * tap_stride + (size_t)(ch * KS + s) * kstr;
            nbh[s] = odu_frag(rh, u, lofs);
            nbl[s] = odu_frag(rl, u, lofs);
          }
        }
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const int m = mpix[mt];
            const int off = ((m / TW + tap) * TW + m % TW) * LDT + ch * CK + 16 * s + koff;
            const f16x8 ah = *reinterpret_cast<const f16x8*>(lhi + off);
            const f16x8 al = *reinterpret_cast<const f16x8*>(llo + off);
            if constexpr (POOL) {   // pixel rows: a register quad is one pool window
              acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s], acc[mt], 0, 0, 0);
              acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[s], acc[mt], 0, 0, 0);
              acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], acc[mt], 0, 0, 0);
            } else {                // C^T: a register quad is 4 channels of one pixel
              acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bl[s], ah, acc[mt], 0, 0, 0);
              acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[s], al, acc[mt], 0, 0, 0);
              acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[s], ah, acc[mt], 0, 0, 0);
            }
          }
        if (tap + 1 < 4) {
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            bh[s] = nbh[s];
            bl[s] = nbl[s];
          }
        }
      }
    }
  }

  // ---- epilogue ------------------------------------------------------------------------------------
  if constexpr (!POOL) {
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
      const int c0 = cob + 8 * qd + hsel;
      const float4 b4 = *reinterpret_cast<const float4*>(a.bb + c0);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = mpix[mt];
        const int i = m / TW, c = m % TW;
        if (w0 + c >= W) continue;
        const float4 r = rsd[mt][qd];
        float4 v = make_float4(fmaf(acc[mt][4 * qd + 0], a.ub, b4.x), fmaf(acc[mt][4 * qd + 1], a.ub, b4.y),
                               fmaf(acc[mt][4 * qd + 2], a.ub, b4.z), fmaf(acc[mt][4 * qd + 3], a.ub, b4.w));
        v = make_float4(v.x + r.x, v.y + r.y, v.z + r.z, v.w + r.w);
        *reinterpret_cast<float4*>(a.y + ((clip * H + i) * W + w0 + c) * C + c0) = v;
      }
    }
  } else {
    // the shortcut Conv2D(1x1, stride 2): A row rho = window (mt = rho >> 3, quad q = rho & 3, lane
    // half (rho >> 2) & 1) of the main tile, i.e. its top-left input pixel; accumulator register
    // 4 mt + q of lane half h then holds main register quad (mt, q) of that half's window
    f32x16 sacc;
#pragma unroll
    for (int i = 0; i < 16; ++i) sacc[i] = 0.0f;
    {
      const int rho = lane & 31;
      const int smt = rho >> 3, sq = rho & 3, sh = (rho >> 2) & 1;
      const bool sok = smt < MT;
      const int m0 = (wm * MT + (sok ? smt : 0)) * 32 + 8 * sq + 4 * sh;
      const float* sx = xc + ((int64_t)(m0 / TW) * W + w0) * CIN + koff;
      const __amdgpu_buffer_rsrc_t rh = odu_rsrc(a.wsh), rl = odu_rsrc(a.wsl);
#pragma unroll
      for (int s = 0; s < CIN / 16; ++s) {
        float4 x0 = make_float4(0.f, 0.f, 0.f, 0.f), x1 = x0;
        if (sok) {
          x0 = *reinterpret_cast<const float4*>(sx + 16 * s);
          x1 = *reinterpret_cast<const float4*>(sx + 16 * s + 4);
        }
        x0 = x16(x0);
        x1 = x16(x1);
        rmax = amax4(amax4(rmax, x0), x1);
        f16x4 h0, l0, h1, l1;
        split4(x0, h0, l0);
        split4(x1, h1, l1);
        const f16x8 xh = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        const f16x8 xl = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
        const f16x8 wh = odu_frag(rh, (size_t)s * kstr, lofs);
        const f16x8 wl = odu_frag(rl, (size_t)s * kstr, lofs);
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wl, sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, wh, sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wh, sacc, 0, 0, 0);
      }
    }
    const int co = cob + (lane & 31);
    const float b = a.bb[co], bsc = a.bs[co];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        // register quad qd: rows i0, i0 + 1 (i0 = m0 / 2, even) x columns w0, w0 + 1
        const int m0 = (wm * MT + mt) * 32 + 8 * qd + hsel;
        const int i0 = m0 / TW;
        float mx = fmaf(acc[mt][4 * qd], a.ub, b);
        mx = fmaxf(mx, fmaf(acc[mt][4 * qd + 1], a.ub, b));
        mx = fmaxf(mx, fmaf(acc[mt][4 * qd + 2], a.ub, b));
        mx = fmaxf(mx, fmaf(acc[mt][4 * qd + 3], a.ub, b));
        mx += fmaf(sacc[4 * mt + qd], a.us, bsc);
        a.y[((clip * (H / 2) + i0 / 2) * (W / 2) + w0 / 2) * C + co] = mx;
      }
  }
  if (!(rmax < SPLIT_MAX) && a.range_flag) *a.range_flag = 1;
}

template <int H, int W, int CIN, int C, int TW, bool POOL, int NW = 4, int MINW = 2>
hipError_t launch(const OduArgs& a, hipStream_t s) {
  constexpr int TLW = (W + TW - 1) / TW;
  const int64_t blocks = (int64_t)a.n * TLW;
  hipLaunchKernelGGL((odu_kernel<H, W, CIN, C, TW, POOL, NW, MINW>), dim3((unsigned)blocks), dim3(64 * NW), 0, s, a);
  return hipGetLastError();
}

}  // namespace

bool odu_supported(int h, int w, int cin, int c, bool pool) {
  return (h == 64 && w == 76 && cin == 32 && c == 64 && pool) ||    // block 4
         (h == 32 && w == 38 && cin == 64 && c == 64 && !pool) ||   // blocks 5-6
         (h == 32 && w == 38 && cin == 64 && c == 128 && pool) ||   // block 7
         (h == 16 && w == 19 && cin == 128 && c == 128 && !pool);   // blocks 8-9
}

hipError_t odu_launch(const OduArgs& a, int h, int w, int cin, int c, bool pool, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  if (!a.x || !a.y || a.x == a.y || !odu_supported(h, w, cin, c, pool) ||
      (pool && (!a.wsh || !a.wsl || !a.bs)))
    return hipErrorInvalidValue;
  // strips and register budgets, measured per kernel (rocprof, one box, per 16 384-clip launch):
  // blocks 5-6 TW 4 at 3 waves per SIMD (<= 168 VGPRs, 1 spilled) 8.56 -> 7.55 ms; TW 2 with two-wave
  // workgroups 8.16 ms; 4 waves per SIMD (<= 128 VGPRs) spill 20-44 VGPRs: block 7 15.5 -> 17.2 ms,
  // blocks 5-6 10.6 ms.  Blocks 4 and 8-9 are LDS-bound at 3 workgroups per CU (42 / 41 KB)
  if (h == 64 && pool) return launch<64, 76, 32, 64, 2, true, 4, 4>(a, s);
  if (h == 32 && c == 64) return launch<32, 38, 64, 64, 4, false, 4, 3>(a, s);
  if (h == 32 && pool) return launch<32, 38, 64, 128, 2, true>(a, s);
  return launch<16, 19, 128, 128, 4, false>(a, s);
}
