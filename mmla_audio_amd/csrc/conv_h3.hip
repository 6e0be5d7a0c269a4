// Halo-tiled implicit-GEMM convolution on gfx950 f16 MFMA with error-compensated 3xFP16 products.
//
// Each float32 operand v is split into v = hi + lo * 2^-11 with hi = fp16(v), lo = fp16((v - hi) * 2^11)
// (|error| <= 2^-22 |v| for |v| < 65504).  A product a*w is accumulated as
//     acc1 += hi(a) hi(w)                       (v_mfma_f32_32x32x16_f16)
//     acc2 += hi(a) lo(w) + lo(a) hi(w)         (two more, same shape)
//     y     = acc1 + 2^-11 acc2                 (dropped term lo*lo*2^-22 <= 2^-22 |a w|)
// i.e. ~22-bit products with float32 accumulation -- float32-class accuracy (the reference's Keras
// layers run float32) at 16/3 = 5.3x the f32-MFMA rate.  Layer-wise parity vs the float64 oracle:
// tests/test_gpu_parity.py::test_od_layerwise_trace.
//
// Tiling (256 threads = 4 waves): one workgroup computes a TH x TW (<= 128 pixel) output tile of one
// clip for BN output channels.  Per chunk of CK input channels the (TH+KH-1) x (TW+KW-1) input halo
// is staged ONCE into LDS -- with the BatchNorm + ELU/ReLU prologue applied once per input element
// (not once per tap) and split into fp16 hi/lo -- and all KH*KW taps read their A fragments from
// it (ds_read_b128, pixel rows padded by 16 B: conflict-free).  B fragments (pre-split weights,
// [tap][cout][cin] so a lane's 8 k-values are one 16-B load) come from L2 with the next tap's
// prefetched under the current tap's MFMAs.  Waves split the tile 4x1 (BN = 32) or 2x2 (BN >= 64).
// Epilogue: bias, optional in-place residual, or (pool blocks) MaxPool2D(2,'same') of the tile
// written at half resolution -- the 2x2 window lives in one lane's accumulator registers when
// TW = 16 (rows r, r+1, r+16, r+17 of a 32-row MFMA tile).
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
constexpr float LO_SCALE = 2048.0f;
constexpr float LO_INV = 1.0f / 2048.0f;

template <int PRO>
MMLA_DEV float pro_fn(float v, float sc, float sh) {
  if constexpr (PRO == PRO_NONE) {
    return v;
  } else {
    v = fmaf(v, sc, sh);
    if constexpr (PRO == PRO_BN_ELU) return v > 0.0f ? v : expm1f(v);
    return fmaxf(v, 0.0f);
  }
}

template <int KH, int KW, int CK, int BN, int PRO, int EPI, bool POOL>
__global__ void __launch_bounds__(NT, BN >= 128 ? 1 : 2) conv_h3_kernel(ConvH3Args a) {
  constexpr int WN = BN >= 64 ? 2 : 1;
  constexpr int WM = 4 / WN;
  constexpr int MT = BM / (WM * 32);      // 32-row tiles per wave
  constexpr int NTL = BN / (WN * 32);     // 32-col tiles per wave
  constexpr int LDP = CK + 8;             // fp16 per staged pixel (16-B pad: conflict-free b128)
  constexpr int KS = CK / 16;             // MFMA k-steps per chunk
  constexpr int TAPS = KH * KW;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int WP = a.tw + KW - 1;
  const int npix = (a.th + KH - 1) * WP;
  _Float16* lds_hi = reinterpret_cast<_Float16*>(smem);
  _Float16* lds_lo = lds_hi + npix * LDP;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int tiles = a.tiles_h * a.tiles_w;
  const int64_t clip = blockIdx.x / tiles;
  const int tile = blockIdx.x - (int)(clip * tiles);
  const int h0 = (tile / a.tiles_w) * a.th;
  const int w0 = (tile - (tile / a.tiles_w) * a.tiles_w) * a.tw;
  const int n0 = blockIdx.y * BN;
  const int tpix = a.th * a.tw;

  int apix[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = (wm * MT + mt) * 32 + (lane & 31);
    const int th = m / a.tw, tw = m - (m / a.tw) * a.tw;
    apix[mt] = m < tpix ? (th * WP + tw) * LDP : 0;
  }
  const int koff = (lane >> 5) * 8;

  f32x16 acc1[MT][NTL], acc2[MT][NTL];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        acc1[mt][nt][i] = 0.0f;
        acc2[mt][nt][i] = 0.0f;
      }

  const uint16_t* whp[NTL];
  const uint16_t* wlp[NTL];
#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) {
    const int co = n0 + (wn * NTL + nt) * 32 + (lane & 31);
    whp[nt] = a.wh + (size_t)co * a.cin_pad + koff;
    wlp[nt] = a.wl + (size_t)co * a.cin_pad + koff;
  }
  const size_t tap_stride = (size_t)a.cout_pad * a.cin_pad;

  const int nchunks = a.cin_pad / CK;
  for (int ch = 0; ch < nchunks; ++ch) {
    const int ci0 = ch * CK;
    __syncthreads();   // every wave is done reading the previous chunk's halo
    // ---- stage the input halo of this channel chunk: prologue once per element, split hi/lo ----
    for (int task = tid; task < npix * (CK / 4); task += NT) {
      const int px = task / (CK / 4), q = task - px * (CK / 4);
      const int py = px / WP, pxx = px - py * WP;
      const int ih = h0 - a.pad_h + py, iw = w0 - a.pad_w + pxx;
      const int ci = ci0 + q * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ih >= 0 && ih < a.h && iw >= 0 && iw < a.w && ci < a.cin) {
        v = *reinterpret_cast<const float4*>(a.x + ((clip * a.h + ih) * a.w + iw) * a.cin + ci);
        if constexpr (PRO != PRO_NONE) {
          const float4 sc = *reinterpret_cast<const float4*>(a.scale + ci);
          const float4 sh = *reinterpret_cast<const float4*>(a.shift + ci);
          v.x = pro_fn<PRO>(v.x, sc.x, sh.x);
          v.y = pro_fn<PRO>(v.y, sc.y, sh.y);
          v.z = pro_fn<PRO>(v.z, sc.z, sh.z);
          v.w = pro_fn<PRO>(v.w, sc.w, sh.w);
        }
      }
      f16x4 hv, lv;
      hv[0] = (_Float16)v.x;
      hv[1] = (_Float16)v.y;
      hv[2] = (_Float16)v.z;
      hv[3] = (_Float16)v.w;
      lv[0] = (_Float16)((v.x - (float)hv[0]) * LO_SCALE);
      lv[1] = (_Float16)((v.y - (float)hv[1]) * LO_SCALE);
      lv[2] = (_Float16)((v.z - (float)hv[2]) * LO_SCALE);
      lv[3] = (_Float16)((v.w - (float)hv[3]) * LO_SCALE);
      *reinterpret_cast<f16x4*>(lds_hi + px * LDP + q * 4) = hv;
      *reinterpret_cast<f16x4*>(lds_lo + px * LDP + q * 4) = lv;
    }
    __syncthreads();

    // ---- all taps of this chunk ------------------------------------------------------------------
    f16x8 bh[NTL][KS], bl[NTL][KS];
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bh[nt][s] = *reinterpret_cast<const f16x8*>(whp[nt] + ci0 + 16 * s);
        bl[nt][s] = *reinterpret_cast<const f16x8*>(wlp[nt] + ci0 + 16 * s);
      }
#pragma unroll
    for (int tap = 0; tap < TAPS; ++tap) {
      const int dy = tap / KW, dx = tap - (tap / KW) * KW;
      const int toff = (dy * WP + dx) * LDP;
      f16x8 nbh[NTL][KS], nbl[NTL][KS];
      if (tap + 1 < TAPS) {   // prefetch the next tap's B fragments under this tap's MFMAs
#pragma unroll
        for (int nt = 0; nt < NTL; ++nt)
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            nbh[nt][s] = *reinterpret_cast<const f16x8*>(whp[nt] + (tap + 1) * tap_stride + ci0 + 16 * s);
            nbl[nt][s] = *reinterpret_cast<const f16x8*>(wlp[nt] + (tap + 1) * tap_stride + ci0 + 16 * s);
          }
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int off = apix[mt] + toff + 16 * s + koff;
          const f16x8 ah = *reinterpret_cast<const f16x8*>(lds_hi + off);
          const f16x8 al = *reinterpret_cast<const f16x8*>(lds_lo + off);
#pragma unroll
          for (int nt = 0; nt < NTL; ++nt) {
            acc1[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[nt][s], acc1[mt][nt], 0, 0, 0);
            acc2[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[nt][s], acc2[mt][nt], 0, 0, 0);
            acc2[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[nt][s], acc2[mt][nt], 0, 0, 0);
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

  // ---- epilogue --------------------------------------------------------------------------------
#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) {
    const int co = n0 + (wn * NTL + nt) * 32 + (lane & 31);
    if (co >= a.cout) continue;
    const float b = a.bias[co];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = acc1[mt][nt][r] + acc2[mt][nt][r] * LO_INV + b;
      const int mbase = (wm * MT + mt) * 32;
      if constexpr (POOL) {
        // TW == 16: this 32-row tile holds output rows (th, th+1), th = mbase / 16 (even)
        const int oh = h0 + mbase / 16;
        const int hp = (a.h + 1) / 2, wp = (a.w + 1) / 2;
        if (mbase < tpix && oh < a.h) {
#pragma unroll
          for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
              const int twi = 8 * q + 4 * (lane >> 5) + e;   // even column of the window
              const int ow = w0 + twi;
              if (ow >= a.w) continue;
              float mx = v[4 * q + e];
              if (ow + 1 < a.w) mx = fmaxf(mx, v[4 * q + e + 1]);
              if (oh + 1 < a.h) {
                mx = fmaxf(mx, v[4 * q + 8 + e]);
                if (ow + 1 < a.w) mx = fmaxf(mx, v[4 * q + 9 + e]);
              }
              a.y[((clip * hp + oh / 2) * wp + ow / 2) * a.cout + co] = mx;
            }
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mbase + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (m >= tpix) continue;
          const int oh = h0 + m / a.tw, ow = w0 + (m - (m / a.tw) * a.tw);
          if (oh >= a.h || ow >= a.w) continue;
          const int64_t p = (clip * a.h + oh) * a.w + ow;
          float val = v[r];
          if constexpr (EPI == EPI_ADD) val += a.res[p * a.cout + co];
          a.y[p * a.cout + co] = val;
        }
      }
    }
  }
}

template <int KH, int KW, int CK, int BN, int PRO, int EPI, bool POOL>
hipError_t launch(const ConvH3Args& a, hipStream_t s) {
  const size_t smem = (size_t)(a.th + KH - 1) * (a.tw + KW - 1) * (CK + 8) * 2 * sizeof(_Float16);
  auto k = conv_h3_kernel<KH, KW, CK, BN, PRO, EPI, POOL>;
  if (smem > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
  }
  dim3 grid((unsigned)((int64_t)a.n * a.tiles_h * a.tiles_w), (unsigned)(a.cout_pad / BN));
  hipLaunchKernelGGL(k, grid, dim3(NT), smem, s, a);
  return hipGetLastError();
}

template <int KH, int KW, int CK, int PRO, int EPI, bool POOL>
hipError_t by_bn(const ConvH3Args& a, hipStream_t s) {
  if (a.cout_pad % 128 == 0) return launch<KH, KW, CK, 128, PRO, EPI, POOL>(a, s);
  if (a.cout_pad % 64 == 0) return launch<KH, KW, CK, 64, PRO, EPI, POOL>(a, s);
  return launch<KH, KW, CK, 32, PRO, EPI, POOL>(a, s);
}

// pick (th, tw): minimise MFMA rows issued + halo staging over the whole image
void pick_tile(ConvH3Args& a) {
  if (a.pool_out) {   // the fused 2x2 pool needs TW = 16, TH = 8 (aligned, even)
    a.tw = 16;
    a.th = 8;
  } else if (a.w == 1) {
    a.tw = 1;
    a.th = 128;
  } else {
    double best = 1e30;
    const int cands[] = {8, 16, 19, 20, 32, 38, 40, 64, 76};
    for (int tw : cands) {
      if (tw > 2 * a.w && tw != 8) continue;
      const int th = BM / tw;
      if (th < 1) continue;
      const int tiles = ((a.h + th - 1) / th) * ((a.w + tw - 1) / tw);
      const double halo = (double)(th + a.kh - 1) * (tw + a.kw - 1);
      const double cost = tiles * (BM * a.kh * a.kw * 1.0 + halo * 2.0);
      if (cost < best) {
        best = cost;
        a.tw = tw;
        a.th = th;
      }
    }
  }
  a.tiles_h = (a.h + a.th - 1) / a.th;
  a.tiles_w = (a.w + a.tw - 1) / a.tw;
}

}  // namespace

hipError_t conv_h3_launch(ConvH3Args a, hipStream_t s) {
  if ((int64_t)a.n * a.h * a.w == 0) return hipSuccess;
  if (a.cin % 4 != 0 || a.cout_pad % 32 != 0) return hipErrorInvalidValue;
  pick_tile(a);
  const int ck = a.cin_pad % 32 == 0 ? 32 : 16;
  if (a.cin_pad % ck != 0) return hipErrorInvalidValue;
#define H3(KH, KW, CK, P, E, PL)                                                            \
  if (a.kh == KH && a.kw == KW && ck == CK && a.pro == P && a.epi == E && (a.pool_out != 0) == PL) \
    return by_bn<KH, KW, CK, P, E, PL>(a, s);
  // OD-NET res_block convs (overlap_detector_temp.py:258-274)
  H3(3, 3, 16, PRO_BN_ELU, EPI_BIAS, false)
  H3(3, 3, 32, PRO_BN_ELU, EPI_BIAS, false)
  H3(4, 1, 32, PRO_BN_ELU, EPI_BIAS, true)
  H3(4, 1, 32, PRO_BN_ELU, EPI_ADD, false)
  // SI-NET res_unit convs (speaker_identification.py:173-188)
  H3(3, 1, 32, PRO_BN_RELU, EPI_BIAS, false)
  H3(3, 1, 32, PRO_BN_RELU, EPI_ADD, false)
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
                           int cout_pad, uint16_t* hi, uint16_t* lo) {
  const size_t n = (size_t)kh * kw * cout_pad * cin_pad;
  for (size_t i = 0; i < n; ++i) hi[i] = lo[i] = 0;
  for (int t = 0; t < kh * kw; ++t)
    for (int ci = 0; ci < cin; ++ci)
      for (int co = 0; co < cout; ++co) {
        const float v = w[((size_t)t * cin + ci) * cout + co];
        const _Float16 h = (_Float16)v;
        const size_t o = ((size_t)t * cout_pad + co) * cin_pad + ci;
        hi[o] = f32_to_f16_bits(v);
        lo[o] = f32_to_f16_bits((v - (float)h) * LO_SCALE);
      }
}
