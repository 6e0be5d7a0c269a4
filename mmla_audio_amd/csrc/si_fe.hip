// SpeakerIdentification front-end: int16 PCM -> [256, 39] MFCC + delta + delta-delta (float64 math).
//
// Replaces input_feature_gen (speaker_identification.py:372-398), i.e.:
//   wav.read int16; len < 4000 => 'silent'                         :374-376
//   python_speech_features.mfcc(sig, 16000, .025, .01, nfft=512)   :386
//     preemphasis 0.97 -> rectangular 400/160 frames, zero tail -> |rfft_512|^2 / 512 ->
//     energy = sum, 26 HTK-mel triangles (floor bins) -> log (0 -> eps) -> DCT-II ortho[:13] ->
//     lifter 22 -> c0 := log(energy)
//   delta(feat, 2) twice (edge padding), concat -> [T, 39]          :387-389 (delta :141-151)
//   zero-pad / truncate to 256 frames                              :391-395
// psf computes in float64; so does this kernel (gfx950 fp64 VALU), so parity is ~1e-12, not the
// ~4e-5 an fp32 FFT gives (SURVEY.md 7 "Hard parts").  Output is stored float32 (predict casts).
//
// The kernel computes a 512-point real FFT per frame as a 256-point complex FFT of the packed frame
// (s[2n] + i s[2n+1]) factored 16 x 16, then the real split; only min(T, 260) frames are computed
// (delta-delta of row 255 reaches feat[259]).
//
// v2.  One wave = one clip (64-thread workgroups, ~19.7 KB LDS: 8 clips in flight per
// CU), frames in rounds of R = 4, no block barriers (a wave's LDS operations execute in issue
// order).  Per round:
//   window   the round's 888 samples, register-prefetched one round ahead (16-B chunks)
//   pass A   lane (f, n2): pre-emphasis from LDS int16, DFT-16 over n1, x W256^(n2 k1) (twiddles
//            in registers), and the frame's sum of squared samples (row reduction, 16 lanes)
//   pass B   lane (f, k1): DFT-16 over n2 -> Z[k1 + 16 k2], in place
//   split    P[k] = |X[k]|^2 / 512 for k and 256 - k from Z[k], Z[256 - k], over the frame's Z
//   filters  the triangular filterbank as segment sums: segment s = bins [bin[s], bin[s+1]) is the
//            rising edge of filter s and the falling edge of filter s - 1, so with
//            A_s = sum P[k], B_s = sum (k - bin[s]) P[k] over the segment,
//              fbank[j] = B_j / w_j + A_{j+1} - B_{j+1} / w_{j+1}        (w_s = segment width)
//            (no cancellation beyond the segment: every falling weight is >= 1/w).  Segments are
//            cut into <= 8-bin sub-segments, one lane task each.  energy = sum_k P[k] by Parseval:
//              sum_{k=0}^{256} |X[k]|^2 / 512 = (sum s^2 + P[0] + P[256]) / 2
//   dct      lane (f, c): 26-term dot with the lifted DCT row held in registers; c0 = log energy
// Cepstra go straight to the output rows (halo frames to LDS); the epilogue re-reads them into LDS
// and writes the deltas (the clip's 264 x 13 cepstra do not fit beside the round buffers).
#include "common.h"
#include "si_fe.h"

#include <cstdlib>
#include <type_traits>

// The power spectrum is stored and the filterbank summed in float32 after the float64
// FFT and real split (which must stay float64: a tone near Nyquist makes the weak low bins the
// difference of two huge values); the sums of positive powers are well conditioned, the features
// move by <= ~3e-6 from the float64 oracle (numpy model on the worst-case tones) against the 1e-4
// bar.  The float64 sub-segment sums had cost 13 % of the kernel (a build without them: 26.6 ->
// 23.2 ms per 3 SI steps)

namespace {

constexpr int HALO = 4;              // delta-delta reach in frames
constexpr int OUTF = 256;
constexpr int NL = OUTF + 2 * HALO;  // local frames per window: [frame0 - 4, frame0 + 260)

MMLA_DEV void lds_order() { asm volatile("" ::: "memory"); }

template <typename C>
MMLA_DEV void fft4c(C& a0, C& a1, C& a2, C& a3) {
  C s02 = cadd(a0, a2), d02 = csub(a0, a2), s13 = cadd(a1, a3), d13 = csub(a1, a3);
  a0 = cadd(s02, s13);
  a2 = csub(s02, s13);
  a1 = cadd(d02, cmul_negi(d13));
  a3 = csub(d02, cmul_negi(d13));
}

// ================================================================================================

// ================================================================================================
namespace v2 {

constexpr int NT = 64;                          // one wave per clip / window
constexpr int R = 4;                            // frames per round (pass A: 16 lanes per frame)
constexpr int WIN = 888;                        // samples [160 g0 - 8, 160 g0 + 880) of a round
constexpr int WCH = WIN / 8;                    // 111 16-B chunks
constexpr int FP = 273;                         // frame region pitch (cd): 16 pass-A rows of 17 + 1
constexpr int PART = 258;                       // region doubles: P[0..256], then (A, B) sub sums
// the power spectrum / sub-sum element type (float32) and the sub sums' offset in that type
typedef float fbt;
typedef float2 fbt2;
constexpr int PSUM = 2 * PART;
constexpr int LFE = PART + 2 * SI_FE_MAX_SUB;   // then 27 log energies
static_assert(LFE + 27 <= 2 * FP, "frame region");
static_assert(NL * 13 * sizeof(float) <= R * FP * sizeof(cd), "epilogue cepstra tile");

struct Smem {                   // 18.7 KB: 8 clip-waves per CU
  // pass A rows [k1][17] -> Z[k] -> P[k] (doubles) + sums + logs.  The round's window
  // x[160 g0 - 8 + w] (0 outside [0, len)) is staged over the start of z: pass A issues all of its
  // window reads before its first row store, and nothing else reads the window
  cd z[R][FP];
  double s2[R];                 // sum of the frame's squared pre-emphasised samples
  float ext[2 * HALO][13];      // cepstra of local frames 0..3 and 260..263 (not output rows)
  double dct[12][13];           // lifted DCT-II rows 1..12, folded (26 -> 13 terms)
};
static_assert(WIN * sizeof(int16_t) <= sizeof(cd) * R * FP, "window inside z");
MMLA_DEV int16_t* win_of(Smem& sm) { return reinterpret_cast<int16_t*>(&sm.z[0][0]); }

// W16^e = exp(-2 pi i e / 16)
constexpr double C8 = 0.92387953251128675613, S8 = 0.38268343236508977173, RH = 0.70710678118654752440;
MMLA_DEV cd w16c(int e) {
  switch (e) {
    case 1: return {C8, -S8};
    case 2: return {RH, -RH};
    case 3: return {S8, -C8};
    case 4: return {0.0, -1.0};
    case 6: return {-RH, -RH};
    default: return {-C8, S8};   // 9
  }
}

// complex 16-point DFT in registers, radix 4 x 4: in v[n], out v[4*q1 + q2] = Y[q1 + 4*q2]
MMLA_DEV void dft16(cd v[16]) {
#pragma unroll
  for (int m2 = 0; m2 < 4; ++m2) fft4c(v[m2], v[4 + m2], v[8 + m2], v[12 + m2]);
#pragma unroll
  for (int q1 = 1; q1 < 4; ++q1)
#pragma unroll
    for (int m2 = 1; m2 < 4; ++m2) {
      const int e = m2 * q1;
      if (e == 4) v[4 * q1 + m2] = cmul_negi(v[4 * q1 + m2]);
      else v[4 * q1 + m2] = cmul(v[4 * q1 + m2], w16c(e));
    }
#pragma unroll
  for (int q1 = 0; q1 < 4; ++q1) fft4c(v[4 * q1 + 0], v[4 * q1 + 1], v[4 * q1 + 2], v[4 * q1 + 3]);
}

// P[k] and P[256 - k] (|X|^2 / 512) of the 512-point real DFT from Z[k], Z[256 - k]
// (computed at twice the scale: the halvings of e and o and the 1/512 fold into one 1/2048 -- powers
// of two, so every rounding is the same and the result bit-identical, four multiplies fewer)
MMLA_DEV void split_power(cd z, cd zr, cd w, double& pk, double& pnk) {
  const cd e = {z.x + zr.x, z.y - zr.y};                   // Z[k] + conj Z[-k]
  const cd o = {z.y + zr.y, zr.x - z.x};                   // (Z[k] - conj Z[-k]) / i
  const cd wo = cmul(w, o);
  const cd xp = cadd(e, wo), xm = csub(e, wo);             // 2 X[k], 2 conj X[256 - k]
  pk = (xp.x * xp.x + xp.y * xp.y) * (1.0 / 2048.0);
  pnk = (xm.x * xm.x + xm.y * xm.y) * (1.0 / 2048.0);
}

// natural log of a positive finite double (the filterbank energies): exponent from frexp, log2 of the
// mantissa in [0.5, 1) by v_log_f32 on its float32 rounding -- absolute error <= ~2e-7, where
// ocml's log (~1e-16) is a ~40-instruction routine run 27 times per frame.  The features' tolerance
// is 1e-4 absolute after the DCT (|coefficient| <= 0.28 over 26 logs) and the lifter (<= 12):
// the bound stays below 2e-5 even if every term's error had the same sign
MMLA_DEV double log_pos(double x) {
  const double m = __builtin_amdgcn_frexp_mant(x);
  const int e = __builtin_amdgcn_frexp_exp(x);
  const float l2 = __builtin_amdgcn_logf((float)m);
  return ((double)e + (double)l2) * 0.69314718055994530942;
}

__global__ void __launch_bounds__(NT, 2) si_fe_kernel(SiFeArgs a) {
  __shared__ __attribute__((aligned(16))) Smem sm;
  const SiFeTables& tb = *a.tables;
  const int lane = threadIdx.x;
  const int64_t blk = blockIdx.x;
  // feature rows of ldf floats: 39, or 40 with a zero 40th column (the fused SI pipeline: the stem
  // Conv1D then stages 16-B aligned rows as float4, conv_h3 V4)
  const int ldf = a.ldf > 39 ? 40 : 39;
  float* out = a.feat + blk * (OUTF * ldf);

  const int16_t* x;
  int64_t len, frame0;
  if (a.seq_len > 0) {            // window blk of one long signal (conversation mode)
    x = a.pcm;
    len = a.seq_len;
    frame0 = OUTF * blk;
  } else {                        // one clip per block (input_feature_gen)
    x = a.pcm + blk * a.clip_stride;
    len = a.lens ? a.lens[blk] : a.clip_len;
    frame0 = 0;
    if (len < 4000) {             // speaker_identification.py:375-376
      float4* o4 = reinterpret_cast<float4*>(out);
      for (int e = lane; e < OUTF * ldf / 4; e += NT) o4[e] = float4{0.f, 0.f, 0.f, 0.f};
      if (a.silent && lane == 0) a.silent[blk] = 1;
      return;
    }
    if (a.silent && lane == 0) a.silent[blk] = 0;
  }
  const int64_t T64 = len <= 400 ? 1 : 1 + (len - 400 + 159) / 160;   // framesig numframes
  // Window-relative 32-bit coordinates (64-bit index arithmetic was ~90 VALU per round): frames count
  // from gs, the window's first existing frame; samples from so = 160 gs - soff (soff = 16 past the
  // first window keeps the round's 8 leading samples at non-negative offsets and xw 16-B aligned as x).
  // T and the readable length are capped past everything the window reads (frames < NL + 4 apart,
  // samples < 160 NL + 888), so every comparison below has the outcome it has in global coordinates.
  const int64_t lb64 = frame0 - HALO;                                // global frame of local 0
  const int64_t gs = lb64 < 0 ? 0 : lb64;
  const int soff = gs > 0 ? 16 : 0;
  const int16_t* const xw = x + (160 * gs - soff);
  const int64_t lrem = len - (160 * gs - soff);
  const int lenw = (int)(lrem < 160 * NL + 1024 ? lrem : 160 * NL + 1024);
  const int64_t trem = T64 - gs;
  const int T = (int)(trem < NL + 16 ? trem : NL + 16);
  const int lbase = (int)(lb64 - gs);                                // -4 .. 0
  constexpr int g_lo = 0;
  const int g_hi = lbase + NL < T ? lbase + NL : T;
  const int nr = g_hi > g_lo ? (g_hi - g_lo + R - 1) / R : 0;

  // ---- per-lane constants (registers for the whole loop) -----------------------------------------
  const int fq = lane >> 4, q = lane & 15;      // pass A (f, n2) / pass B (f, k1)
  // W256^(n2 k1) = a^q1 b^q2 for k1 = q1 + 4 q2 (a = W256^n2, b = a^4): six powers in registers,
  // the other nine products formed per round
  cd ta[4], tq[4];
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    ta[i] = {tb.w256[q][i][0], tb.w256[q][i][1]};
    tq[i] = {tb.w256[q][4 * i][0], tb.w256[q][4 * i][1]};
  }
  const cd wa = {tb.w512[lane][0], tb.w512[lane][1]};
  const cd wb = {tb.w512[lane + 64][0], tb.w512[lane + 64][1]};
  // sub-segment tasks t = lane + 64 s -> (frame, sub-segment)
  const int n_sub = tb.n_sub;
  // packed into one register each (the kernel sits at the register limit): first bin [0, 9),
  // count [9, 13), frame [13, 15), sub-segment [15, 21), offset in its segment [21, 30)
  int stask[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int t = lane + NT * s;
    const bool on = t < R * n_sub;
    const int f = on ? t / n_sub : 0, u = on ? t - f * n_sub : 0;
    stask[s] = tb.sub_start[u] | (on ? tb.sub_cnt[u] : 0) << 9 | f << 13 | u << 15 | tb.sub_d0[u] << 21;
  }
  // filter tasks (lane < 52): filter j of frames lane / 26 and 2 + lane / 26; lanes 52..55: energy
  const int fj = lane % 26;
  const int u0 = tb.seg_sub[fj], u1 = tb.seg_sub[fj + 1], u2 = tb.seg_sub[fj + 2];
  const double iw0 = tb.inv_w[fj], iw1 = tb.inv_w[fj + 1];
  // DCT tasks (lane < 48): coefficient c = 1 + lane % 12 of frame lane / 12; lanes 48..51: c0
  const int dcf = lane < 48 ? lane / 12 : lane - 48, dcc = lane < 48 ? 1 + lane % 12 : 0;
  // DCT-II rows are (anti)symmetric: dct[c][25 - j] = (-1)^c dct[c][j] -> 13 coefficients, and the
  // dot product folds the log energies pairwise first
  // (in LDS: as 13 registers per lane they were spilled to scratch, and every reload waited for
  // all of the wave's outstanding window loads and cepstra stores)
  for (int e = lane; e < 12 * 13; e += NT) sm.dct[e / 13][e % 13] = tb.dct[1 + e / 13][e % 13];
  const double dsg = (dcc & 1) ? -1.0 : 1.0;

  // ---- the round's window: register prefetch one round ahead when it lies inside [0, len) --------
  const bool vec_ok = (reinterpret_cast<uintptr_t>(xw) & 15) == 0;
  auto fast = [&](int g0_) {
    const int b_ = 160 * g0_ + soff - 8;
    return vec_ok && b_ >= 0 && b_ + WIN <= lenw;
  };
  const bool l1 = lane < WCH - NT;
  uint4 nx0 = {0, 0, 0, 0}, nx1 = {0, 0, 0, 0};
#define SI_PREFETCH(g0_)                                                         \
  do {                                                                           \
    const uint4* s4_ = reinterpret_cast<const uint4*>(xw + 160 * (g0_) + soff - 8); \
    nx0 = s4_[lane];                                                             \
    nx1 = s4_[l1 ? lane + NT : WCH - 1];                                         \
  } while (0)
  if (nr > 0 && fast(g_lo)) SI_PREFETCH(g_lo);

  for (int r = 0; r < nr; ++r) {
    const int g0 = g_lo + R * r;
    const int base = 160 * g0 + soff - 8;
    const bool fr = fast(g0);
    lds_order();   // the previous round's reads of win / z are issued
    if (fr) {
      uint4* w4 = reinterpret_cast<uint4*>(win_of(sm));
      w4[lane] = nx0;
      if (l1) w4[lane + NT] = nx1;
    } else {
      constexpr int SPL = (WIN + NT - 1) / NT;   // 14
      int16_t v[SPL];
#pragma unroll
      for (int j = 0; j < SPL; ++j) {
        const int w = lane + NT * j;
        const int i = base + w;
        v[j] = (w < WIN && i >= 0 && i < lenw) ? xw[i] : (int16_t)0;
      }
#pragma unroll
      for (int j = 0; j < SPL; ++j)
        if (lane + NT * j < WIN) win_of(sm)[lane + NT * j] = v[j];
    }
    if (r + 1 < nr && fast(g0 + R)) SI_PREFETCH(g0 + R);
    lds_order();

    // ---- pass A: z[n] = s[2n] + i s[2n+1], n = 16 n1 + q (< 200: 400-sample frame in 512) ----------
    {
      const uint32_t* wv = reinterpret_cast<const uint32_t*>(win_of(sm)) + 4 + 80 * fq + q;
      const int lim = lenw - (160 * (g0 + fq) + soff + 2 * q);   // s[2n] exists iff 32 n1 < lim
      cd v[16];
      double e2 = 0.0;
      auto load = [&](int n1, bool gated) {
        const uint32_t cur = wv[16 * n1], prv = wv[16 * n1 - 1];
        const double xe = (double)(int16_t)(cur & 0xffffu), xo = (double)((int32_t)cur >> 16);
        const double xp = (double)((int32_t)prv >> 16);
        double se = xe - 0.97 * xp, so = xo - 0.97 * xe;   // numpy: x[1:] - 0.97 * x[:-1]
        if (gated) {
          se = 32 * n1 < lim ? se : 0.0;
          so = 32 * n1 + 1 < lim ? so : 0.0;
        }
        v[n1] = {se, so};
        e2 = fma(se, se, fma(so, so, e2));
      };
      if (fr) {
#pragma unroll
        for (int n1 = 0; n1 < 12; ++n1) load(n1, false);
        if (q < 8) load(12, false); else v[12] = {0.0, 0.0};
      } else {
#pragma unroll
        for (int n1 = 0; n1 < 12; ++n1) load(n1, true);
        if (q < 8) load(12, true); else v[12] = {0.0, 0.0};
      }
      v[13] = v[14] = v[15] = cd{0.0, 0.0};
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) e2 += __shfl_xor(e2, o, 16);
      if (q == 0) sm.s2[fq] = e2;
      dft16(v);
      cd* dst = &sm.z[fq][q];
#pragma unroll
      for (int q1 = 0; q1 < 4; ++q1)
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
          const int k1 = q1 + 4 * q2;
          const cd w = q1 == 0 ? tq[q2] : (q2 == 0 ? ta[q1] : cmul(ta[q1], tq[q2]));
          dst[17 * k1] = k1 == 0 ? v[0] : cmul(v[4 * q1 + q2], w);
        }
    }
    lds_order();
    // ---- pass B: DFT-16 over n2 of row [f][k1][*] -> Z[k1 + 16 k2] (flat in the frame region) -----
    {
      cd v[16];
      const cd* row = &sm.z[fq][17 * q];
#pragma unroll
      for (int n2 = 0; n2 < 16; ++n2) v[n2] = row[n2];
      lds_order();
      dft16(v);
#pragma unroll
      for (int q1 = 0; q1 < 4; ++q1)
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) sm.z[fq][q + 16 * (q1 + 4 * q2)] = v[4 * q1 + q2];
    }
    lds_order();
    // ---- split: P[k] for k = lane, 256 - lane, lane + 64, 192 - lane (+ 128), fbt over Z ----------
#pragma unroll
    for (int f = 0; f < R; ++f) {
      const cd* Z = sm.z[f];
      fbt* P = reinterpret_cast<fbt*>(sm.z[f]);
      const cd za = Z[lane], zar = Z[(256 - lane) & 255], zb = Z[lane + 64], zbr = Z[192 - lane];
      const cd zm = Z[128];
      lds_order();
      double p0, p1, p2, p3;
      split_power(za, zar, wa, p0, p1);
      split_power(zb, zbr, wb, p2, p3);
      P[lane] = (fbt)p0;
      P[256 - lane] = (fbt)p1;
      P[lane + 64] = (fbt)p2;
      P[192 - lane] = (fbt)p3;
      if (lane == 0) P[128] = (fbt)((zm.x * zm.x + zm.y * zm.y) * (1.0 / 512.0));
    }
    lds_order();
    // ---- sub-segment sums: A = sum P[k], B = sum (k - bin[s]) P[k] = sum i P + d0 A -------------------
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int scn = (stask[s] >> 9) & 15;
      if (scn > 0) {
        fbt* Q = reinterpret_cast<fbt*>(sm.z[(stask[s] >> 13) & 3]);
        const fbt* p = Q + (stask[s] & 511);
        fbt A = 0, B = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const fbt v = p[i];                    // past the sub-segment: finite LDS words, not used
          const fbt pv = i < scn ? v : (fbt)0;
          A += pv;
          if (i > 0) B = fma((fbt)i, pv, B);
        }
        int d0 = (stask[s] >> 21) & 511;
        asm volatile("" : "+v"(d0));   // converted here: a hoisted double of it was spilled
        reinterpret_cast<fbt2*>(Q + PSUM)[(stask[s] >> 15) & 63] = fbt2{A, fma((fbt)d0, A, B)};
      }
    }
    lds_order();
    // ---- filterbank energies and frame energy -> log (0 -> eps) --------------------------------------
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (lane < 52 || (s == 0 && lane < 56)) {
        const int f = lane < 52 ? 2 * s + lane / 26 : lane - 52;
        const fbt* Q = reinterpret_cast<const fbt*>(sm.z[f]);
        const fbt2* ps = reinterpret_cast<const fbt2*>(Q + PSUM);
        double arg;
        int slot;
        if (lane < 52) {
          fbt bj = 0, aj1 = 0, bj1 = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (u0 + i < u1) bj += ps[u0 + i].y;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (u1 + i < u2) {
              const fbt2 v = ps[u1 + i];
              aj1 += v.x;
              bj1 += v.y;
            }
          arg = (double)fma(bj, (fbt)iw0, aj1 - bj1 * (fbt)iw1);
          slot = fj;
        } else {
          arg = 0.5 * (sm.s2[f] + (double)Q[0] + (double)Q[256]);   // Parseval: sum_{k=0}^{256} P[k]
          slot = 26;
        }
        if (arg == 0.0) arg = 2.220446049250313e-16;   // numpy.finfo(float).eps
        reinterpret_cast<double*>(sm.z[f])[LFE + slot] = log_pos(arg);
      }
    }
    lds_order();
    // ---- DCT-II ortho x lifter (c = 1..12), c0 = log energy -> output row / halo -------------------
    if (lane < 52) {
      const double* L = reinterpret_cast<const double*>(sm.z[dcf]) + LFE;
      double v;
      if (lane < 48) {
        v = 0.0;
#pragma unroll
        for (int j = 0; j < 13; ++j) v = fma(fma(dsg, L[25 - j], L[j]), sm.dct[dcc - 1][j], v);
      } else {
        v = L[26];
      }
      const int g = g0 + dcf;
      if (g < g_hi) {
        const int lf = g - lbase;
        if (lf >= HALO && lf < HALO + OUTF) out[(lf - HALO) * ldf + dcc] = (float)v;
        else sm.ext[lf < HALO ? lf : lf - OUTF][dcc] = (float)v;
      }
    }
  }
#undef SI_PREFETCH

  // ---- epilogue: cepstra of local frames [g_lo, g_hi) into LDS, then the 39 output columns --------
  wave_stores_done();   // this wave's cepstra stores have completed (common.h)
  lds_order();
  float* C = reinterpret_cast<float*>(&sm.z[0][0]);   // [NL][13]
  constexpr int CPL = (NL * 13 + NT - 1) / NT;         // 54
#pragma unroll 9
  for (int i = 0; i < CPL; ++i) {
    const int e = lane + NT * i;
    if (e < NL * 13) {
      const int lf = e / 13, c = e - lf * 13;
      const int g = lbase + lf;
      if (g >= g_lo && g < g_hi)
        C[e] = (lf >= HALO && lf < HALO + OUTF) ? out[(lf - HALO) * ldf + c]
                                                : sm.ext[lf < HALO ? lf : lf - OUTF][c];
    }
  }
  lds_order();
  // delta(feat, 2) (speaker_identification.py:141-151): edge padding clamps to the TRUE sequence
  // [0, T - 1]; delta-delta is the delta of the delta sequence, edge-padded again
  auto cv = [&](int g, int c) {
    g = g < 0 ? 0 : (g > T - 1 ? T - 1 : g);
    return (double)C[(g - lbase) * 13 + c];
  };
  auto dl = [&](int g, int c) {
    g = g < 0 ? 0 : (g > T - 1 ? T - 1 : g);
    return (-2.0 * cv(g - 2, c) - cv(g - 1, c) + cv(g + 1, c) + 2.0 * cv(g + 2, c)) * 0.1;
  };
  constexpr int EPL = OUTF * 13 / NT;   // 52 elements per lane per column group
#pragma unroll 4
  for (int i = 0; i < EPL; ++i) {
    const int e = lane + NT * i;
    const int t = e / 13, c = e - t * 13;
    const int g = lbase + HALO + t;   // frame0 + t, window-relative
    float* o = out + t * ldf + c;
    if (ldf == 40 && c == 12) o[27] = 0.0f;   // the pad column 39 (t * 40 + 39)
    float v0 = 0.0f, v1 = 0.0f, v2 = 0.0f;
    if (g < T) {
      v0 = C[(t + HALO) * 13 + c];
      v1 = (float)dl(g, c);
      double d2;
      if (g >= 4 && g + 4 <= T - 1) {   // interior: the 9-tap composition of the two deltas
        const float* cc = C + (t + HALO - 4) * 13 + c;
        d2 = 0.04 * ((double)cc[0] + (double)cc[13] + (double)cc[91] + (double)cc[104]) +
             0.01 * ((double)cc[26] + (double)cc[78]) -
             0.04 * ((double)cc[39] + (double)cc[65]) - 0.1 * (double)cc[52];
      } else {
        d2 = (-2.0 * dl(g - 2, c) - dl(g - 1, c) + dl(g + 1, c) + 2.0 * dl(g + 2, c)) * 0.1;
      }
      v2 = (float)d2;
    }
    o[0] = v0;
    o[13] = v1;
    o[26] = v2;
  }
}

}  // namespace v2

}  // namespace

hipError_t si_fe_launch(const SiFeArgs& a, int64_t n_clips, hipStream_t stream) {
  if (n_clips <= 0) return hipSuccess;
  hipLaunchKernelGGL(v2::si_fe_kernel, dim3((unsigned)n_clips), dim3(v2::NT), 0, stream, a);
  return hipGetLastError();
}

bool si_fe_tables_ok(const SiFeTables& t) {
  if (t.n_sub < 1 || t.n_sub > SI_FE_MAX_SUB || v2::R * t.n_sub > 3 * v2::NT) return false;
  for (int s = 0; s < 27; ++s) {   // a filter edge spans <= 4 sub-segments (the unrolled loops)
    const int n = t.seg_sub[s + 1] - t.seg_sub[s];
    if (n < 1 || n > 4) return false;
  }
  return true;
}

void si_fe_build_tables(SiFeTables* t) {
  const double PI = 3.14159265358979323846;
  for (int n2 = 0; n2 < 16; ++n2)
    for (int k1 = 0; k1 < 16; ++k1) {
      t->w256[n2][k1][0] = cos(2.0 * PI * n2 * k1 / 256.0);
      t->w256[n2][k1][1] = -sin(2.0 * PI * n2 * k1 / 256.0);
    }
  for (int e = 0; e < 16; ++e) {
    t->w16[e][0] = cos(2.0 * PI * e / 16.0);
    t->w16[e][1] = -sin(2.0 * PI * e / 16.0);
  }
  for (int k = 0; k <= 256; ++k) {
    t->w512[k][0] = cos(2.0 * PI * k / 512.0);
    t->w512[k][1] = -sin(2.0 * PI * k / 512.0);
  }
  // psf.get_filterbanks(26, 512, 16000, 0, 8000): bins = floor(513 * mel2hz(linspace) / 16000)
  auto hz2mel = [](double hz) { return 2595 * log10(1 + hz / 700.); };
  auto mel2hz = [](double mel) { return 700 * (pow(10.0, mel / 2595.0) - 1); };
  double bin[28];
  const double lo = hz2mel(0.0), hi = hz2mel(8000.0);
  for (int i = 0; i < 28; ++i) {
    const double step = (hi - lo) / 27;
    const double m = i == 27 ? hi : lo + i * step;
    bin[i] = floor((512 + 1) * mel2hz(m) / 16000);
  }
  for (int j = 0; j < 26; ++j) {
    t->fb_lo[j] = (int)bin[j];
    t->fb_hi[j] = (int)bin[j + 2];
    for (int i = 0; i < 48; ++i) t->fb_w[j][i] = 0.0;
    for (int i = (int)bin[j]; i < (int)bin[j + 1]; ++i)
      t->fb_w[j][i - (int)bin[j]] = (i - bin[j]) / (bin[j + 1] - bin[j]);
    for (int i = (int)bin[j + 1]; i < (int)bin[j + 2]; ++i)
      t->fb_w[j][i - (int)bin[j]] = (bin[j + 2] - i) / (bin[j + 2] - bin[j + 1]);
  }
  // v2 segments [bin[s], bin[s+1]) cut into <= 8-bin sub-segments
  int n = 0;
  for (int s = 0; s < 27; ++s) {
    const int b0 = (int)bin[s], b1 = (int)bin[s + 1];
    t->seg_sub[s] = n;
    t->inv_w[s] = b1 > b0 ? 1.0 / (b1 - b0) : 0.0;
    for (int st = b0; st < b1 && n < SI_FE_MAX_SUB; st += 8, ++n) {
      t->sub_start[n] = st;
      t->sub_cnt[n] = b1 - st < 8 ? b1 - st : 8;
      t->sub_d0[n] = st - b0;
    }
  }
  t->seg_sub[27] = n;
  t->n_sub = n;
  for (int u = n; u < SI_FE_MAX_SUB; ++u) t->sub_start[u] = t->sub_cnt[u] = t->sub_d0[u] = 0;
  // scipy.fftpack.dct(type=2, norm='ortho'), rows 1..12 (sqrt(2/N) scale), times the lifter
  for (int c = 0; c < 13; ++c) {
    const double lift = 1 + (22 / 2.) * sin(PI * c / 22);
    for (int j = 0; j < 26; ++j) {
      const double s = c == 0 ? sqrt(1.0 / 26) : sqrt(2.0 / 26);
      t->dct[c][j] = lift * s * cos(PI * c * (2 * j + 1) / (2.0 * 26));
    }
  }
}
