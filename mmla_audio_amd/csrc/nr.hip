// Stationary spectral-gate noise reduction on gfx950, float64 like the
// reference's chunk buffers.
//
// Replaces nr.reduce_noise(y_noise=noise, y=y, sr=sr, stationary=True)
//   OverlapDetection/scripts/record_on_pc.py:208-212, SpeakerIdentification/scripts/record_on_pc.py:189,
//   speaker_identification_post_processing.py:171, record_on_pi.py:112
// i.e. noisereduce 2.0.x SpectralGateStationary on librosa 0.8 stft/istft (oracle/noisereduce.py).
//
// Work unit = one "item": a buffer of L = chunk + 2 * padding samples read from a float32 signal
// (zeros outside it), exactly the float64 buffer SpectralGate._read_chunk builds.  All items of a
// launch share L, so an item has T = 1 + L / 256 STFT frames (n_fft 1024, hop 256, centre reflect).
//   nr_stft_kernel     one wave per (item, frame): 1024-point real DFT as a 512-point complex FFT
//                      of the even/odd-packed frame (radix 8 x 8 x 8 in LDS) + real split -> S[513]
//                      (complex128 to HBM), mask bit dB > thresh per bin, the frame's max dB; frames
//                      whose window only covers zeros skip the FFT (S = 0, dB = 10 log10(1e-40))
//   nr_rows_kernel     one wave per (item, frame) within 3 frames of the kept interior: the item's
//                      max dB, the frame's mask row OR'ed with (max - 80 > thresh) (top_db clamp),
//                      smoothed over frequency (33 taps; the filter is separable) -> HBM row
//   nr_gate_kernel     one wave per (item, frame) touching the kept interior: the time smoothing
//                      of rows t-3..t+3 (7 taps, zero outside the array like fftconvolve 'same'),
//                      S * mask, inverse real FFT, x window -> the frame in the time domain
//   nr_ola_kernel      overlap-add of the <= 4 frames covering each kept sample, / window
//                      sum-square, float32 out
// The noise profile (per-bin threshold) is computed once per noise clip by nr_noise_db_kernel +
// nr_noise_thresh_kernel in the reference's float32 arithmetic.
#include "common.h"
#include "nr.h"

#include <algorithm>

#include <cmath>
#include <vector>

namespace {

constexpr int NT = 64;
constexpr int NFFT = NR_NFFT;       // 1024
constexpr int HOP = NR_HOP;         // 256
constexpr int NB = NFFT / 2 + 1;    // 513 bins
constexpr int NG_F = NR_NGF;        // 33 frequency taps
constexpr int NG_T = NR_NGT;        // 7 time taps
constexpr int KPL = (NB + 63) / 64;  // bins per lane (k = lane + 64 i)

// complex 8-point DFT in registers (W8^(nk)), in/out natural order
MMLA_DEV void dft8(cd v[8]) {
  const double r = 0.70710678118654752440;
  cd a[4], b[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    a[k] = cadd(v[k], v[k + 4]);
    b[k] = csub(v[k], v[k + 4]);
  }
  b[1] = cmul(b[1], cd{r, -r});
  b[2] = cmul_negi(b[2]);
  b[3] = cmul(b[3], cd{-r, -r});
  // two 4-point DFTs
  auto dft4 = [](cd& x0, cd& x1, cd& x2, cd& x3) {
    const cd s02 = cadd(x0, x2), d02 = csub(x0, x2), s13 = cadd(x1, x3), d13 = csub(x1, x3);
    x0 = cadd(s02, s13);
    x2 = csub(s02, s13);
    x1 = cadd(d02, cmul_negi(d13));
    x3 = csub(d02, cmul_negi(d13));
  };
  dft4(a[0], a[1], a[2], a[3]);
  dft4(b[0], b[1], b[2], b[3]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = a[k];
    v[2 * k + 1] = b[k];
  }
}

MMLA_DEV void lds_order() { asm volatile("" ::: "memory"); }

// In-place forward 512-point complex FFT of buf (one wave; LDS ops of a wave execute in order).
// n = 64 n1 + 8 n2 + n3, k = k1 + 8 k2 + 64 k3; tw[m] = W512^m.
MMLA_DEV void fft512(cd* buf, const cd* tw, int lane) {
  cd v[8];
  // this lane's 14 twiddles, all loads issued before the first pass
  cd t1[8], t2[8];
#pragma unroll
  for (int k = 1; k < 8; ++k) {
    t1[k] = tw[(lane * k) & 511];
    t2[k] = tw[(8 * (lane & 7) * k) & 511];
  }
  // pass 1: lane = 8 n2 + n3, DFT-8 over n1, x W512^(lane k1) -> buf[64 k1 + lane]
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = buf[64 * i + lane];
  lds_order();
  dft8(v);
#pragma unroll
  for (int k1 = 0; k1 < 8; ++k1) buf[64 * k1 + lane] = k1 ? cmul(v[k1], t1[k1]) : v[0];
  lds_order();
  // pass 2: lane = 8 k1 + n3, DFT-8 over n2 of buf[64 k1 + 8 n2 + n3], x W64^(n3 k2)
  {
    const int k1 = lane >> 3, n3 = lane & 7;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = buf[64 * k1 + 8 * i + n3];
    lds_order();
    dft8(v);
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2)
      buf[64 * k1 + 8 * k2 + n3] = k2 ? cmul(v[k2], t2[k2]) : v[0];
  }
  lds_order();
  // pass 3: lane = 8 k1 + k2, DFT-8 over n3 -> Z[k1 + 8 k2 + 64 k3]; written back in natural order
  {
    const int k1 = lane >> 3, k2 = lane & 7;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = buf[64 * k1 + 8 * k2 + i];
    lds_order();
    dft8(v);
#pragma unroll
    for (int k3 = 0; k3 < 8; ++k3) buf[k1 + 8 * k2 + 64 * k3] = v[k3];
  }
  lds_order();
}

// Workgroups are dealt to the 8 XCDs round-robin (block b -> XCD b % 8): give each XCD one
// contiguous range of the launch's frames, so neighbouring frames -- which share the overlapping
// signal samples and the 7 smoothing rows -- meet in the same L2.  -1: past the last frame.
constexpr int NXCD = 8;
MMLA_DEV int64_t frame_of_block(const NrArgs& a) {
  const int64_t total = a.n_items * a.t_n, per = (total + NXCD - 1) / NXCD;
  const int64_t f = (int64_t)(blockIdx.x % NXCD) * per + blockIdx.x / NXCD;
  return f < total ? f : -1;
}

MMLA_DEV double db_of_power(double p) { return 10.0 * log10(fmax(1e-40, p)); }

// frame t of the item's buffer: 1024 centred samples, reflect at the buffer edges, zeros outside
// the signal; returns whether any sample is nonzero (wave-uniform)
MMLA_DEV bool load_frame(const NrArgs& a, const NrItem& it, int t, cd* buf, int lane) {
  const float* y = a.y + it.sig_off;
  const double* win = a.tables->win;
  bool nz = false;
#pragma unroll
  for (int m = lane; m < NFFT / 2; m += NT) {
    double v[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      int64_t u = (int64_t)HOP * t - NFFT / 2 + 2 * m + e;     // buffer index before reflect
      if (u < 0) u = -u;
      if (u >= a.L) u = 2 * (a.L - 1) - u;
      const int64_t i = it.i1 + u;                           // signal index
      const double x = (i >= 0 && i < it.n) ? (double)y[i] : 0.0;
      nz |= x != 0.0;
      v[e] = x * win[2 * m + e];
    }
    buf[m] = cd{v[0], v[1]};
  }
  return __any(nz);
}

}  // namespace

// ---- signal STFT: S, mask bits, frame max dB ------------------------------------------------------
__global__ void __launch_bounds__(NT) nr_stft_kernel(NrArgs a) {
  __shared__ cd buf[512];
  const int lane = threadIdx.x;
  const int64_t fr = frame_of_block(a);
  if (fr < 0) return;
  const int64_t item = fr / a.t_n;
  const int t = a.t_lo + (int)(fr - item * a.t_n);
  const NrItem it = a.items[item];
  const NrTables& tb = *a.tables;
  double2* S = a.S + (item * a.T + t) * NB;
  uint8_t* bits = a.bits + (item * a.T + t) * NB;
  double mx = -INFINITY;
  if (!load_frame(a, it, t, buf, lane)) {
    // a window of zeros: its mask bits are read by the smoothing rows of frames within NG_T / 2
    // of the kept interior; S = 0 is read by nr_gate_kernel when the frame itself reaches the
    // interior (a run of >= 1024 zero samples inside the signal), so it is written then -- the
    // scratch holds the previous call's spectra
    const double dz = db_of_power(0.0);
    const int64_t f_lo = (int64_t)HOP * (t - NG_T / 2) - NFFT / 2, f_hi = (int64_t)HOP * (t + NG_T / 2) + NFFT / 2;
    if (f_lo < a.keep0 + a.keep_len && f_hi > a.keep0)
      for (int k = lane; k < NB; k += NT) bits[k] = dz > (double)a.thresh[k];
    const int64_t g_lo = (int64_t)HOP * t - NFFT / 2, g_hi = (int64_t)HOP * t + NFFT / 2;
    if (g_lo < a.keep0 + a.keep_len && g_hi > a.keep0)
      for (int k = lane; k < NB; k += NT) S[k] = double2{0.0, 0.0};
    mx = dz;
  } else {
    // the split's per-bin tables (bins k = lane + 64 i), loaded under the FFT
    cd wk[KPL];
    float th[KPL];
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      const int k = min(lane + NT * i, NB - 1);
      wk[i] = cd{tb.w1024[k][0], tb.w1024[k][1]};
      th[i] = a.thresh[k];
    }
    lds_order();
    fft512(buf, tb.w512, lane);
    // real split: X[k] = (Z[k] + conj Z[512-k]) / 2 - i W1024^k (Z[k] - conj Z[512-k]) / 2
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      const int k = lane + NT * i;
      if (k >= NB) continue;
      const cd z = buf[k & 511], zr = buf[(512 - k) & 511];
      const cd e = {0.5 * (z.x + zr.x), 0.5 * (z.y - zr.y)};
      const cd o = {0.5 * (z.y + zr.y), -0.5 * (z.x - zr.x)};
      const cd X = cadd(e, cmul(wk[i], o));
      S[k] = double2{X.x, X.y};
      const double db = db_of_power(X.x * X.x + X.y * X.y);
      bits[k] = db > (double)th[i];
      mx = fmax(mx, db);
    }
  }
  mx = wave_max(mx);
  if (lane == 0) a.fmax[item * a.T + t] = mx;
}

// frames whose smoothed mask the gate needs: those within NG_T / 2 of a frame reaching the kept
// interior [keep0, keep0 + keep_len) of the buffer
MMLA_DEV bool reaches(const NrArgs& a, int64_t t, int halo) {
  const int64_t f_lo = (int64_t)HOP * (t - halo) - NFFT / 2, f_hi = (int64_t)HOP * (t + halo) + NFFT / 2;
  return f_lo < a.keep0 + a.keep_len && f_hi > a.keep0;
}

// ---- the item's max dB over all frames (amplitude_to_db's top_db reference): frames outside the
// launched range [t_lo, t_lo + t_n) are all-zero windows, whose dB (-400) no frame is below ----------
__global__ void __launch_bounds__(NT) nr_gmax_kernel(NrArgs a) {
  const int64_t item = blockIdx.x;
  double gm = -INFINITY;
  for (int i = a.t_lo + threadIdx.x; i < a.t_lo + a.t_n; i += NT) gm = fmax(gm, a.fmax[item * a.T + i]);
  gm = wave_max(gm);
  if (threadIdx.x == 0) a.gmax[item] = gm;
}

// ---- mask row (dB > th OR top_db floor > th), smoothed over frequency: once per frame ---------------
__global__ void __launch_bounds__(NT) nr_rows_kernel(NrArgs a) {
  __shared__ __attribute__((aligned(16))) float mrow[NB + NG_F];   // 16 zero bins each side
  const int lane = threadIdx.x;
  const int64_t fr = frame_of_block(a);
  if (fr < 0) return;
  const int64_t item = fr / a.t_n;
  const int t = a.t_lo + (int)(fr - item * a.t_n);
  if (!reaches(a, t, NG_T / 2)) return;
  const NrTables& tb = *a.tables;
  constexpr int HF = NG_F / 2;
  // the item's max dB (nr_gmax_kernel) -> the top_db floor c; mask = max(dB, c) > th
  // = (dB > th) | (c > th)
  const double c = a.gmax[item] - 80.0;
  const double p = a.prop_decrease;
  const uint8_t* br = a.bits + (item * a.T + t) * NB;
  constexpr int MPL = (NB + 2 * HF + NT - 1) / NT;   // 9
  uint8_t bv[MPL];
  float thv[MPL];
#pragma unroll
  for (int i = 0; i < MPL; ++i) {                   // all loads first
    const int kb = min(max(lane + NT * i - HF, 0), NB - 1);
    bv[i] = br[kb];
    thv[i] = a.thresh[kb];
  }
  double g[NG_F];
#pragma unroll
  for (int j = 0; j < NG_F; ++j) g[j] = tb.gf[j];
#pragma unroll
  for (int i = 0; i < MPL; ++i) {
    const int k = lane + NT * i, kb = k - HF;
    if (k >= NB + 2 * HF) continue;
    float v = 0.0f;
    if (kb >= 0 && kb < NB) {
      const bool m = bv[i] || c > (double)thv[i];
      v = (float)((m ? 1.0 : 0.0) * p + (1.0 - p));     // exact in float for p = 1 (0 / 1)
    }
    mrow[k] = v;
  }
  lds_order();
  // lane: bins 8 lane .. 8 lane + 7 from the 40 mask values mrow[8 lane .. 8 lane + 39] (ten
  // 16-B reads); bin 512 by lane 0.  Same summation order as the direct 33-tap sum.
  double* row = a.rows + (item * a.T + t) * NB;
  {
    float m[8 + NG_F - 1];
    const float4* m4 = reinterpret_cast<const float4*>(mrow + 8 * lane);
#pragma unroll
    for (int q = 0; q < (8 + NG_F - 1) / 4; ++q) {
      const float4 u = m4[q];
      m[4 * q] = u.x;
      m[4 * q + 1] = u.y;
      m[4 * q + 2] = u.z;
      m[4 * q + 3] = u.w;
    }
    double o[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      double sacc = 0.0;
#pragma unroll
      for (int j = 0; j < NG_F; ++j) sacc = fma(g[j], (double)m[b + j], sacc);
      o[b] = sacc;
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) row[8 * lane + b] = o[b];
    if (lane == 0) {
      double sacc = 0.0;
#pragma unroll
      for (int j = 0; j < NG_F; ++j) sacc = fma(g[j], (double)mrow[512 + j], sacc);
      row[512] = sacc;
    }
  }
}

// ---- time smoothing of the rows x S -> inverse FFT -> windowed time-domain frame ------------------
__global__ void __launch_bounds__(NT) nr_gate_kernel(NrArgs a) {
  __shared__ cd buf[512];
  __shared__ double msk[NB];
  const int lane = threadIdx.x;
  const int64_t fr = frame_of_block(a);
  if (fr < 0) return;
  const int64_t item = fr / a.t_n;
  const int t = a.t_lo + (int)(fr - item * a.t_n);
  if (!reaches(a, t, 0)) return;
  const NrTables& tb = *a.tables;
  constexpr int HT = NG_T / 2;
  const double* rows[NG_T];                          // rows t-3..t+3 (zero outside [0, T))
  bool rin[NG_T];
#pragma unroll
  for (int j = 0; j < NG_T; ++j) {
    const int tr = t + j - HT;
    rin[j] = tr >= 0 && tr < a.T;
    rows[j] = a.rows + (item * a.T + (rin[j] ? tr : 0)) * NB;
  }
  const double2* S = a.S + (item * a.T + t) * NB;
  // the time-smoothed mask of the frame, once per bin (the gate reads bins k and 512 - k); the
  // rows' loads are all issued before the first FMA, S and the twiddles right behind them
  double gt[NG_T];
#pragma unroll
  for (int j = 0; j < NG_T; ++j) gt[j] = tb.gt[j];
  {
    double rv[KPL][NG_T];
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      const int k = min(lane + NT * i, NB - 1);
#pragma unroll
      for (int j = 0; j < NG_T; ++j) rv[i][j] = rows[j][k];
    }
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      const int k = lane + NT * i;
      double mk = 0.0;
#pragma unroll
      for (int j = 0; j < NG_T; ++j)
        if (rin[j]) mk = fma(gt[j], rv[i][j], mk);
      if (k < NB) msk[k] = mk;
    }
  }
  constexpr int ZPL = 512 / NT;   // 8
  double2 s0v[ZPL], s1v[ZPL];
  cd wcv[ZPL];
#pragma unroll
  for (int i = 0; i < ZPL; ++i) {
    const int k = lane + NT * i;
    s0v[i] = S[k];
    s1v[i] = S[512 - k];
    wcv[i] = cd{tb.w1024[k][0], -tb.w1024[k][1]};                       // W1024^-k
  }
  lds_order();
  // gated spectrum -> Z[k] = E[k] + i O[k] of the inverse real FFT (k = 0..511)
#pragma unroll
  for (int i = 0; i < ZPL; ++i) {
    const int k = lane + NT * i;
    const double mk = msk[k], mr = msk[512 - k];
    const double2 s0 = s0v[i], s1 = s1v[i];
    const cd X = {s0.x * mk, s0.y * mk}, Xr = {s1.x * mr, s1.y * mr};   // X[k], X[512 - k]
    const cd e = {0.5 * (X.x + Xr.x), 0.5 * (X.y - Xr.y)};             // (X[k] + conj X[512-k]) / 2
    const cd d = {0.5 * (X.x - Xr.x), 0.5 * (X.y + Xr.y)};             // (X[k] - conj X[512-k]) / 2
    const cd wc = wcv[i];
    const cd o = cmul(d, wc);                                          // O[k]
    // conj(Z) for the forward FFT used as an inverse: Z = E + i O
    const cd Z = {e.x - o.y, e.y + o.x};
    buf[k] = cd{Z.x, -Z.y};
  }
  lds_order();
  fft512(buf, tb.w512, lane);
  // z[n] = conj(FFT(conj Z))[n] / 512 = x[2n] + i x[2n+1]; windowed frame to HBM
  double* out = a.frames + (item * a.T + t) * NFFT;
#pragma unroll
  for (int n = lane; n < 512; n += NT) {
    const cd z = buf[n];
    const double x0 = z.x * (1.0 / 512.0), x1 = -z.y * (1.0 / 512.0);
    out[2 * n] = x0 * tb.win[2 * n];
    out[2 * n + 1] = x1 * tb.win[2 * n + 1];
  }
}

// ---- overlap-add, window-sum-square normalisation, float32 out -------------------------------------
__global__ void nr_ola_kernel(NrArgs a) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t item = gid / a.keep_len;
  if (item >= a.n_items) return;
  const int64_t i = gid - item * a.keep_len;
  const NrItem it = a.items[item];
  if (i >= it.out_len) return;
  const int64_t j = a.keep0 + i + NFFT / 2;            // index into the untrimmed istft signal
  int64_t t0 = (j - (NFFT - 1) + HOP - 1) / HOP;
  if (j - (NFFT - 1) < 0) t0 = 0;
  int64_t t1 = j / HOP;
  if (t1 > a.T - 1) t1 = a.T - 1;
  double acc = 0.0, wss = 0.0;
  for (int64_t t = t0; t <= t1; ++t) {
    const int off = (int)(j - HOP * t);
    acc += a.frames[(item * a.T + t) * NFFT + off];
    const double w = a.tables->win[off];
    wss += w * w;
  }
  if (wss > 2.2250738585072014e-308) acc /= wss;
  a.out[it.out_off + i] = (float)acc;
}

// ---- noise profile ----------------------------------------------------------------------------
// float32 like the reference: librosa.load gives float32, so stft -> complex64, |X| (hypotf),
// square, 10 log10(max(1e-40, .)) in float32; the global max / top_db clamp and the per-bin
// mean / std over frames follow in nr_noise_thresh_kernel.
__global__ void __launch_bounds__(NT) nr_noise_db_kernel(const float* noise, int64_t m, int Tn,
                                                         const NrTables* tables, float* db,
                                                         float* fmaxv) {
  __shared__ cd buf[512];
  const int lane = threadIdx.x;
  const int t = blockIdx.x;
  const NrTables& tb = *tables;
  for (int q = lane; q < 512; q += NT) {
    double v[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      int64_t u = (int64_t)HOP * t - NFFT / 2 + 2 * q + e;
      if (u < 0) u = -u;
      if (u >= m) u = 2 * (m - 1) - u;
      v[e] = (double)noise[u] * tb.win[2 * q + e];
    }
    buf[q] = cd{v[0], v[1]};
  }
  lds_order();
  fft512(buf, tb.w512, lane);
  float mx = -INFINITY;
  for (int k = lane; k < NB; k += NT) {
    const cd z = buf[k & 511], zr = buf[(512 - k) & 511];
    const cd e = {0.5 * (z.x + zr.x), 0.5 * (z.y - zr.y)};
    const cd o = {0.5 * (z.y + zr.y), -0.5 * (z.x - zr.x)};
    const cd w = {tb.w1024[k][0], tb.w1024[k][1]};
    const cd X = cadd(e, cmul(w, o));
    const float re = (float)X.x, im = (float)X.y;        // complex64 storage
    const float mag = hypotf(re, im);
    const float pw = mag * mag;
    const float d = 10.0f * log10f(fmaxf(1e-40f, pw));
    db[(int64_t)t * NB + k] = d;
    mx = fmaxf(mx, d);
  }
  mx = wave_max(mx);
  if (lane == 0) fmaxv[t] = mx;
}

__global__ void nr_noise_thresh_kernel(const float* db, const float* fmaxv, int Tn, float n_std,
                                       float* thresh) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= NB) return;
  float gm = -INFINITY;
  for (int t = 0; t < Tn; ++t) gm = fmaxf(gm, fmaxv[t]);
  const float c = gm - 80.0f;
  double s = 0.0;
  for (int t = 0; t < Tn; ++t) s += (double)fmaxf(db[(int64_t)t * NB + k], c);
  const float mean = (float)(s / Tn);
  double v = 0.0;
  for (int t = 0; t < Tn; ++t) {
    const float d = fmaxf(db[(int64_t)t * NB + k], c) - mean;
    v += (double)d * (double)d;
  }
  const float sd = sqrtf((float)(v / Tn));
  thresh[k] = mean + sd * n_std;
}

// ---- host --------------------------------------------------------------------------------------
void nr_build_tables(NrTables* t, int sr) {
  const double PI = 3.14159265358979323846;
  for (int n = 0; n < NFFT; ++n) t->win[n] = 0.5 - 0.5 * cos(2.0 * PI * n / NFFT);
  for (int m = 0; m < 512; ++m) {
    t->w512[m].x = cos(2.0 * PI * m / 512.0);
    t->w512[m].y = -sin(2.0 * PI * m / 512.0);
  }
  for (int k = 0; k < NB; ++k) {
    t->w1024[k][0] = cos(2.0 * PI * k / 1024.0);
    t->w1024[k][1] = -sin(2.0 * PI * k / 1024.0);
  }
  // noisereduce _smoothing_filter(n_grad_freq, n_grad_time) = outer(f, g) / sum: separable into
  // f / sum(f) and g / sum(g) (SpectralGate._generate_mask_smoothing_filter: 500 Hz, 50 ms)
  const int ngf = (int)(500.0 / (sr / (NFFT / 2.0))), ngt = (int)(50.0 / ((double)HOP / sr * 1000.0));
  auto ramp = [](int ng, std::vector<double>& out) {
    std::vector<double> v;
    for (int i = 0; i < ng + 1; ++i) v.push_back((double)i / (ng + 1));         // linspace(0,1,ng+1,endpoint=False)
    for (int i = 0; i < ng + 2; ++i) v.push_back(1.0 - (double)i / (ng + 1));   // linspace(1,0,ng+2)
    out.assign(v.begin() + 1, v.end() - 1);
  };
  std::vector<double> f, g;
  ramp(ngf, f);
  ramp(ngt, g);
  double sf = 0, sg = 0;
  for (double v : f) sf += v;
  for (double v : g) sg += v;
  t->ngf = (int)f.size();
  t->ngt = (int)g.size();
  for (int j = 0; j < NG_F; ++j) t->gf[j] = j < (int)f.size() ? f[j] / sf : 0.0;
  for (int j = 0; j < NG_T; ++j) t->gt[j] = j < (int)g.size() ? g[j] / sg : 0.0;
}

hipError_t nr_noise_launch(const float* noise, int64_t m, const NrTables* tables, float* db_scratch,
                           float* fmax_scratch, float n_std, float* thresh, hipStream_t s) {
  const int Tn = (int)(1 + m / HOP);
  hipLaunchKernelGGL(nr_noise_db_kernel, dim3(Tn), dim3(NT), 0, s, noise, m, Tn, tables, db_scratch,
                     fmax_scratch);
  hipLaunchKernelGGL(nr_noise_thresh_kernel, dim3((NB + 63) / 64), dim3(64), 0, s, db_scratch,
                     fmax_scratch, Tn, n_std, thresh);
  return hipGetLastError();
}

void nr_frame_range(const NrItem* items, int64_t n_items, int64_t L, int T, int64_t keep0,
                    int64_t keep_len, int* t_lo, int* t_hi) {
  // frame t reads buffer samples [HOP t - NFFT/2, HOP t + NFFT/2), reflected into [0, L)
  const int64_t H = NG_T / 2;
  int64_t lo = std::max<int64_t>(0, (keep0 - NFFT / 2) / HOP - H - 1);
  int64_t hi = std::min<int64_t>(T - 1, (keep0 + keep_len + NFFT / 2) / HOP + H + 1);
  for (int64_t i = 0; i < n_items; ++i) {
    const int64_t s0 = std::max<int64_t>(0, -items[i].i1), s1 = std::min<int64_t>(L, items[i].n - items[i].i1);
    if (s1 <= s0) continue;
    lo = std::min<int64_t>(lo, s0 <= NFFT / 2 + 1 ? 0 : (s0 - NFFT / 2) / HOP - 1);
    hi = std::max<int64_t>(hi, s1 >= L - NFFT / 2 - 1 ? T - 1 : std::min<int64_t>(T - 1, (s1 + NFFT / 2) / HOP + 1));
  }
  *t_lo = (int)std::max<int64_t>(0, lo);
  *t_hi = (int)std::min<int64_t>(T - 1, hi);
}

hipError_t nr_gate_launch(const NrArgs& a, hipStream_t s) {
  if (a.n_items <= 0) return hipSuccess;
  const int64_t total = a.n_items * a.t_n;
  const unsigned frames = (unsigned)((total + NXCD - 1) / NXCD * NXCD);   // frame_of_block
  hipLaunchKernelGGL(nr_stft_kernel, dim3(frames), dim3(NT), 0, s, a);
  hipLaunchKernelGGL(nr_gmax_kernel, dim3((unsigned)a.n_items), dim3(NT), 0, s, a);
  hipLaunchKernelGGL(nr_rows_kernel, dim3(frames), dim3(NT), 0, s, a);
  hipLaunchKernelGGL(nr_gate_kernel, dim3(frames), dim3(NT), 0, s, a);
  const int64_t tot = a.n_items * a.keep_len;
  hipLaunchKernelGGL(nr_ola_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}
