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
// One workgroup (256 threads) per clip; frames in tiles of 16.  512-point real FFT per frame as a
// 256-point complex FFT of (s[2n] + i s[2n+1]) factored 16 x 16, then the real split.
// Only min(T, 260) frames are computed: delta-delta of row 255 reaches feat[259].
#include "common.h"
#include "si_fe.h"

#pragma clang fp contract(off)   // match numpy's separately rounded float64 ops (preemphasis, etc.)

namespace {

constexpr int NT = 256;
constexpr int FT = 12;          // frames per tile: LDS 64 KB -> 2 workgroups per CU
constexpr int HALO = 4;              // delta-delta reach in frames
constexpr int OUTF = 256;
constexpr int NL = OUTF + 2 * HALO;  // local frames per window: [frame0 - 4, frame0 + 260)

struct Smem {
  cd buf[FT][256];      // pass A output -> (in place) Z -> (in place) power spectrum [f][258]
  double lfe[FT][28];   // log filterbank energies + log energy
  float feat[NL][13];   // cepstra (float64 math, stored float32: the deltas' inputs); the deltas
                        // themselves are recomputed per output element instead of staged
};

template <typename C>
MMLA_DEV void fft4c(C& a0, C& a1, C& a2, C& a3) {
  C s02 = cadd(a0, a2), d02 = csub(a0, a2), s13 = cadd(a1, a3), d13 = csub(a1, a3);
  a0 = cadd(s02, s13);
  a2 = csub(s02, s13);
  a1 = cadd(d02, cmul_negi(d13));
  a3 = csub(d02, cmul_negi(d13));
}

// complex 16-point DFT in registers, radix 4 x 4: in v[n], out v[4*q1 + q2] = Y[q1 + 4*q2]
MMLA_DEV void dft16(cd v[16], const double (*w16)[2]) {
#pragma unroll
  for (int m2 = 0; m2 < 4; ++m2) fft4c(v[m2], v[4 + m2], v[8 + m2], v[12 + m2]);
#pragma unroll
  for (int q1 = 1; q1 < 4; ++q1)
#pragma unroll
    for (int m2 = 1; m2 < 4; ++m2) {
      const int e = m2 * q1;   // W16^(m2 q1)
      const cd w = {w16[e][0], w16[e][1]};
      v[4 * q1 + m2] = cmul(v[4 * q1 + m2], w);
    }
#pragma unroll
  for (int q1 = 0; q1 < 4; ++q1) fft4c(v[4 * q1 + 0], v[4 * q1 + 1], v[4 * q1 + 2], v[4 * q1 + 3]);
}

// pre-emphasised sample s[i] = x[i] - 0.97 x[i-1] (s[0] = x[0]); 0 beyond the signal
MMLA_DEV double pre(const int16_t* x, int64_t i, int64_t len) {
  if (i >= len) return 0.0;
  return i == 0 ? (double)x[0] : (double)x[i] - 0.97 * (double)x[i - 1];
}

__global__ void __launch_bounds__(NT, 2) si_fe_kernel(SiFeArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  Smem& sm = *reinterpret_cast<Smem*>(smem_raw);
  const SiFeTables& tb = *a.tables;
  const int tid = threadIdx.x;
  const int64_t blk = blockIdx.x;
  float* out = a.feat + blk * (OUTF * 39);

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
      for (int e = tid; e < OUTF * 39; e += NT) out[e] = 0.0f;
      if (a.silent && tid == 0) a.silent[blk] = 1;
      return;
    }
    if (a.silent && tid == 0) a.silent[blk] = 0;
  }
  const int64_t T = len <= 400 ? 1 : 1 + (len - 400 + 159) / 160;   // framesig numframes
  // local frame lf <-> global frame g = frame0 - HALO + lf, computed where 0 <= g < T
  const int64_t g_lo = frame0 - HALO < 0 ? 0 : frame0 - HALO;
  const int64_t g_hi = frame0 - HALO + NL < T ? frame0 - HALO + NL : T;
  const int nloc = (int)(g_hi - g_lo);
  const int lf0 = (int)(g_lo - (frame0 - HALO));
  double* pw = reinterpret_cast<double*>(&sm.buf[0][0]);

  for (int t0 = 0; t0 < nloc; t0 += FT) {
    const int nfr = min(FT, nloc - t0);
    // pass A: task (f, n2): DFT-16 over n1 of z[16 n1 + n2], z[n] = s[2n] + i s[2n+1]
    for (int task = tid; task < nfr * 16; task += NT) {
      const int f = task >> 4, n2 = task & 15;
      const int64_t fs = 160 * (g_lo + t0 + f);
      cd v[16];
#pragma unroll
      for (int n1 = 0; n1 < 16; ++n1) {
        const int n = 16 * n1 + n2;
        const bool in = 2 * n < 400;   // rectangular 400-sample frame, zero-padded to 512
        v[n1] = {in ? pre(x, fs + 2 * n, len) : 0.0, in ? pre(x, fs + 2 * n + 1, len) : 0.0};
      }
      dft16(v, tb.w16);
#pragma unroll
      for (int q1 = 0; q1 < 4; ++q1)
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
          const int k1 = q1 + 4 * q2;
          const cd w = {tb.w256[n2][k1][0], tb.w256[n2][k1][1]};
          sm.buf[f][k1 * 16 + n2] = cmul(v[4 * q1 + q2], w);
        }
    }
    __syncthreads();
    // pass B (in place): task (f, k1): DFT-16 over n2 -> Z[k1 + 16 k2]
    {
      cd v[16];
      const int task = tid;
      const bool act = task < nfr * 16;
      const int f = task >> 4, k1 = task & 15;
      if (act) {
#pragma unroll
        for (int n2 = 0; n2 < 16; ++n2) v[n2] = sm.buf[f][k1 * 16 + n2];
        dft16(v, tb.w16);
      }
      __syncthreads();
      if (act) {
#pragma unroll
        for (int q1 = 0; q1 < 4; ++q1)
#pragma unroll
          for (int q2 = 0; q2 < 4; ++q2) sm.buf[f][k1 + 16 * (q1 + 4 * q2)] = v[4 * q1 + q2];
      }
    }
    __syncthreads();
    // pass C (in place): real split -> P[f][k] = |X[k]|^2 / 512, k = 0..256, at pw[f*258 + k]
    {
      constexpr int PER = (FT * 257 + NT - 1) / NT;
      double pv[PER];
#pragma unroll
      for (int r = 0; r < PER; ++r) {
        const int task = tid + NT * r;
        pv[r] = 0.0;
        if (task < nfr * 257) {
          const int f = task / 257, k = task - f * 257;
          const cd zk = sm.buf[f][k & 255];
          const cd zr = cconj(sm.buf[f][(256 - k) & 255]);
          const cd e = cscale(cadd(zk, zr), 0.5);
          const cd d = csub(zk, zr);
          const cd o = {0.5 * d.y, -0.5 * d.x};
          const cd w = {tb.w512[k][0], tb.w512[k][1]};
          const cd X = cadd(e, cmul(w, o));
          // numpy: square(absolute(X)) / 512 with absolute = hypot; x^2 + y^2 differs from
          // hypot^2 by an ulp (no fp64 sqrt/div on the hot path)
          const double mag2 = X.x * X.x + X.y * X.y;
          pv[r] = mag2 * (1.0 / 512.0);
        }
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < PER; ++r) {
        const int task = tid + NT * r;
        if (task < nfr * 257) {
          const int f = task / 257, k = task - f * 257;
          pw[f * 258 + k] = pv[r];
        }
      }
    }
    __syncthreads();
    // pass D: 26 filterbank energies + frame energy -> log (0 -> eps)
    for (int task = tid; task < nfr * 27; task += NT) {
      const int f = task / 27, j = task - f * 27;
      const double* p = pw + f * 258;
      double acc = 0.0;
      if (j < 26) {
        const int lo = tb.fb_lo[j], n = tb.fb_hi[j] - lo;
        for (int i = 0; i < n; ++i) acc += tb.fb_w[j][i] * p[lo + i];
      } else {
        for (int i = 0; i < 257; ++i) acc += p[i];
      }
      if (acc == 0.0) acc = 2.220446049250313e-16;   // numpy.finfo(float).eps
      sm.lfe[f][j] = log(acc);
    }
    __syncthreads();
    // pass E: DCT-II ortho x lifter for c = 1..12; c0 = log(energy)
    for (int task = tid; task < nfr * 13; task += NT) {
      const int f = task / 13, c = task - f * 13;
      double v;
      if (c == 0) {
        v = sm.lfe[f][26];
      } else {
        v = 0.0;
        for (int j = 0; j < 26; ++j) v += sm.lfe[f][j] * tb.dct[c][j];
      }
      sm.feat[lf0 + t0 + f][c] = (float)v;
    }
    __syncthreads();
  }

  // delta(feat, 2): d[g] = (-2 f[g-2] - f[g-1] + f[g+1] + 2 f[g+2]) / 10, edges clamped to the
  // TRUE sequence [0, T-1] (speaker_identification.py:147 np.pad mode='edge').
  auto loc = [&](int64_t g) {
    g = g < 0 ? 0 : (g > T - 1 ? T - 1 : g);
    return (int)(g - (frame0 - HALO));
  };
  // delta of feat column c at global frame g (g clamped by the caller)
  auto dfe = [&](int64_t g, int c) {
    const double v = -2.0 * (double)sm.feat[loc(g - 2)][c] - 1.0 * (double)sm.feat[loc(g - 1)][c] +
                     1.0 * (double)sm.feat[loc(g + 1)][c] + 2.0 * (double)sm.feat[loc(g + 2)][c];
    return v / 10.0;
  };
  auto clampg = [&](int64_t g) { return g < 0 ? (int64_t)0 : (g > T - 1 ? T - 1 : g); };
  for (int e = tid; e < OUTF * 39; e += NT) {
    const int t = e / 39, c = e - t * 39;
    const int64_t g = frame0 + t;
    float v = 0.0f;
    if (g < T) {
      if (c < 13) {
        v = sm.feat[loc(g)][c];
      } else if (c < 26) {
        v = (float)dfe(g, c - 13);
      } else {
        // delta of the delta sequence, itself edge-padded at the true ends
        const int cc = c - 26;
        const double d = -2.0 * dfe(clampg(g - 2), cc) - 1.0 * dfe(clampg(g - 1), cc) +
                         1.0 * dfe(clampg(g + 1), cc) + 2.0 * dfe(clampg(g + 2), cc);
        v = (float)(d / 10.0);
      }
    }
    out[e] = v;
  }
}

}  // namespace

hipError_t si_fe_launch(const SiFeArgs& a, int64_t n_clips, hipStream_t stream) {
  if (n_clips <= 0) return hipSuccess;
  const size_t smem = sizeof(Smem);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(si_fe_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(si_fe_kernel, dim3((unsigned)n_clips), dim3(NT), smem, stream, a);
  return hipGetLastError();
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
  // scipy.fftpack.dct(type=2, norm='ortho'), rows 1..12 (sqrt(2/N) scale), times the lifter
  for (int c = 0; c < 13; ++c) {
    const double lift = 1 + (22 / 2.) * sin(PI * c / 22);
    for (int j = 0; j < 26; ++j) {
      const double s = c == 0 ? sqrt(1.0 / 26) : sqrt(2.0 / 26);
      t->dct[c][j] = lift * s * cos(PI * c * (2 * j + 1) / (2.0 * 26));
    }
  }
}
