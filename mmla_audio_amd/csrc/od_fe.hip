// OverlapDetection front-end: int16 PCM -> log-mel (librosa 0.8 semantics) + ZCR + model image.
//
// Replaces:
//   librosa.load + pad/trunc            overlap_features_generator.py:72-80,93-98
//   melspectrogram(n_fft 400, hop 160)  :81   (reflect-padded periodic-Hann STFT, Slaney mel)
//   power_to_db(ref=np.max, top_db=80)  :82
//   normalize_matrix                    :103-117
//   zero_crossing_rate(400, 160)        :100  (edge padding, signbit crossings)
//   generate_zcr_image + imsave + decode_png   :133-151, record_on_pc.py:156-158
//
// Layout / schedule (one workgroup = one clip, 512 threads = 8 waves, 2 per SIMD):
//   LDS: pcm int16[24000] (48 000 B) + STFT scratch (2 x FT*225 complex) + S f32[128][151]
//        (77 312 B) -> ~154 KB, one workgroup per CU.
//   The clip's normalisation needs the clip-global max/min of S, so all 151 frames of mel power
//   stay on chip and the outputs are written once, coalesced, after a block reduction.
// 400-point real DFT per frame, factored n = 25*n1 + n2, k = k1 + 16*k2:
//   pass 1 (25 tasks/frame): real 16-point DFT over n1 (via a complex 8-point FFT), k1 = 0..8,
//                            times W400^(n2*k1)
//   pass 2 (45 tasks/frame): 5-point DFTs over a (n2 = 5a + b), times W25^(b*c)
//   pass 3 (45 tasks/frame): 5-point DFTs over b -> X[k1 + 16*(c + 5d)] -> |X|^2; bins > 200
//                            fold onto 400 - k (conjugate symmetry) for k1 = 1..7
//   mel: sparse Slaney filterbank (394 non-zeros, <= 9 per band) from the per-frame power.
// Arithmetic is float32 (the reference runs the FFT in float64 and stores complex64; the measured
// deviation on the normalised log-mel is ~1e-6, tolerance 1e-4).  The scalar steps
// that the reference does in float64 (ref dB, image quantisation) are done in float64 here.
#include "common.h"
#include "od_fe.h"

namespace {

constexpr int N_FFT = 400;
constexpr int HOP = 160;
constexpr int CLIP = 24000;
constexpr int NF = 151;
constexpr int NMEL = 128;
constexpr int FT = 8;            // frames per STFT tile
constexpr int NT = 512;          // threads per workgroup
constexpr int NCHUNK = 305;      // ZCR: 80-sample chunks of the 24400-sample edge-padded signal

struct Smem {
  int16_t pcm[CLIP];
  cf t1[FT][9][25];              // pass-1 output  [frame][k1][n2]
  cf t2[FT][9][25];              // pass-2 output  [frame][k1][c*5+b]; pass 3 writes power into t1
  float s[NMEL][NF];             // mel power
  int cc[NCHUNK + 3];            // ZCR chunk counts
  int zc[NF];                    // ZCR counts per frame
  float red[2][NT / 64];
};

MMLA_DEV float sample(const Smem& sm, int i) {   // reflect padding of the 24000-sample clip
  i = i < 0 ? -i : i;
  i = i >= CLIP ? 2 * (CLIP - 1) - i : i;
  return (float)sm.pcm[i] * (1.0f / 32768.0f);
}

MMLA_DEV void fft4(cf& a0, cf& a1, cf& a2, cf& a3) {
  cf s02 = cadd(a0, a2), d02 = csub(a0, a2), s13 = cadd(a1, a3), d13 = csub(a1, a3);
  a0 = cadd(s02, s13);
  a2 = csub(s02, s13);
  a1 = cadd(d02, cmul_negi(d13));
  a3 = csub(d02, cmul_negi(d13));
}

// complex 8-point DFT in registers (radix-2 DIF + two 4-point DFTs)
MMLA_DEV void fft8(cf z[8]) {
  const float r = 0.70710678118654752f;
  cf a[4], b[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    a[k] = cadd(z[k], z[k + 4]);
    b[k] = csub(z[k], z[k + 4]);
  }
  b[1] = cmul(b[1], cf{r, -r});
  b[2] = cmul_negi(b[2]);
  b[3] = cmul(b[3], cf{-r, -r});
  fft4(a[0], a[1], a[2], a[3]);
  fft4(b[0], b[1], b[2], b[3]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    z[2 * k] = a[k];
    z[2 * k + 1] = b[k];
  }
}

MMLA_DEV void dft5(cf x0, cf x1, cf x2, cf x3, cf x4, cf y[5]) {
  const float c1 = 0.30901699437494742f, c2 = -0.80901699437494742f;
  const float s1 = 0.95105651629515357f, s2 = 0.58778525229247313f;
  cf a1 = cadd(x1, x4), b1 = csub(x1, x4), a2 = cadd(x2, x3), b2 = csub(x2, x3);
  y[0] = cadd(x0, cadd(a1, a2));
  cf p1 = {x0.x + c1 * a1.x + c2 * a2.x, x0.y + c1 * a1.y + c2 * a2.y};
  cf p2 = {x0.x + c2 * a1.x + c1 * a2.x, x0.y + c2 * a1.y + c1 * a2.y};
  cf q1 = {s1 * b1.x + s2 * b2.x, s1 * b1.y + s2 * b2.y};
  cf q2 = {s2 * b1.x - s1 * b2.x, s2 * b1.y - s1 * b2.y};
  y[1] = cadd(p1, cmul_negi(q1));
  y[4] = csub(p1, cmul_negi(q1));
  y[2] = cadd(p2, cmul_negi(q2));
  y[3] = csub(p2, cmul_negi(q2));
}

__global__ void __launch_bounds__(NT) od_fe_kernel(OdFeArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  Smem& sm = *reinterpret_cast<Smem*>(smem_raw);
  const OdFeTables& tb = *a.tables;
  const int tid = threadIdx.x;
  const int64_t clip = blockIdx.x;

  // ---- stage the clip (first 24000 samples, zero-padded) into LDS -------------------------------
  int len = a.lens ? a.lens[clip] : a.clip_len;
  len = len < 0 ? 0 : (len > CLIP ? CLIP : len);
  const int16_t* src = a.pcm + clip * a.clip_stride;
  if (len == CLIP && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(sm.pcm);
    for (int i = tid; i < CLIP / 8; i += NT) d4[i] = s4[i];
  } else {
    for (int i = tid; i < CLIP; i += NT) sm.pcm[i] = i < len ? src[i] : (int16_t)0;
  }
  __syncthreads();

  // ---- zero-crossing counts (edge-padded signal, padded index p <-> clip index clamp(p-200)) ----
  for (int q = tid; q < NCHUNK; q += NT) {
    int cnt = 0;
    int p0 = q * 80;
    int prev = p0 == 0 ? -1 : sm.pcm[min(max(p0 - 1 - 200, 0), CLIP - 1)] < 0;
    for (int j = 0; j < 80; ++j) {
      int p = p0 + j;
      int sgn = sm.pcm[min(max(p - 200, 0), CLIP - 1)] < 0;
      cnt += (prev >= 0) & (sgn != prev);
      prev = sgn;
    }
    sm.cc[q] = cnt;
  }
  __syncthreads();
  for (int f = tid; f < NF; f += NT) {
    // frame f covers padded [160 f, 160 f + 400): chunks 2f .. 2f+4, minus the change at 160 f
    int c = sm.cc[2 * f] + sm.cc[2 * f + 1] + sm.cc[2 * f + 2] + sm.cc[2 * f + 3] + sm.cc[2 * f + 4];
    int p = HOP * f;
    if (p > 0) {
      int s0 = sm.pcm[min(max(p - 1 - 200, 0), CLIP - 1)] < 0;
      int s1 = sm.pcm[min(max(p - 200, 0), CLIP - 1)] < 0;
      c -= (s0 != s1);
    }
    sm.zc[f] = c;
  }

  // ---- STFT -> power -> mel, FT frames per tile ---------------------------------------------------
  float smax = 0.0f, smin = INFINITY;
  for (int f0 = 0; f0 < NF; f0 += FT) {
    const int nfr = min(FT, NF - f0);
    // pass 1: real 16-point DFT over n1 of x[25 n1 + n2] * hann
    for (int task = tid; task < nfr * 25; task += NT) {
      const int f = task / 25, n2 = task - f * 25;
      const int base = HOP * (f0 + f) - N_FFT / 2;
      cf z[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int ne = 25 * (2 * m) + n2, no = 25 * (2 * m + 1) + n2;
        z[m] = {sample(sm, base + ne) * tb.hann[ne], sample(sm, base + no) * tb.hann[no]};
      }
      fft8(z);
#pragma unroll
      for (int k = 0; k <= 8; ++k) {
        cf zk = z[k & 7], zr = cconj(z[(8 - k) & 7]);
        cf e = cscale(cadd(zk, zr), 0.5f);
        cf d = csub(zk, zr);
        cf o = {0.5f * d.y, -0.5f * d.x};                     // d / (2i)
        cf w16 = {tb.w16[k][0], tb.w16[k][1]};
        cf y = cadd(e, cmul(w16, o));
        cf tw = {tb.w400[k][n2][0], tb.w400[k][n2][1]};
        sm.t1[f][k][n2] = cmul(y, tw);
      }
    }
    __syncthreads();
    // pass 2: DFT-5 over a of t1[k1][5a + b], times W25^(b c)
    for (int task = tid; task < nfr * 45; task += NT) {
      const int f = task / 45, r = task - f * 45, k1 = r / 5, b = r - k1 * 5;
      cf y[5];
      dft5(sm.t1[f][k1][b], sm.t1[f][k1][5 + b], sm.t1[f][k1][10 + b], sm.t1[f][k1][15 + b],
           sm.t1[f][k1][20 + b], y);
#pragma unroll
      for (int c = 0; c < 5; ++c) {
        cf tw = {tb.w25[b][c][0], tb.w25[b][c][1]};
        sm.t2[f][k1][c * 5 + b] = cmul(y[c], tw);
      }
    }
    __syncthreads();
    // pass 3: DFT-5 over b -> X[k1 + 16 (c + 5 d)] -> power into t1 (reused as float[FT][201+])
    float* pw = reinterpret_cast<float*>(&sm.t1[0][0][0]);
    for (int task = tid; task < nfr * 45; task += NT) {
      const int f = task / 45, r = task - f * 45, k1 = r / 5, c = r - k1 * 5;
      cf y[5];
      dft5(sm.t2[f][k1][c * 5 + 0], sm.t2[f][k1][c * 5 + 1], sm.t2[f][k1][c * 5 + 2],
           sm.t2[f][k1][c * 5 + 3], sm.t2[f][k1][c * 5 + 4], y);
#pragma unroll
      for (int d = 0; d < 5; ++d) {
        const int bin = k1 + 16 * (c + 5 * d);
        const float p = fmaf(y[d].x, y[d].x, y[d].y * y[d].y);
        if (bin <= 200)
          pw[f * 208 + bin] = p;
        else if (k1 >= 1 && k1 <= 7)
          pw[f * 208 + (N_FFT - bin)] = p;
      }
    }
    __syncthreads();
    // mel: S[m][f] = sum_j w[m][j] * P[f][start_m + j]
    for (int task = tid; task < nfr * NMEL; task += NT) {
      const int f = task / NMEL, m = task - f * NMEL;
      const int st = tb.mel_start[m], cnt = tb.mel_cnt[m];
      const float* p = pw + f * 208 + st;
      float acc = 0.0f;
      for (int j = 0; j < cnt; ++j) acc = fmaf(tb.mel_w[m][j], p[j], acc);
      sm.s[m][f0 + f] = acc;
      smax = fmaxf(smax, acc);
      smin = fminf(smin, acc);
    }
    __syncthreads();
  }

  // ---- clip-global max / min of the mel power -----------------------------------------------------
  smax = wave_max(smax);
  smin = wave_min(smin);
  if ((tid & 63) == 0) {
    sm.red[0][tid >> 6] = smax;
    sm.red[1][tid >> 6] = smin;
  }
  __syncthreads();
  smax = sm.red[0][0];
  smin = sm.red[1][0];
#pragma unroll
  for (int w = 1; w < NT / 64; ++w) {
    smax = fmaxf(smax, sm.red[0][w]);
    smin = fminf(smin, sm.red[1][w]);
  }

  // power_to_db(ref=np.max, amin=1e-10, top_db=80) with numpy-1.21 dtypes, then normalize_matrix.
  // log10 is monotone, so max/min of the dB matrix are the dB of max/min S.  Each numpy op rounds
  // separately: no FMA contraction from here on.
  {
#pragma clang fp contract(off)
  const float amin = 1e-10f;
  const float ref_db = (float)(10.0 * log10(fmax(1e-10, (double)smax)));
  const float d_max = 10.0f * log10f(fmaxf(amin, smax)) - ref_db;
  const float thr = d_max - 80.0f;
  const float d_min = fmaxf(10.0f * log10f(fmaxf(amin, smin)) - ref_db, thr);
  const float diff = d_max - d_min;

  float* db_out = a.db ? a.db + clip * (NMEL * NF) : nullptr;
  float* nm_out = a.norm ? a.norm + clip * (NMEL * NF) : nullptr;
  for (int e = tid; e < NMEL * NF; e += NT) {
    const int m = e / NF, t = e - m * NF;
    float d = 10.0f * log10f(fmaxf(amin, sm.s[m][t])) - ref_db;
    d = fmaxf(d, thr);
    const float nv = (d - d_min) / diff;
    if (db_out) db_out[e] = d;
    if (nm_out) nm_out[e] = nv;
    sm.s[m][t] = nv;   // keep the normalised value for the image
  }
  if (a.zcr) {
    for (int f = tid; f < NF; f += NT) a.zcr[clip * NF + f] = (float)sm.zc[f] * (1.0f / 400.0f);
  }
  if (a.img) {
    __syncthreads();
    // img[h][w][ch]: R = trunc(255 * zcr[w]) (float64), G = B = trunc(255 * (1 - norm[127-h][w]))
    // (float64: numpy-1.21 '1 - np.float32' promotes); NaN -> 0.
    uint32_t* out = reinterpret_cast<uint32_t*>(a.img + clip * (NMEL * NF * 3));
    for (int wd = tid; wd < NMEL * NF * 3 / 4; wd += NT) {
      uint32_t word = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = wd * 4 + j;
        const int px = q / 3, ch = q - px * 3;
        const int h = px / NF, w = px - h * NF;
        double v;
        if (ch == 0)
          v = ((double)sm.zc[w] / 400.0) * 255.0;
        else
          v = (1.0 - (double)sm.s[NMEL - 1 - h][w]) * 255.0;
        const uint32_t byte = (v >= 0.0) ? (uint32_t)(int)v : 0u;   // NaN fails v >= 0
        word |= (byte & 255u) << (8 * j);
      }
      out[wd] = word;
    }
  }
  }
}

}  // namespace

size_t od_fe_smem_bytes() { return sizeof(Smem); }

hipError_t od_fe_launch(const OdFeArgs& a, int64_t n_clips, hipStream_t stream) {
  if (n_clips <= 0) return hipSuccess;
  const size_t smem = sizeof(Smem);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(od_fe_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(od_fe_kernel, dim3((unsigned)n_clips), dim3(NT), smem, stream, a);
  return hipGetLastError();
}

void od_fe_build_tables(OdFeTables* t) {
  const double PI = 3.14159265358979323846;
  for (int n = 0; n < N_FFT; ++n) t->hann[n] = (float)(0.5 - 0.5 * cos(2.0 * PI * n / N_FFT));
  for (int k = 0; k < 9; ++k) {
    t->w16[k][0] = (float)cos(2.0 * PI * k / 16.0);
    t->w16[k][1] = (float)-sin(2.0 * PI * k / 16.0);
    for (int n2 = 0; n2 < 25; ++n2) {
      t->w400[k][n2][0] = (float)cos(2.0 * PI * n2 * k / 400.0);
      t->w400[k][n2][1] = (float)-sin(2.0 * PI * n2 * k / 400.0);
    }
  }
  for (int b = 0; b < 5; ++b)
    for (int c = 0; c < 5; ++c) {
      t->w25[b][c][0] = (float)cos(2.0 * PI * b * c / 25.0);
      t->w25[b][c][1] = (float)-sin(2.0 * PI * b * c / 25.0);
    }
  // librosa.filters.mel(16000, 400, n_mels=128, fmin=0, fmax=8000, htk=False, norm='slaney'):
  // float64 triangles stored float32, then float32 * float64 enorm -> float32.
  auto hz_to_mel = [](double f) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = 1000.0 / f_sp;
    const double logstep = log(6.4) / 27.0;
    return f >= min_log_hz ? min_log_mel + log(f / min_log_hz) / logstep : f / f_sp;
  };
  auto mel_to_hz = [](double m) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = 1000.0 / f_sp;
    const double logstep = log(6.4) / 27.0;
    return m >= min_log_mel ? min_log_hz * exp(logstep * (m - min_log_mel)) : f_sp * m;
  };
  double mel_f[NMEL + 2];
  const double mmin = hz_to_mel(0.0), mmax = hz_to_mel(8000.0);
  for (int i = 0; i < NMEL + 2; ++i) {
    // np.linspace(min, max, n): start + i * step, last element exactly max
    const double step = (mmax - mmin) / (NMEL + 1);
    const double m = (i == NMEL + 1) ? mmax : mmin + i * step;
    mel_f[i] = mel_to_hz(m);
  }
  for (int m = 0; m < NMEL; ++m) {
    int st = -1, cnt = 0;
    float w[16] = {0};
    const double enorm = 2.0 / (mel_f[m + 2] - mel_f[m]);
    const double fd0 = mel_f[m + 1] - mel_f[m], fd1 = mel_f[m + 2] - mel_f[m + 1];
    for (int k = 0; k <= N_FFT / 2; ++k) {
      const double fk = 8000.0 * k / (N_FFT / 2);     // np.linspace(0, 8000, 201)
      const double lower = -(mel_f[m] - fk) / fd0;
      const double upper = (mel_f[m + 2] - fk) / fd1;
      double v = fmin(lower, upper);
      v = v > 0.0 ? v : 0.0;
      const float v32 = (float)v;
      const float wv = (float)((double)v32 * enorm);
      if (wv != 0.0f) {
        if (st < 0) st = k;
        w[k - st] = wv;
        cnt = k - st + 1;
      }
    }
    t->mel_start[m] = st < 0 ? 0 : st;
    t->mel_cnt[m] = cnt;
    for (int j = 0; j < 10; ++j) t->mel_w[m][j] = j < cnt ? w[j] : 0.0f;
  }
}
