// Silence removal on the GPU: the save_wave_file(silence_remove=True) step of
// OverlapDetection/scripts/record_on_pc.py:214-226 (and its SpeakerIdentification twins).
//
//   vad_speech_kernel   webrtcvad.Vad(mode).is_speech on every 30 ms frame, ONE THREAD PER STREAM:
//                       the detector is a chain of IIR filters and an adaptive GMM whose state
//                       carries from frame to frame and call to call (the reference keeps one
//                       module-level Vad(3)), so frames of a stream are sequential and streams are
//                       the parallel axis.  Fixed-point arithmetic exactly as WebRTC's
//                       common_audio/vad (restated in oracle/webrtc_vad.py, the checker): 16 -> 8 kHz
//                       all-pass downsampler, a 5-level splitting-filter tree into six bands, log
//                       energies, two-Gaussian noise / speech models with adaptation, hangover.
//                       Per-thread band buffers and the FindMinimum tables live in LDS (indexed by
//                       data), the rest of the state in registers.
//   vad_collect_kernel  vad_collector (:246-295) + the rewrite, ONE WAVE PER ITEM: lane 0 walks the
//                       frame decisions through the 10-frame ring-buffer trigger logic into a keep
//                       mask, then the wave copies the kept 480-sample frames, compacted, to the
//                       output (coalesced 16-B chunks).
//   pcm16_kernel        sf.write(path, y, 16000) PCM_16 (:212): (short) lrintf(y * 32767).
#include "common.h"
#include "vad.h"

#include <cstring>

namespace {

constexpr int NUM_CH = 6, NUM_G = 2, TBL = 12;
constexpr int MIN_ENERGY = 10;
constexpr int FRAME = 480;            // 30 ms at 16 kHz
constexpr int NT_VAD = 64;            // streams per workgroup (one thread each)

__constant__ int16_t kSpectrumWeight[NUM_CH] = {6, 8, 10, 12, 14, 16};
__constant__ int16_t kMinimumDifference[NUM_CH] = {544, 544, 576, 576, 576, 576};
__constant__ int16_t kMaximumSpeech[NUM_CH] = {11392, 11392, 11520, 11520, 11520, 11520};
__constant__ int16_t kMinimumMean[NUM_G] = {640, 768};
__constant__ int16_t kMaximumNoise[NUM_CH] = {9216, 9088, 8960, 8832, 8704, 8576};
__constant__ int16_t kNoiseWeights[TBL] = {34, 62, 72, 66, 53, 25, 94, 66, 56, 62, 75, 103};
__constant__ int16_t kSpeechWeights[TBL] = {48, 82, 45, 87, 50, 47, 80, 46, 83, 41, 78, 81};
__constant__ int16_t kOffsetVector[NUM_CH] = {368, 368, 272, 176, 176, 176};

constexpr int16_t NOISE_MEANS[TBL] = {6738, 4892, 7065, 6715, 6771, 3369, 7646, 3863, 7820, 7266, 5020, 4362};
constexpr int16_t SPEECH_MEANS[TBL] = {8306, 10085, 10078, 11823, 11843, 6309, 9473, 9571, 10879, 7581, 8180, 7483};
constexpr int16_t NOISE_STDS[TBL] = {378, 1064, 493, 582, 688, 593, 474, 697, 475, 688, 421, 455};
constexpr int16_t SPEECH_STDS[TBL] = {555, 505, 567, 524, 585, 1231, 509, 828, 492, 1540, 1079, 850};
// 30 ms entries of the mode tables (WebRtcVad_set_mode_core): oh1, oh2, individual, total
constexpr int16_t MODE30[4][4] = {{3, 5, 24, 57}, {3, 5, 37, 100}, {2, 3, 82, 285}, {2, 3, 94, 1100}};

MMLA_DEV int16_t s16(int32_t x) { return (int16_t)x; }   // int16_t store (wraps)

// WebRtcSpl_DivW32W16: truncating division, 0x7FFFFFFF for a zero denominator
MMLA_DEV int32_t div32_16(int32_t num, int16_t den) { return den != 0 ? num / (int32_t)den : 0x7FFFFFFF; }

MMLA_DEV int norm_w32(int32_t a) {   // WebRtcSpl_NormW32
  if (a == 0) return 0;
  const uint32_t u = (uint32_t)(a < 0 ? ~a : a);
  return (u == 0 ? 32 : __clz(u)) - 1;
}

MMLA_DEV int norm_u32(uint32_t a) { return a == 0 ? 0 : __clz(a); }

MMLA_DEV int size_in_bits(uint32_t n) { return n == 0 ? 0 : 32 - __clz(n); }

// splitting filter on data[0..2 half): upper all-pass on even samples, lower on odd ones; outputs
// hp[i] = up - lo, lp[i] = lo + up (vad_filterbank.c SplitFilter / AllPassFilter)
MMLA_DEV void split(const int16_t* data, int half, int16_t& ust, int16_t& lst, int16_t* hp,
                    int16_t* lp) {
  int32_t su = (int32_t)ust * 65536, sl = (int32_t)lst * 65536;
  for (int i = 0; i < half; ++i) {
    const int32_t xu = data[2 * i], xl = data[2 * i + 1];
    // int32 sums wrap as in the C (uint32 arithmetic, then an arithmetic shift)
    const int16_t tu = s16((int32_t)((uint32_t)su + (uint32_t)(20972 * xu)) >> 16);
    su = (int32_t)((uint32_t)(xu * 16384 - 20972 * tu) * 2u);
    const int16_t tl = s16((int32_t)((uint32_t)sl + (uint32_t)(5571 * xl)) >> 16);
    sl = (int32_t)((uint32_t)(xl * 16384 - 5571 * tl) * 2u);
    hp[i] = s16(tu - tl);
    lp[i] = s16(tl + tu);
  }
  ust = s16(su >> 16);
  lst = s16(sl >> 16);
}

// LogOfEnergy (vad_filterbank.c) with WebRtcSpl_Energy / GetScalingSquare
MMLA_DEV int16_t log_energy(const int16_t* x, int n, int16_t offset, int16_t& total) {
  int smax = -1;
  for (int i = 0; i < n; ++i) {
    const int v = x[i];
    const int sabs = v > 0 ? v : (int)s16(-v);
    smax = sabs > smax ? sabs : smax;
  }
  const int nbits = size_in_bits((uint32_t)n);
  const int t = norm_w32(smax * smax);
  const int scaling = smax == 0 ? 0 : (t > nbits ? 0 : nbits - t);
  int32_t en = 0;
  for (int i = 0; i < n; ++i) en = (int32_t)((uint32_t)en + (uint32_t)((x[i] * x[i]) >> scaling));
  uint32_t energy = (uint32_t)en;
  if (energy == 0) return offset;
  int tot_rshifts = scaling;
  const int nr = 17 - norm_u32(energy);
  tot_rshifts += nr;
  energy = nr < 0 ? energy << -nr : energy >> nr;
  const int16_t log2_energy = s16(14336 + (int)((energy & 0x3FFF) >> 4));
  int16_t le = s16(((24660 * log2_energy) >> 19) + ((tot_rshifts * 24660) >> 9));
  if (le < 0) le = 0;
  le = s16(le + offset);
  if (total <= MIN_ENERGY) {
    if (tot_rshifts >= 0) total = s16(total + MIN_ENERGY + 1);
    else total = s16(total + s16((int32_t)(energy >> -tot_rshifts)));
  }
  return le;
}

// WebRtcVad_GaussianProbability: Q20 probability, delta in Q11
MMLA_DEV int32_t gauss(int16_t input, int16_t mean, int16_t std, int16_t& delta) {
  const int16_t inv_std = s16(div32_16(131072 + (std >> 1), std));
  int16_t t16 = inv_std >> 2;
  const int16_t inv_std2 = s16((t16 * t16) >> 2);
  t16 = s16(s16(input << 3) - mean);
  delta = s16((inv_std2 * t16) >> 10);
  const int32_t t32 = (delta * t16) >> 9;
  int32_t exp_value = 0;
  if (t32 < 22005) {
    int16_t e = s16((5909 * t32) >> 12);
    e = s16(-e);
    exp_value = 0x0400 | (e & 0x03FF);
    e = s16(e ^ 0xFFFF);
    e >>= 10;
    e += 1;
    exp_value >>= e;
  }
  return (int32_t)((uint32_t)inv_std * (uint32_t)exp_value);
}

// WebRtcVad_FindMinimum: the 16 smallest features of the last 100 frames (LDS), median, smoothing
MMLA_DEV int16_t find_minimum(int16_t* sv, int16_t* age, int16_t& mean_value, int32_t frame_counter,
                              int16_t value) {
  for (int i = 0; i < 16; ++i) {
    if (age[i] != 100) {
      age[i] += 1;
    } else {
      for (int j = i; j < 15; ++j) {
        sv[j] = sv[j + 1];
        age[j] = age[j + 1];
      }
      age[15] = 101;
      sv[15] = 10000;
    }
  }
  int pos = -1;
  for (int p = 0; p < 16; ++p)
    if (value < sv[p]) {
      pos = p;
      break;
    }
  if (pos > -1) {
    for (int i = 15; i > pos; --i) {
      sv[i] = sv[i - 1];
      age[i] = age[i - 1];
    }
    sv[pos] = value;
    age[pos] = 1;
  }
  int16_t median = 1600;
  if (frame_counter > 2) median = sv[2];
  else if (frame_counter > 0) median = sv[0];
  int16_t alpha = 0;
  if (frame_counter > 0) alpha = median < mean_value ? 6553 : 32439;
  const int32_t t32 = (alpha + 1) * mean_value + (32767 - alpha) * median + 16384;
  mean_value = s16(t32 >> 15);
  return mean_value;
}

// per-thread LDS: the frame at 8 kHz and the band buffers of the splitting tree, FindMinimum tables
struct VadLds {
  int16_t x8[240];
  int16_t a120[120], b120[120];
  int16_t a60[60], b60[60];
  int16_t lv[96], age[96];
};

__global__ void __launch_bounds__(NT_VAD) vad_speech_kernel(VadArgs a) {
  __shared__ VadLds lds[NT_VAD];
  const int64_t st = (int64_t)blockIdx.x * NT_VAD + threadIdx.x;
  const int64_t n_streams = a.n_items / a.items_per_stream;
  if (st >= n_streams) return;
  VadLds& L = lds[threadIdx.x];
  VadState S = a.state[st];
  for (int i = 0; i < 96; ++i) {
    L.lv[i] = S.low_value[i];
    L.age[i] = S.age[i];
  }
  for (int64_t it = st * a.items_per_stream; it < (st + 1) * a.items_per_stream; ++it) {
    int len = a.lens ? a.lens[it] : a.clip_len;
    if (len < 0) len = 0;
    if (len > a.stride) len = (int)a.stride;   // never past the item's row (device-pointer lens)
    const int nf = min(vad_frames(len), a.max_frames);
    const int16_t* src = a.pcm + it * a.stride;
    uint8_t* flags = a.speech + it * a.max_frames;
    for (int f = 0; f < nf; ++f) {
      const int16_t* x = src + f * FRAME;
      // ---- 16 -> 8 kHz (vad_sp.c Downsampling) ----
      int32_t t1 = S.ds[0], t2 = S.ds[1];
      for (int n = 0; n < 240; ++n) {
        const int32_t xe = x[2 * n], xo = x[2 * n + 1];
        const int16_t u = s16((t1 >> 1) + ((5243 * xe) >> 14));
        t1 = xe - ((5243 * u) >> 12);
        const int16_t w = s16((t2 >> 1) + ((1392 * xo) >> 14));
        t2 = xo - ((1392 * w) >> 12);
        L.x8[n] = s16(u + w);
      }
      S.ds[0] = t1;
      S.ds[1] = t2;
      // ---- features (vad_filterbank.c CalculateFeatures) ----
      int16_t feat[NUM_CH];
      int16_t total = 0;
      split(L.x8, 120, S.upper[0], S.lower[0], L.a120, L.b120);     // hp 2-4 kHz, lp 0-2 kHz
      split(L.a120, 60, S.upper[1], S.lower[1], L.a60, L.b60);      // 3-4 / 2-3 kHz
      feat[5] = log_energy(L.a60, 60, kOffsetVector[5], total);
      feat[4] = log_energy(L.b60, 60, kOffsetVector[4], total);
      split(L.b120, 60, S.upper[2], S.lower[2], L.a60, L.b60);      // 1-2 / 0-1 kHz
      feat[3] = log_energy(L.a60, 60, kOffsetVector[3], total);
      split(L.b60, 30, S.upper[3], S.lower[3], L.a120, L.b120);     // 0.5-1 / 0-0.5 kHz
      feat[2] = log_energy(L.a120, 30, kOffsetVector[2], total);
      split(L.b120, 15, S.upper[4], S.lower[4], L.a60, L.b60);      // 250-500 / 0-250 Hz
      feat[1] = log_energy(L.a60, 15, kOffsetVector[1], total);
      for (int i = 0; i < 15; ++i) {                                 // 80 Hz high-pass of 0-250 Hz
        const int32_t v = L.b60[i];
        int32_t t = 6631 * v + -13262 * S.hp[0] + 6631 * S.hp[1];
        S.hp[1] = S.hp[0];
        S.hp[0] = s16(v);
        t -= -7756 * S.hp[2];
        t -= 5620 * S.hp[3];
        S.hp[3] = S.hp[2];
        S.hp[2] = s16(t >> 14);
        L.a120[i] = S.hp[2];
      }
      feat[0] = log_energy(L.a120, 15, kOffsetVector[0], total);
      // ---- GMM decision + model update (vad_core.c GmmProbability), 30 ms thresholds ----
      int vadflag = 0;
      if (total > MIN_ENERGY) {
        int16_t dn[TBL], ds_[TBL], ngpr[TBL], sgpr[TBL];
        int32_t sum_llr = 0;
#pragma unroll
        for (int ch = 0; ch < NUM_CH; ++ch) {
          int32_t h0t = 0, h1t = 0, np0 = 0, sp0 = 0;
#pragma unroll
          for (int k = 0; k < NUM_G; ++k) {
            const int g = ch + k * NUM_CH;
            const int32_t pn = (int32_t)((uint32_t)kNoiseWeights[g] *
                                         (uint32_t)gauss(feat[ch], S.noise_means[g], S.noise_stds[g], dn[g]));
            const int32_t ps = (int32_t)((uint32_t)kSpeechWeights[g] *
                                         (uint32_t)gauss(feat[ch], S.speech_means[g], S.speech_stds[g], ds_[g]));
            h0t = (int32_t)((uint32_t)h0t + (uint32_t)pn);
            h1t = (int32_t)((uint32_t)h1t + (uint32_t)ps);
            if (k == 0) {
              np0 = pn;
              sp0 = ps;
            }
          }
          const int sh0 = h0t == 0 ? 31 : norm_w32(h0t);
          const int sh1 = h1t == 0 ? 31 : norm_w32(h1t);
          const int16_t llr = s16(sh0 - sh1);
          sum_llr += llr * kSpectrumWeight[ch];
          if (llr * 4 > S.individual) vadflag = 1;
          const int16_t h0 = s16(h0t >> 12);
          ngpr[ch] = 16384;
          ngpr[ch + NUM_CH] = 0;
          if (h0 > 0) {
            const int32_t t = (int32_t)(((uint32_t)np0 & 0xFFFFF000u) << 2);
            ngpr[ch] = s16(div32_16(t, h0));
            ngpr[ch + NUM_CH] = s16(16384 - ngpr[ch]);
          }
          const int16_t h1 = s16(h1t >> 12);
          sgpr[ch] = 0;
          sgpr[ch + NUM_CH] = 0;
          if (h1 > 0) {
            const int32_t t = (int32_t)(((uint32_t)sp0 & 0xFFFFF000u) << 2);
            sgpr[ch] = s16(div32_16(t, h1));
            sgpr[ch + NUM_CH] = s16(16384 - sgpr[ch]);
          }
        }
        vadflag |= sum_llr >= S.total ? 1 : 0;
        int16_t maxspe = 12800;
#pragma unroll
        for (int ch = 0; ch < NUM_CH; ++ch) {
          const int16_t fmin = find_minimum(L.lv + 16 * ch, L.age + 16 * ch, S.mean_value[ch],
                                            S.frame_counter, feat[ch]);
          int32_t ngm = S.noise_means[ch] * kNoiseWeights[ch] +
                        S.noise_means[ch + NUM_CH] * kNoiseWeights[ch + NUM_CH];
          const int16_t t1s = s16(ngm >> 6);
#pragma unroll
          for (int k = 0; k < NUM_G; ++k) {
            const int g = ch + k * NUM_CH;
            const int16_t nmk = S.noise_means[g], smk = S.speech_means[g];
            int16_t nsk = S.noise_stds[g], ssk = S.speech_stds[g];
            int16_t nmk2 = nmk;
            if (!vadflag) {
              const int16_t delt = s16((ngpr[g] * dn[g]) >> 11);
              nmk2 = s16(nmk + s16((delt * 655) >> 22));
            }
            const int16_t ndelt = s16((fmin << 4) - t1s);
            int16_t nmk3 = s16(nmk2 + s16((ndelt * 154) >> 9));
            const int16_t lo = s16((k + 5) << 7), hi = s16((72 + k - ch) << 7);
            if (nmk3 < lo) nmk3 = lo;
            if (nmk3 > hi) nmk3 = hi;
            S.noise_means[g] = nmk3;
            if (vadflag) {
              const int16_t delt = s16((sgpr[g] * ds_[g]) >> 11);
              int16_t t16 = s16((delt * 6554) >> 21);
              int16_t smk2 = s16(smk + ((t16 + 1) >> 1));
              const int maxmu = maxspe + 640;
              if (smk2 < kMinimumMean[k]) smk2 = kMinimumMean[k];
              if (smk2 > maxmu) smk2 = s16(maxmu);
              S.speech_means[g] = smk2;
              t16 = s16((smk + 4) >> 3);
              t16 = s16(feat[ch] - t16);
              int32_t a32 = (ds_[g] * t16) >> 3;
              int32_t b32 = a32 - 4096;
              t16 = sgpr[g] >> 2;
              a32 = (int32_t)((uint32_t)t16 * (uint32_t)b32);
              b32 = a32 >> 4;
              if (b32 > 0) t16 = s16(div32_16(b32, s16(ssk * 10)));
              else t16 = s16(-s16(div32_16(-b32, s16(ssk * 10))));
              t16 = s16(t16 + 128);
              ssk = s16(ssk + (t16 >> 8));
              if (ssk < 384) ssk = 384;
              S.speech_stds[g] = ssk;
            } else {
              int16_t t16 = s16(feat[ch] - (nmk >> 3));
              int32_t a32 = (dn[g] * t16) >> 3;
              a32 -= 4096;
              t16 = (ngpr[g] + 2) >> 2;
              const int32_t b32 = (int32_t)((uint32_t)t16 * (uint32_t)a32);
              a32 = b32 >> 14;
              if (a32 > 0) t16 = s16(div32_16(a32, nsk));
              else t16 = s16(-s16(div32_16(-a32, nsk)));
              t16 = s16(t16 + 32);
              nsk = s16(nsk + (t16 >> 6));
              if (nsk < 384) nsk = 384;
              S.noise_stds[g] = nsk;
            }
          }
          ngm = S.noise_means[ch] * kNoiseWeights[ch] + S.noise_means[ch + NUM_CH] * kNoiseWeights[ch + NUM_CH];
          int32_t sgm = S.speech_means[ch] * kSpeechWeights[ch] +
                        S.speech_means[ch + NUM_CH] * kSpeechWeights[ch + NUM_CH];
          const int16_t diff = s16(s16(sgm >> 9) - s16(ngm >> 9));
          if (diff < kMinimumDifference[ch]) {
            const int16_t t16 = s16(kMinimumDifference[ch] - diff);
            const int16_t aa = s16((13 * t16) >> 2), bb = s16((3 * t16) >> 2);
            S.speech_means[ch] = s16(S.speech_means[ch] + aa);
            S.speech_means[ch + NUM_CH] = s16(S.speech_means[ch + NUM_CH] + aa);
            sgm = S.speech_means[ch] * kSpeechWeights[ch] + S.speech_means[ch + NUM_CH] * kSpeechWeights[ch + NUM_CH];
            S.noise_means[ch] = s16(S.noise_means[ch] - bb);
            S.noise_means[ch + NUM_CH] = s16(S.noise_means[ch + NUM_CH] - bb);
            ngm = S.noise_means[ch] * kNoiseWeights[ch] + S.noise_means[ch + NUM_CH] * kNoiseWeights[ch + NUM_CH];
          }
          maxspe = kMaximumSpeech[ch];
          int16_t t2s = s16(sgm >> 7);
          if (t2s > maxspe) {
            t2s = s16(t2s - maxspe);
            S.speech_means[ch] = s16(S.speech_means[ch] - t2s);
            S.speech_means[ch + NUM_CH] = s16(S.speech_means[ch + NUM_CH] - t2s);
          }
          t2s = s16(ngm >> 7);
          if (t2s > kMaximumNoise[ch]) {
            t2s = s16(t2s - kMaximumNoise[ch]);
            S.noise_means[ch] = s16(S.noise_means[ch] - t2s);
            S.noise_means[ch + NUM_CH] = s16(S.noise_means[ch + NUM_CH] - t2s);
          }
        }
        S.frame_counter += 1;
      }
      if (!vadflag) {
        if (S.over_hang > 0) {
          vadflag = 2 + S.over_hang;
          S.over_hang -= 1;
        }
        S.num_of_speech = 0;
      } else {
        S.num_of_speech += 1;
        if (S.num_of_speech > 6) {
          S.num_of_speech = 6;
          S.over_hang = S.oh2;
        } else {
          S.over_hang = S.oh1;
        }
      }
      flags[f] = vadflag > 0 ? 1 : 0;
    }
  }
  for (int i = 0; i < 96; ++i) {
    S.low_value[i] = L.lv[i];
    S.age[i] = L.age[i];
  }
  a.state[st] = S;
}

constexpr int NT_COL = 64;
constexpr int MAXF_LDS = 4096;   // frames per item the collector's LDS mask holds (> 2 min)

__global__ void __launch_bounds__(NT_COL) vad_collect_kernel(VadArgs a) {
  __shared__ int32_t dst[MAXF_LDS];     // output frame index of each kept frame, -1 = dropped
  __shared__ int32_t n_keep;
  const int64_t it = blockIdx.x;
  const int lane = threadIdx.x;
  int len = a.lens ? a.lens[it] : a.clip_len;
  if (len < 0) len = 0;
  if (len > a.stride) len = (int)a.stride;     // reads and the rewrite stay inside the item's row
  const int nf = min(min(vad_frames(len), a.max_frames), MAXF_LDS);
  const uint8_t* sp = a.speech + it * a.max_frames;
  if (lane == 0) {
    // vad_collector: ring of the last 10 (frame, is_speech), TRIGGERED after > 9 voiced, back to
    // NOTTRIGGERED (yielding the voiced frames) after > 9 unvoiced; leftover voiced frames yielded
    int ring[10], rs = 0, rn = 0;   // ring of frame indices (speech bit in bit 30), start, count
    bool trig = false;
    int vstart = -1;                // first voiced frame of the current segment (all frames from it on)
    for (int f = 0; f < nf; ++f) dst[f] = -1;
    int kept = 0;
    for (int f = 0; f < nf; ++f) {
      const int s = sp[f] ? 1 : 0;
      if (rn == 10) {
        rs = (rs + 1) % 10;
        rn = 9;
      }
      ring[(rs + rn) % 10] = f | (s << 30);
      ++rn;
      int cnt = 0;
      for (int j = 0; j < rn; ++j) cnt += trig ? !(ring[(rs + j) % 10] >> 30) : (ring[(rs + j) % 10] >> 30);
      if (!trig) {
        if (cnt > 9) {               // > 0.9 * 10
          trig = true;
          vstart = ring[rs] & 0x3fffffff;
          rn = 0;
        }
      } else if (cnt > 9) {
        trig = false;
        for (int j = vstart; j <= f; ++j) dst[j] = kept++;
        vstart = -1;
        rn = 0;
      }
    }
    if (vstart >= 0)
      for (int j = vstart; j < nf; ++j) dst[j] = kept++;
    n_keep = kept;
  }
  __syncthreads();
  const int kept = n_keep;
  const int16_t* src = a.pcm + it * a.stride;
  int16_t* out = a.out + it * a.stride;
  // 480-sample frames = 60 chunks of 8 samples; aligned pointers take 16-B moves
  const bool v16 = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(out) |
                     (uintptr_t)(a.stride * 2)) & 15) == 0;
  for (int f = 0; f < nf; ++f) {
    const int d = dst[f];
    if (d < 0) continue;
    if (v16) {
      const uint4* s4 = reinterpret_cast<const uint4*>(src + f * FRAME);
      uint4* o4 = reinterpret_cast<uint4*>(out + d * FRAME);
      if (lane < FRAME / 8) o4[lane] = s4[lane];
    } else {
      for (int i = lane; i < FRAME; i += NT_COL) out[d * FRAME + i] = src[f * FRAME + i];
    }
  }
  if (lane == 0) a.out_lens[it] = kept * FRAME;
}

__global__ void pcm16_kernel(const float* __restrict__ y, int64_t n, int16_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // libsndfile f2s_array: lrintf(0x7FFF * x) (round half to even) stored into a short
  out[i] = (int16_t)(int32_t)__builtin_rintf(32767.0f * y[i]);
}

}  // namespace

bool vad_init_state(VadState* s, int mode) {
  if (mode < 0 || mode > 3) return false;
  memset(s, 0, sizeof(*s));
  for (int i = 0; i < TBL; ++i) {
    s->noise_means[i] = NOISE_MEANS[i];
    s->speech_means[i] = SPEECH_MEANS[i];
    s->noise_stds[i] = NOISE_STDS[i];
    s->speech_stds[i] = SPEECH_STDS[i];
  }
  for (int i = 0; i < 96; ++i) {
    s->low_value[i] = 10000;
    s->age[i] = 0;
  }
  for (int i = 0; i < NUM_CH; ++i) s->mean_value[i] = 1600;
  s->oh1 = MODE30[mode][0];
  s->oh2 = MODE30[mode][1];
  s->individual = MODE30[mode][2];
  s->total = MODE30[mode][3];
  return true;
}

hipError_t vad_speech_launch(const VadArgs& a, hipStream_t s) {
  if (a.n_items <= 0) return hipSuccess;
  if (a.items_per_stream < 1 || a.n_items % a.items_per_stream) return hipErrorInvalidValue;
  const int64_t n_streams = a.n_items / a.items_per_stream;
  hipLaunchKernelGGL(vad_speech_kernel, dim3((unsigned)((n_streams + NT_VAD - 1) / NT_VAD)),
                     dim3(NT_VAD), 0, s, a);
  return hipGetLastError();
}

hipError_t vad_collect_launch(const VadArgs& a, hipStream_t s) {
  if (a.n_items <= 0) return hipSuccess;
  if (a.max_frames > MAXF_LDS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(vad_collect_kernel, dim3((unsigned)a.n_items), dim3(NT_COL), 0, s, a);
  return hipGetLastError();
}

hipError_t pcm16_launch(const float* y, int64_t n, int16_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(pcm16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, y, n, out);
  return hipGetLastError();
}
