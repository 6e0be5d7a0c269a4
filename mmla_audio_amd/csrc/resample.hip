// Rate conversion of the offline pre-conditioning chains.
//
// Replaces:
//   pydub AudioSegment.set_frame_rate(16000) = audioop.ratecv(data, 2, channels, rate, 16000, None)
//       OverlapDetection/scripts/overlap_detection_post_processing.py:120-121 (48 kHz stereo zoom
//       exports), SpeakerIdentification/scripts/speaker_identification_post_processing.py:159-160
//       (the 22.05 kHz PCM_16 file that librosa.load wrote)
//   librosa.load(path) at its default sr = 22050 = resampy.resample(filter='kaiser_best')
//       speaker_identification_post_processing.py:142
//
// ratecv_kernel: CPython's audioop.ratecv loop (weightA 1, weightB 0, fresh state) keeps a phase
// counter d = -outrate; every input frame adds outrate, every output frame subtracts inrate.  So
// output frame j is written right after input frame k = ceil(j inrate / outrate) was read, at
// d = k outrate - j inrate, and is a pure function of (j, frames k - 1 and k): one thread per output
// frame, bit-identical to the sequential C loop (the double products are exact; the one division is
// IEEE-rounded on both sides; (int) truncates; >> 16 floors as the C shift does).
//
// sinc_resample_kernel: resampy 0.2 resample_f for one channel, one thread per output sample: left
// then right wing of the linearly interpolated filter, each tap's float64 product added to a float32
// accumulator (numba stores y[t] as float32 after every tap).  The float64 time register of the
// sequential loop (repeated addition of 1 / ratio) comes from the host.  fp contraction is off so
// every multiply and add rounds as numpy / numba do.
#include "resample.h"

namespace {

__global__ void ratecv_kernel(const int16_t* __restrict__ in, int64_t n_frames, int nch, int ir,
                              int orr, int16_t* __restrict__ out, int64_t n_out) {
#pragma clang fp contract(off)
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_out) return;
  const int64_t k = (j * ir + orr - 1) / orr;       // ceil(j ir / or) <= n_frames - 1
  const int64_t d = k * orr - j * ir;               // [0, or)
  if (k >= n_frames) return;                        // (host sizes n_out so this never happens)
  for (int ch = 0; ch < nch; ++ch) {
    const int prev = k > 0 ? ((int)in[(k - 1) * nch + ch]) * 65536 : 0;   // GETSAMPLE32: x << 16
    const int cur = ((int)in[k * nch + ch]) * 65536;
    const double v = ((double)prev * (double)d + (double)cur * (double)(orr - d)) / (double)orr;
    const int o = (int)v;                                                   // C cast: truncation
    out[j * nch + ch] = (int16_t)(o >> 16);                                 // SETSAMPLE32
  }
}

__global__ void sinc_resample_kernel(SincResampleArgs a) {
#pragma clang fp contract(off)
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.n_out) return;
  const double2* __restrict__ wd = reinterpret_cast<const double2*>(a.win);   // (win, dwin) pairs
  const double tr = a.tr[t];
  // n <= n_orig - 1 for every rate pair (the last time is ~ n_orig - 1 / ratio); clamped anyway so a
  // time register that drifted past the input (ratios far beyond audio's) cannot read past x
  int64_t n = (int64_t)tr;
  n = n < a.n_orig ? n : a.n_orig - 1;
  double frac = a.scale * (tr - (double)n);
  double index_frac = frac * (double)a.num_table;
  int64_t offset = (int64_t)index_frac;
  double eta = index_frac - (double)offset;
  float y = 0.0f;
  const int64_t i_max = min(n + 1, (a.nwin - offset) / a.index_step);
  for (int64_t i = 0; i < i_max; ++i) {
    const double2 w = wd[offset + i * a.index_step];
    const double weight = w.x + eta * w.y;
    y = (float)((double)y + weight * (double)a.x[n - i]);
  }
  frac = a.scale - frac;
  index_frac = frac * (double)a.num_table;
  offset = (int64_t)index_frac;
  eta = index_frac - (double)offset;
  const int64_t k_max = min(a.n_orig - n - 1, (a.nwin - offset) / a.index_step);
  for (int64_t k = 0; k < k_max; ++k) {
    const double2 w = wd[offset + k * a.index_step];
    const double weight = w.x + eta * w.y;
    y = (float)((double)y + weight * (double)a.x[n + k + 1]);
  }
  a.y[t] = y;
}

}  // namespace

hipError_t ratecv_launch(const int16_t* in, int64_t n_frames, int nch, int inrate, int outrate,
                         int16_t* out, int64_t n_out, hipStream_t s) {
  if (n_out <= 0) return hipSuccess;
  if (nch < 1 || inrate < 1 || outrate < 1 || n_frames < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ratecv_kernel, dim3((unsigned)((n_out + 255) / 256)), dim3(256), 0, s, in,
                     n_frames, nch, inrate, outrate, out, n_out);
  return hipGetLastError();
}

hipError_t sinc_resample_launch(const SincResampleArgs& a, hipStream_t s) {
  if (a.n_out <= 0) return hipSuccess;
  if (a.index_step < 1 || a.nwin < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sinc_resample_kernel, dim3((unsigned)((a.n_out + 255) / 256)), dim3(256), 0, s,
                     a);
  return hipGetLastError();
}
