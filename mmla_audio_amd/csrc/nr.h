// Stationary spectral-gate noise reduction kernel interface (see nr.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

constexpr int NR_NFFT = 1024;   // noisereduce 2.0 defaults: n_fft 1024, win_length = n_fft,
constexpr int NR_HOP = 256;     // hop = win_length // 4
constexpr int NR_NGF = 33;      // smoothing filter at 16 kHz: 2 * 16 + 1 bins (500 Hz) ...
constexpr int NR_NGT = 7;       // ... x 2 * 3 + 1 frames (50 ms)

struct NrTables {
  double win[NR_NFFT];          // periodic Hann
  cd w512[512];                 // W512^m
  double w1024[NR_NFFT / 2 + 1][2];   // W1024^k
  double gf[NR_NGF];            // smoothing filter = gf (x) gt (separable, each normalised)
  double gt[NR_NGT];
  int ngf, ngt;                 // taps the ramps actually have (must equal NR_NGF / NR_NGT)
};

// one buffer of L samples: buffer index u <-> signal index i1 + u (zeros outside [0, n));
// output = buffer [keep0, keep0 + out_len) -> out[out_off ..]
struct NrItem {
  int64_t sig_off, n, i1, out_off, out_len;
};

struct NrArgs {
  const float* y;               // signals (float32, as librosa.load returns)
  const NrItem* items;
  int64_t n_items;
  int64_t L;                    // buffer length: chunk + 2 * padding
  int T;                        // STFT frames per buffer: 1 + L / 256
  int t_lo, t_n;                // frames launched per item: every frame that is not an all-zero
                                // window or whose mask the gate needs (host: nr_frame_range)
  int64_t keep0, keep_len;      // kept interior of every buffer
  const NrTables* tables;
  const float* thresh;          // [513] noise threshold (dB, float32)
  double prop_decrease;
  double2* S;                   // scratch [n_items][T][513] complex128
  uint8_t* bits;                // scratch [n_items][T][513] dB > thresh
  double* fmax;                 // scratch [n_items][T] frame max dB
  double* gmax;                 // scratch [n_items] max over the item's frames
  double* rows;                 // scratch [n_items][T][513] frequency-smoothed mask rows
  double* frames;               // scratch [n_items][T][1024] gated windowed frames
  float* out;
};

void nr_build_tables(NrTables* t, int sr);
// noise profile: db_scratch [1 + m/256][513], fmax_scratch [1 + m/256] -> thresh [513]
hipError_t nr_noise_launch(const float* noise, int64_t m, const NrTables* tables, float* db_scratch,
                           float* fmax_scratch, float n_std, float* thresh, hipStream_t s);
hipError_t nr_gate_launch(const NrArgs& a, hipStream_t s);
// [t_lo, t_hi] covering, for every item, the frames whose window overlaps its signal and the frames
// within the time-smoothing halo of the kept interior
void nr_frame_range(const NrItem* items, int64_t n_items, int64_t L, int T, int64_t keep0,
                    int64_t keep_len, int* t_lo, int* t_hi);
