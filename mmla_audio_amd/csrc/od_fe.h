// OverlapDetection front-end kernel interface (see od_fe.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct OdFeTables {
  float hann[400];          // periodic Hann (scipy get_window('hann', 400, fftbins=True))
  float w16[9][2];          // W16^k, k = 0..8
  float w400[9][25][2];     // W400^(n2*k1)
  float w25[5][5][2];       // W25^(b*c)
  int mel_start[128];       // first non-zero bin of each Slaney mel band
  int mel_cnt[128];         // number of non-zero bins (<= 9)
  float mel_w[128][10];     // float32 band weights
  // v2 (200-point complex FFT of the even/odd-packed frame, 20 x 10 Cooley-Tukey)
  float hann2[200][2];      // (hann[2m], hann[2m + 1]) / 32768
  float tw[20][10][2];      // W200^(k1 * n2)
  float w400k[101][2];      // W400^k, k = 0..100 (even/odd split)
  int mel_taps_lo, mel_taps_hi;   // max non-zeros over bands 0..63 / 64..127
};

struct OdFeArgs {
  const int16_t* pcm;
  int64_t clip_stride;
  const int32_t* lens;      // nullable
  int32_t clip_len;
  const OdFeTables* tables; // device copy
  float* db;                // [n,128,151] nullable
  float* norm;              // [n,128,151] nullable
  float* zcr;               // [n,151]     nullable
  uint8_t* img;             // [n,128,151,3] nullable
  float* scratch;           // [n,151,128] mel-power scratch (frame-major), required
};

void od_fe_build_tables(OdFeTables* t);
bool od_fe_tables_ok(const OdFeTables& t);   // the mel tap counts fit the kernel's unrolling
size_t od_fe_smem_bytes();
hipError_t od_fe_launch(const OdFeArgs& a, int64_t n_clips, hipStream_t stream);
