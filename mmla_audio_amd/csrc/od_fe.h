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
size_t od_fe_smem_bytes();
hipError_t od_fe_launch(const OdFeArgs& a, int64_t n_clips, hipStream_t stream);
