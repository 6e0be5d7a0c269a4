// OverlapDetection front-end kernel interface (see od_fe.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct OdFeTables {
  int mel_start[128];       // first non-zero bin of each Slaney mel band
  int mel_cnt[128];         // number of non-zero bins (<= 10)
  float mel_w[128][10];     // float32 band weights
  // two-stage matrix DFT on the f16 MFMA (od_fe.hip): the 32x32x16 A fragments of both stages,
  // fp16 hi / lo bit patterns in fragment order [gemm][k-step][hi, lo][lane][8]
  //   stage 1, gemm n1 = 0..15:  rows c = 2 k2 + ri, k = n2      (window x DFT-25, x 2^8)
  //   stage 2, gemm k2' = 0..12: rows 2 i + ri,    k = 2 n1 + ri (twiddle x DFT-16, x 2^8)
  uint16_t a1[16][2][2][64][8];
  uint16_t a2[13][2][2][64][8];
  // mel on the f32 MFMA (v_mfma_f32_16x16x4f32): 8 tiles of 16 bands x the two 16-frame halves of
  // a 32-frame tile = 16 units, one per wave.  Band tile bt reads P rows mel_bt_bin0[bt] .. + 4 nk - 1
  // (nk = mel_bt_nk[bt], a multiple of 4) against A fragments mel_bt_frag[bt] .. + nk - 1
  int mel_bt_bin0[8], mel_bt_nk[8], mel_bt_frag[8];
  int mel_unit[16];         // wave -> 2 bt + frame half; per SIMD (waves w, w + 4, w + 8, w + 12) balanced
  float mel_a[64][64];      // A fragments [frag][lane]: A[m = l & 15][k = l >> 4] = mel_w[16 bt + m][bin0 + 4 j + k] x 2^-38
  uint16_t zero16;          // a zero sample: the target of reads past a clip's length
};

struct OdFeArgs {
  const int16_t* pcm;
  const float* pcm_f32;     // nullable: float PCM (librosa.load scale, y = x / 32768) instead of pcm
  int64_t clip_stride;
  const int32_t* lens;      // nullable
  int32_t clip_len;
  const OdFeTables* tables; // device copy
  float* db;                // [n,128,151] nullable
  float* norm;              // [n,128,151] nullable
  float* zcr;               // [n,151]     nullable
  uint8_t* img;             // [n,128,151,3] nullable
  int* range_flag;          // nullable: set when a float PCM sample is outside the split range
                            // (|y| >= 8188 or not finite: y 2^3 must fit fp16)
};

void od_fe_build_tables(OdFeTables* t);
bool od_fe_tables_ok(const OdFeTables& t);   // the mel schedule fits the kernel's LDS rows and fragments
hipError_t od_fe_launch(const OdFeArgs& a, int64_t n_clips, hipStream_t stream);
