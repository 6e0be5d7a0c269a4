// SpeakerIdentification front-end kernel interface (see si_fe.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct SiFeTables {
  double w256[16][16][2];   // W256^(n2*k1)
  double w512[257][2];      // W512^k
  double w16[16][2];        // W16^e
  int fb_lo[26];            // filter j covers bins [fb_lo[j], fb_hi[j])
  int fb_hi[26];
  double fb_w[26][48];      // weights of filter j for bins fb_lo[j] + i
  double dct[13][26];       // ortho DCT-II rows 0..12 times the lifter (row 0 unused: log energy)
  // v2 filterbank: segment s = bins [bin[s], bin[s+1]) (s = 0..26) is the rising edge of filter s
  // and the falling edge of filter s-1; it is cut into sub-segments of <= 8 bins
  int n_sub;                // number of sub-segments (<= SI_FE_MAX_SUB)
  int sub_start[48];        // first bin of sub-segment u
  int sub_cnt[48];          // bins in u (1..8)
  int sub_d0[48];           // sub_start[u] - bin[s(u)]: offset of its first bin inside the segment
  int seg_sub[28];          // sub-segments of segment s: [seg_sub[s], seg_sub[s+1])
  double inv_w[27];         // 1 / (bin[s+1] - bin[s])
};
constexpr int SI_FE_MAX_SUB = 48;

struct SiFeArgs {
  const int16_t* pcm;
  int64_t clip_stride;
  const int32_t* lens;      // nullable (clip mode)
  int32_t clip_len;
  int64_t seq_len;          // > 0: sequence mode -- block s = 256-frame window s of one signal
  const SiFeTables* tables;
  float* feat;              // [n,256,ldf]
  int ldf;                  // feature row stride: 39 (0 = 39), or 40 with a zero 40th column
  uint8_t* silent;          // [n] nullable (clip mode only)
};

void si_fe_build_tables(SiFeTables* t);
bool si_fe_tables_ok(const SiFeTables& t);
hipError_t si_fe_launch(const SiFeArgs& a, int64_t n_blocks, hipStream_t stream);
