// One SpeakerIdentification res_unit without pooling as a single fused kernel.  See siu.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct SiuArgs {
  const float* x;          // [n * t, C] the unit's input (raw: also its residual), rows of all clips
  float* y;                // [n * t, C] x + Conv1D_b(ReLU(BN_mid(Conv1D_a(ReLU(BN_in(x)))))), y != x
  const uint16_t* wah;     // the two Conv1D(C, 3) weights, conv_h3_split_weights layout (cin = cout = C)
  const uint16_t* wal;
  const uint16_t* wbh;
  const uint16_t* wbl;
  const float* ba;         // biases [C]
  const float* bb;
  const float* s_in;       // folded BatchNorms [C]: v * s + t
  const float* t_in;
  const float* s_mid;
  const float* t_mid;
  float ua, ub;            // 1 / (2^4 x the weight tensor's split scale), conv_h3's unscale
  int n, t;                // clips, rows per clip (pool units: pooled rows, (t_src + 1) / 2)
  int* range_flag;         // nullable: an operand split into fp16 left the fp16 range
  // pool units only (sipu_launch): x is [n * t_src, CIN]; the shortcut Conv1D(C, 1, strides=2)
  int t_src;
  const uint16_t* wsh;     // its weight, conv_h3_split_weights layout (cin = CIN, cout = C)
  const uint16_t* wsl;
  const float* bs;         // its bias [C]
  float us;                // its unscale
  // siu_launch with seq set (the last unit, siu_final_supported): instead of y, seq [n * t / 4, C] =
  // AveragePooling1D(4)(ReLU(x_out * fs + ft)) (the final BatchNormalization, folded)
  float* seq;
  const float* fs;
  const float* ft;
  uint32_t tdiv_m, tdiv_s;   // set by the launchers: row / t as a multiply-high (callers leave 0)
};

bool siu_supported(int c);
bool siu_final_supported(int c);
hipError_t siu_launch(const SiuArgs& a, int c, hipStream_t stream);
// two consecutive units without pooling (a then b, b.x / a.y unused: the intermediate stays on chip);
// b.seq set: b is the last unit (siu_final_supported's epilogue)
bool siu_pair_supported(int c);
hipError_t siu_pair_launch(const SiuArgs& a, const SiuArgs& b, int c, hipStream_t stream);
// a pool unit p and the two units after it (p.x the input, b.y / b.seq the output: the
// intermediates stay on chip)
bool siu_triple_supported(int cin, int c);
hipError_t siu_triple_launch(const SiuArgs& p, const SiuArgs& a, const SiuArgs& b, int cin, int c,
                             hipStream_t stream);
// the pool unit (speaker_identification.py:170-172 + 173-188) with t1 kept on chip
bool sipu_supported(int cin, int c);
hipError_t sipu_launch(const SiuArgs& a, int cin, int c, hipStream_t stream);
