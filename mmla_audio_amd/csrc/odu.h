// One OverlapDetection res_block of the 64- / 128-channel stages (blocks 4-9) as a single fused kernel.
// See odu.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct OduArgs {
  const float* x;          // [n, h, w, cin] the block's input (raw: also the residual of blocks 5-6, 8-9)
  float* y;                // [n, h, w, c] (pool blocks: [n, h / 2, w / 2, c]); y != x
  const uint16_t* wah;     // Conv2D(c, 3x3) weights, conv_h3_split_weights layout
  const uint16_t* wal;
  const uint16_t* wbh;     // Conv2D(c, (4, 1)) weights, conv_h3_split_weights layout
  const uint16_t* wbl;
  const float* ba;         // biases [c]
  const float* bb;
  const float* s_in;       // folded BatchNorms: v * s + t (BN_in over cin, BN_mid over c)
  const float* t_in;
  const float* s_mid;
  const float* t_mid;
  float ua, ub;            // 1 / (2^4 x the weight tensor's split scale): conv_h3's unscale
  int n;                   // clips
  int* range_flag;         // nullable: an operand split into fp16 left the fp16 range
  // pool blocks (4, 7): the shortcut Conv2D(c, 1x1, strides 2) of x, conv_h3_split_weights layout
  const uint16_t* wsh;
  const uint16_t* wsl;
  const float* bs;
  float us;
};

// block geometry (h, w, cin, c, pool) handled by odu_launch
bool odu_supported(int h, int w, int cin, int c, bool pool);
hipError_t odu_launch(const OduArgs& a, int h, int w, int cin, int c, bool pool, hipStream_t stream);
