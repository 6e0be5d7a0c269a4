// One fused OD-NET res_block on gfx950 f16 MFMA (3xFP16).  See resblk.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct ResBlkArgs {
  const float* x;          // [N, H, W, CIN] block input (raw: also the residual of non-pool blocks)
  const uint16_t* w1h;     // Conv2D(3x3) fp16 hi [C][K1PAD], k = (dy * 3 + dx) * CIN + ci
  const uint16_t* w1l;     //                 lo = fp16(w * 2^8 - hi), hi = fp16(w * 2^8)
  const float* b1;         // [C]
  const float* s1;         // BatchNorm before the 3x3 conv, folded: y = x * s1 + t1   [CIN]
  const float* t1;
  const uint16_t* w2h;     // Conv2D((4,1)) fp16 hi [C][4 * C], k = dy * C + ci
  const uint16_t* w2l;
  const float* b2;         // [C]
  const float* s2;         // BatchNorm before the (4,1) conv, folded [C]
  const float* t2;
  const uint16_t* wsh;     // pool blocks: Conv2D(1x1, stride 2) shortcut, fp16 hi [C][KSC], k = ci
  const uint16_t* wsl;     //   (KSC = CIN rounded up to 32)
  const float* bs;         //   shortcut bias [C]
  const uint8_t* img8;     // block 1 fused with the stem: the decoded image [N, H, W, 3] (uint8)
  const float* imgf;       //   or float NHWC; x is then unused
  const float* wst;        //   stem Conv2D(16, 1x1) weights [3][ldst] and bias [16]
  const float* bst;
  int ldst;
  float* y;                // non-pool: [N, H, W, C] = x + conv;  pool: [N, ceil(H/2), ceil(W/2), C]
  int n, h, w;             //   = MaxPool2D(2, 'same')(conv) + Conv2D(1x1, stride 2)(x)
  int tiles_h, tiles_w;    // set by resblk_launch
  int* range_flag;         // nullable: set to 1 when an operand split into fp16 is >= 65504 / inf
  // 1 / (2^4 x the power-of-two weight scale) of GEMM 1 (w1), GEMM 2 (w2) and the shortcut (ws)
  float u1, u2, us;
};

// K of the 3x3 conv padded to the MFMA k-step (32).
int resblk_k1pad(int cin);
// True when (cin, c, pool) has a fused kernel.
bool resblk_supported(int cin, int c, bool pool);
hipError_t resblk_launch(ResBlkArgs a, int cin, int c, bool pool, hipStream_t stream);
// Host: float32 Keras weights [taps][cin][cout] -> fp16 hi/lo [cout][kpad] with k = tap * cin + ci
// (zero for k >= taps * cin); frag: the 16x16x32 MFMA B-fragment order [k / 32][cout / 16][64 lanes][8]
// (GEMM 1's 3x3 and GEMM 2's conv(4,1) weights; the 1x1 shortcut keeps the [cout][kpad] rows).
void resblk_split_weights(const float* w, int taps, int cin, int cout, int kpad, uint16_t* hi,
                          uint16_t* lo, bool frag, float wscale);

// Blocks 1-3 as rolling 16-column strips on 32x32x16 MFMAs (rbs.hip).  The weights are in the
// conv_h3 layout (conv_h3_split_weights: w1h / w1l the 3x3, w2h / w2l the (4,1), wsh / wsl the 1x1
// shortcut); a.h / a.w are the block's input size.  Block 1 (pool) needs the stem fused (img8 / imgf).
bool rbs_supported(int h, int w, int cin, int c, bool pool);
hipError_t rbs_launch(const ResBlkArgs& a, int cin, int c, bool pool, hipStream_t stream);
