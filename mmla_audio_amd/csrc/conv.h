// Implicit-GEMM convolution (NHWC, Keras 'same' padding) on gfx950 f32 MFMA, with fused prologue
// (BatchNorm + activation on the input as it is loaded) and epilogue (bias, residual add, or
// residual + 2x2 'same' max-pool of another tensor).  See conv.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

enum ConvPro { PRO_NONE = 0, PRO_BN_ELU = 1, PRO_BN_RELU = 2 };
enum ConvEpi { EPI_BIAS = 0, EPI_ADD = 1, EPI_ADD_POOL = 2 };

struct ConvArgs {
  const float* x;      // [N, H, W, Cin]
  const float* wt;     // [KH, KW, Cin, CoutPad]  (Keras layout, columns padded to a multiple of 32)
  const float* bias;   // [CoutPad]
  const float* scale;  // [Cin] prologue BN scale  (gamma / sqrt(var + eps))
  const float* shift;  // [Cin] prologue BN shift  (beta - mean * scale)
  const float* res;    // EPI_ADD: [N, Ho, Wo, Cout]; EPI_ADD_POOL: [N, Hp, Wp, Cout] pooled 2x2
  float* y;            // [N, Ho, Wo, ldy]
  int n, h, w, cin;
  int ho, wo, cout, cout_pad, ldy;
  int kh, kw, stride, pad_h, pad_w;
  int hp, wp;          // EPI_ADD_POOL source spatial dims
  int pro, epi;
};

hipError_t conv_launch(const ConvArgs& a, hipStream_t stream);
