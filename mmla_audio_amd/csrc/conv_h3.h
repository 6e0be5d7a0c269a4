// Halo-tiled implicit-GEMM convolution on gfx950 f16 MFMA with error-compensated 3xFP16 products.
// See conv_h3.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct ConvH3Args {
  const float* x;        // [N, H, W, Cin] float32 NHWC
  const uint16_t* wh;    // [KH*KW][CoutPad][CinPad] fp16 hi(w)
  const uint16_t* wl;    // [KH*KW][CoutPad][CinPad] fp16 lo = fp16(w * 2^8 - hi), hi = fp16(w * 2^8)
  const float* bias;     // [CoutPad]
  const float* scale;    // [Cin] prologue BN scale (nullable when pro == 0)
  const float* shift;    // [Cin]
  const float* res;      // EPI_ADD residual [N, H, W, Cout] (may alias y)
  float* y;              // [N, H, W, Cout]  or pooled [N, ceil(H/2), ceil(W/2), Cout] (pool_out)
  int n, h, w, cin, cin_pad, cout, cout_pad;
  int kh, kw, pad_h, pad_w;
  int th, tw;            // output tile (th * tw <= 128)
  int tiles_h, tiles_w;
  int pro, epi, pool_out;
  int pool_in;           // Conv1D only: x is [N, h_in, 1, Cin] and the conv reads MaxPool1D(2, same) of it
  int h_in;
  int* range_flag;       // nullable: set to 1 when a staged operand is >= 65504 in magnitude / inf
  // shortcut Conv(1x1, stride 2) of sc_x as a 3xFP16 GEMM in the epilogue:
  //   pooled blocks (pool_out): sc_x [N, H, W, sc_cin], added to the pooled output
  //     (overlap_detector_temp.py:265-270);
  //   Conv1D (tw 1) with epi EPI_ADD: sc_x [N, sc_h, 1, sc_cin] (sc_h input rows per clip), the
  //     residual the output adds instead of res (speaker_identification.py:179-186 pool units)
  const float* sc_x;     // nullable: no shortcut
  const uint16_t* sc_wh; // conv_h3_split_weights layout, kh = kw = 1
  const uint16_t* sc_wl;
  const float* sc_bias;  // [cout_pad]
  int sc_cin;            // multiple of 16
  int sc_h;              // Conv1D: input rows per clip
  // 1 / (2^4 activation scale x the power-of-two weight scale of conv_h3_split_weights): per weight
  // tensor, so that any finite checkpoint fits the fp16 split (capi.cpp pick_wscale)
  float unscale;
  float sc_unscale;
};

// Picks the tile and launches; returns hipErrorInvalidValue for unsupported shapes.
hipError_t conv_h3_launch(ConvH3Args a, hipStream_t stream);
// Host: split float32 weights [kh,kw,cin,cout] into fp16 hi/lo, per tap in MFMA fragment order
// [cin_pad / 16][cout_pad / 32][64 lanes][8] (conv_h3_kernel).
void conv_h3_split_weights(const float* w, int kh, int kw, int cin, int cout, int cin_pad,
                           int cout_pad, uint16_t* hi, uint16_t* lo, float wscale);
