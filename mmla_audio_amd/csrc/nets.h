// Small network kernels around the conv GEMM: OD stem, pooling/reduction glue, BiLSTM, heads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// OD stem Conv2D 1x1 3->16 on the decoded PNG (uint8) or a float NHWC input.
hipError_t od_stem_launch(const uint8_t* img_u8, const float* img_f32, int64_t n_pix, int ldw,
                          const float* w /*[3][16]*/, const float* b /*[16]*/, float* y,
                          hipStream_t s);
// Lambda(K.mean(x, axis=1)): [n, h, w, c] -> [n, w, c]
hipError_t mean_h_launch(const float* x, int n, int h, int w, int c, float* y, hipStream_t s);
// MaxPool1D(2, 'same') on [n, t, c] -> [n, ceil(t/2), c]
hipError_t maxpool_t2_launch(const float* x, int n, int t, int c, float* y, hipStream_t s);
// SI tail: BatchNorm -> ReLU -> AveragePooling1D(4) on [n, t, c] -> [n, t/4, c]
hipError_t bn_relu_avgpool4_launch(const float* x, int n, int t, int c, const float* scale,
                                   const float* shift, float* y, hipStream_t s);
// Bidirectional(LSTM(256), merge 'concat') last state.  seq [n, T, D]; wcat[dir] =
// [(256 + D) x 1024] (recurrent kernel rows first, then input kernel rows); bias[dir] [1024];
// out [n, 512] = [h_fwd(T-1), h_bwd(after x[0])].
hipError_t bilstm_launch(const float* seq, int n, int T, int D, const float* wcat_fwd,
                         const float* wcat_bwd, const float* bias_fwd, const float* bias_bwd,
                         float* out, hipStream_t s);
// The same BiLSTM on the f16 MFMA with 3xFP16 products (error-compensated hi/lo splits, f32
// accumulation); w*h / w*l = bilstm_h3_split_weights(wcat): 1024 x (256 + D) fp16 bits in MFMA fragment order.
hipError_t bilstm_h3_launch(const float* seq, int n, int T, int D, const uint16_t* wfh,
                            const uint16_t* wfl, const uint16_t* wbh, const uint16_t* wbl,
                            const float* bias_fwd, const float* bias_bwd, float* out,
                            int* range_flag /*nullable: set when |x| >= 65504 / 64*/,
                            float ws_fwd, float ws_bwd, hipStream_t s);
// The same for n <= bilstm_h3_split_max_clips() with each direction's eight hidden-unit groups on
// eight workgroups per 32 clips (h exchanged through ws between steps; bit-identical).  ws:
// bilstm_h3_split_ws_bytes() of device memory owned by the stream.  A workgroup that gave up waiting
// for the others (after `spin` polls; 0: the default bound; < 0: at the first wait, a test hook) writes NaN for its units and sets int
// word 63 of ws and *timeout_flag (nullable): the caller must not use that launch's outputs.
hipError_t bilstm_h3_split_launch(const float* seq, int n, int T, int D, const uint16_t* wfh,
                                  const uint16_t* wfl, const uint16_t* wbh, const uint16_t* wbl,
                                  const float* bias_fwd, const float* bias_bwd, float* out,
                                  int* range_flag, float ws_fwd, float ws_bwd, void* ws,
                                  int* timeout_flag, int spin, hipStream_t s);
size_t bilstm_h3_split_ws_bytes();
int bilstm_h3_split_max_clips();
// split at the direction's power-of-two weight scale ws (the kernel's ws_fwd / ws_bwd)
void bilstm_h3_split_weights(const float* wcat, int D, uint16_t* hi, uint16_t* lo, float ws);
// OD head: LeakyReLU(0.3) -> Dense(512 -> 2) -> softmax; probs [n,2], argmax [n] (nullable).
// The 'silent' gate of record_on_pc.py:141-154: with clip_len >= 0, clips with fewer than 4000
// samples (lens[i], or clip_len when lens is null) get argmax -1 and silent[i] = 1 (nullable).
hipError_t od_head_launch(const float* h, int n, const float* w /*[512][2]*/, const float* b,
                          float* probs, int32_t* argmax, const int32_t* lens, int clip_len,
                          uint8_t* silent, hipStream_t s);
// SI head activation on logits [n, ld]: softmax (head 0) or sigmoid (head 1) over the first k;
// argmax [n] (-1 where silent[i] != 0).
hipError_t si_head_launch(const float* logits, int n, int k, int ld, int head, float* probs,
                          int32_t* argmax, const uint8_t* silent, hipStream_t s);
