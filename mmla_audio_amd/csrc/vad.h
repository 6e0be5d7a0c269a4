// Silence removal of the reference's save_wave_file(silence_remove=True): webrtcvad.Vad(mode)
// decisions on 30 ms frames + vad_collector + the rewrite of the voiced frames.  See vad.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// One webrtcvad.Vad instance (WebRTC VadInstT, the 16 kHz path), kept in device memory.
struct VadState {
  int32_t ds[2];                    // 16 -> 8 kHz all-pass downsampler
  int32_t frame_counter;
  int16_t over_hang, num_of_speech;
  int16_t noise_means[12], speech_means[12], noise_stds[12], speech_stds[12];
  int16_t low_value[96], age[96];   // FindMinimum: 16 smallest features per channel and their age
  int16_t mean_value[6];
  int16_t upper[5], lower[5];       // splitting-filter all-pass states
  int16_t hp[4];                    // 80 Hz high-pass state
  int16_t oh1, oh2, individual, total;   // mode thresholds for 30 ms frames
};

struct VadArgs {
  const int16_t* pcm;      // item i at pcm + i * stride
  int64_t stride;
  const int32_t* lens;     // nullable: every item has clip_len samples
  int32_t clip_len;
  int64_t n_items;
  int64_t items_per_stream; // stream s owns items [s * ips, (s + 1) * ips), processed in order
  VadState* state;          // [n_items / ips]
  uint8_t* speech;          // [n_items][max_frames] per-frame decisions (written by the VAD kernel,
                            //   read by the collector)
  int32_t max_frames;
  int16_t* out;             // item i's voiced frames at out + i * stride
  int32_t* out_lens;        // [n_items]
};

// Host: a fresh webrtcvad.Vad(mode) (WebRtcVad_Init + set_mode); false for a mode outside 0..3.
bool vad_init_state(VadState* s, int mode);
// Frames of an item of `len` samples (frame_generator: k * 480 + 480 < len).
__host__ __device__ inline int vad_frames(int64_t len) { return len > 480 ? (int)((len - 1) / 480) : 0; }
// Per-frame decisions of every item, stream by stream (one thread per stream).
hipError_t vad_speech_launch(const VadArgs& a, hipStream_t s);
// vad_collector + the rewrite from `speech` (one wave per item).
hipError_t vad_collect_launch(const VadArgs& a, hipStream_t s);
// soundfile's PCM_16 write of float audio (libsndfile f2s: (short) lrintf(x * 0x7FFF)).
hipError_t pcm16_launch(const float* y, int64_t n, int16_t* out, hipStream_t s);
