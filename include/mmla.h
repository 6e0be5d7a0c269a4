/*
 * mmla.h -- C ABI of the MI355X-native mmla-audio hot path (libmmla.so).
 *
 * The reference (lizaibeim/mmla-audio) has no FFI of its own: its per-clip path is a set of plain
 * Python functions over librosa / python_speech_features / TensorFlow.  Each entry
 * point below replaces one of those call sites; the Python drop-in shim (mmla_audio_amd/) binds them
 * with ctypes under the reference's own names (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - Every function returns MMLA_OK (0) or a negative MMLA_E_* code; the message is in
 *     mmla_last_error(ctx).  Nothing throws across the ABI.
 *   - Buffers are caller-owned.  By default they are HOST pointers (the call copies in and out and
 *     is synchronous).  With MMLA_DEVICE_PTR they are device pointers on the context's GPU and the
 *     call only enqueues work on the context stream (mmla_set_stream), returning immediately.
 *   - A context is not thread-safe: use one per thread / per GPU.  The multi-GPU driver (one process
 *     per GPU, RCCL all-gather of logits) lives above this ABI.
 *   - PCM is 16 kHz mono int16; clip c starts at pcm + c * clip_stride (in samples) and has
 *     lens[c] valid samples (lens == NULL: every clip has clip_len samples).  Without lens the
 *     stride may be smaller than clip_len: overlapping windows of one signal (the offline
 *     segmentation of overlap_detection_post_processing.py:23-85 with step < window).
 */
#ifndef MMLA_H_
#define MMLA_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMLA_ABI_VERSION 2

enum mmla_status {
  MMLA_OK = 0,
  MMLA_E_INVALID = -1,   /* bad argument (null pointer, negative size, unknown model kind) */
  MMLA_E_HIP = -2,       /* HIP runtime error */
  MMLA_E_NOWEIGHTS = -3, /* forward called before mmla_load_weights for that model */
  MMLA_E_OOM = -4,       /* device allocation failed */
  MMLA_E_SHAPE = -5,     /* packed weight blob has the wrong number of floats */
  MMLA_E_RANGE = -6      /* 3xFP16: an operand left the fp16 range in a device-pointer call */
};

enum mmla_model { MMLA_MODEL_OD = 0, MMLA_MODEL_SI = 1 };
enum mmla_head { MMLA_HEAD_SOFTMAX = 0, MMLA_HEAD_SIGMOID = 1 };

#define MMLA_DEVICE_PTR 0x1u /* data pointers are device pointers; call is asynchronous */

/* OD front-end geometry (overlap_features_generator.py:39-42,73-81) */
#define MMLA_OD_MELS 128
#define MMLA_OD_FRAMES 151
#define MMLA_OD_CLIP 24000
/* SI front-end geometry (speaker_identification.py:386-395) */
#define MMLA_SI_FRAMES 256
#define MMLA_SI_DIMS 39
#define MMLA_SI_SILENT_LEN 4000

typedef struct mmla_ctx mmla_ctx;

int mmla_abi_version(void);

/* CRC-32C (Castagnoli) of n bytes -> *crc (host only, no context or device): the checksum TF's
 * tensor bundle stores per tensor (BundleEntryProto.crc32c, masked as LevelDB does; tfbundle.py
 * verifies every tensor it loads from variables.data-*, replacing the check of
 * tf.keras.models.load_model at record_on_pc.py:88 / SI record_on_pc.py:77). */
int mmla_crc32c(const void* data, int64_t n, uint32_t* crc);

/* PNG scanline reconstruction (host only, no context or device): `raw` is the inflated IDAT stream
 * of a non-interlaced image, h rows of 1 filter-type byte + row_bytes bytes; `bpp` = bytes per
 * complete pixel (>= 1; 1 for sub-byte depths).  Undoes filters 0-4 (None, Sub, Up, Average, Paeth;
 * PNG spec section 9) into out[h * row_bytes].  MMLA_E_INVALID on an unknown filter type.  Replaces
 * libpng's row reconstruction inside tf.image.decode_png (record_on_pc.py:157,
 * overlap_detection_post_processing.py:205; mmla_audio_amd/tf_compat/image.py). */
int mmla_png_unfilter(const uint8_t* raw, int64_t h, int64_t row_bytes, int32_t bpp, uint8_t* out);

/* Create a context on HIP device `device` (owns a stream, device workspaces and loaded weights). */
int mmla_create(int device, mmla_ctx** out);
int mmla_destroy(mmla_ctx* ctx);
const char* mmla_last_error(const mmla_ctx* ctx);
/* Use an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL = the context's
 * own stream, a blocking stream (it orders with the legacy NULL stream, i.e. with PyTorch's default
 * stream; work on any other stream that produces a call's device inputs must be ordered by the
 * caller, e.g. by passing that stream here).  The new stream first waits (hipStreamWaitEvent) for
 * the work already enqueued on the old one, which still uses this context's workspaces. */
int mmla_set_stream(mmla_ctx* ctx, void* hip_stream);
/* Wait for the context stream; returns MMLA_E_RANGE (see mmla_range_check) if a device-pointer call
 * since the last check overflowed the fp16 range, MMLA_E_HIP if one ran the split BiLSTM (batches of
 * <= 128 clips) and a workgroup of it timed out (NaN probabilities; host-pointer calls re-run such a
 * micro-batch on the unsplit kernel instead, bit-identical). */
int mmla_synchronize(mmla_ctx* ctx);
/*
 * Arithmetic of the spatial convolutions (98 % of OD-NET FLOPs) and the BiLSTM:
 *   MMLA_PREC_F16X3 (default) error-compensated 3xFP16 on f16 MFMA: operands split hi + 2^-11 lo,
 *                   hi*hi + hi*lo + lo*hi accumulated in f32 (~22-bit products, f32 accumulation);
 *                   needs |activations| < 65504 in the fused res_blocks, < 4094 in the halo-tiled
 *                   convs (split x 2^4) and < 1023 in the LSTM (x 2^6).  Each weight tensor is split
 *                   at its own power-of-two scale (2^8 for max |w| in [1/16, 255.9), else the one
 *                   putting max |w| in [2^13, 2^14)), so any finite checkpoint stays on this path;
 *                   a tensor holding inf / NaN makes that model run exact f32 (decided at
 *                   mmla_load_weights).  Range guard: every kernel that splits an activation flags
 *                   a value outside its range.  Host-pointer calls then re-run the micro-batch in exact f32
 *                   (counted by mmla_range_check); device-pointer calls report MMLA_E_RANGE from
 *                   the next mmla_range_check / mmla_synchronize.
 *   MMLA_PREC_F32   exact f32 MFMA (v_mfma_f32_32x32x2_f32), 1/5.3 of the throughput.
 * The front-ends (OD f32, SI f64), the OD stem Conv2D(1x1), the OD Dense(2) head and the softmax /
 * sigmoid are the same in both modes; under MMLA_PREC_F16X3 the strided 1x1 shortcuts (OD blocks 1,
 * 4, 7; SI pool units) and the SI Dense(K) run 3xFP16 with the convolutions they are fused into.
 */
enum mmla_precision { MMLA_PREC_F32 = 0, MMLA_PREC_F16X3 = 1 };
int mmla_set_precision(mmla_ctx* ctx, int mode);
/* Waits for the context stream.  *f32_reruns (nullable) = host-pointer micro-batches re-run in
 * exact f32 so far; returns MMLA_E_RANGE (and clears the flag) if a device-pointer call since the
 * last check split an out-of-range operand -- its results are invalid. */
int mmla_range_check(mmla_ctx* ctx, int64_t* f32_reruns);
/*
 * Clips per internal micro-batch (activation memory).  0 = sized at each call from the device's
 * free memory, capped at 16384 (OD) / 65536 (SI) clips; an allocation failure halves it and
 * retries.  Per-clip device footprint of a micro-batch: OD ~7.6 MB (three n*128*151*32 f32
 * activation buffers + image + front-end scratch), so the 16384-clip default holds ~124 GB;
 * SI ~0.14 MB (65536 clips ~9 GB).  Weights: OD ~12 MB, SI ~10 MB.  Workspaces are kept for
 * reuse until mmla_release_workspace or mmla_destroy.
 */
int mmla_set_microbatch(mmla_ctx* ctx, int64_t od_clips, int64_t si_clips);
/* The micro-batch sizes the next call would use. */
int mmla_get_microbatch(mmla_ctx* ctx, int64_t* od_clips, int64_t* si_clips);
/* Free every device workspace of the context (after its stream drains). */
int mmla_release_workspace(mmla_ctx* ctx);

/*
 * Load network weights from the packed float32 blob (host memory) in the canonical order of
 * mmla_audio_amd/weights.py spec(): ascending Keras `layer_with_weights-k`; conv/dense = kernel,
 * bias; BatchNorm = gamma, beta, moving_mean, moving_variance; Bidirectional LSTM = forward
 * kernel, recurrent_kernel, bias, backward kernel, recurrent_kernel, bias.  Keras layouts.
 * Replaces tf.keras.models.load_model(...) (record_on_pc.py:88; SI record_on_pc.py:77).
 * n_classes: OD must be 2; SI = 630 (base model) or N speakers (deployed head).
 * head: MMLA_HEAD_SOFTMAX (base Dense(630, softmax), speaker_identification.py:215) or
 *       MMLA_HEAD_SIGMOID (deployed customized_dense, speaker_identification.py:409).
 */
int mmla_load_weights(mmla_ctx* ctx, int model_kind, const float* packed, int64_t n_floats,
                      int32_t n_classes, int32_t head);

/*
 * OverlapDetection front-end, replaces OverlapFeaturesGenerator.generate_mels / generate_zcr /
 * generate_zcr_image + the PNG round trip (overlap_features_generator.py:65-151;
 * record_on_pc.py:156-158).  Per clip (first 24000 samples, zero-padded if shorter):
 *   db      [n,128,151] f32  power_to_db(melspectrogram, ref=max, top_db=80)   (nullable)
 *   norm_db [n,128,151] f32  normalize_matrix(db) in [0,1] (NaN for digital silence) (nullable)
 *   zcr     [n,151]     f32  zero_crossing_rate(frame 400, hop 160)                 (nullable)
 *   img     [n,128,151,3] u8 the decoded PNG the model reads: rows flipped
 *                            (origin="lower"), R = trunc(255*zcr), G = B = trunc(255*(1-norm))
 *                                                                                   (nullable)
 */
int mmla_od_features(mmla_ctx* ctx, const int16_t* pcm, int64_t n_clips, int64_t clip_stride,
                     const int32_t* lens, int32_t clip_len, float* db, float* norm_db, float* zcr,
                     uint8_t* img, uint32_t flags);
/* Same on float PCM in librosa.load's scale (y = x / 32768 for 16-bit files; |y| < 8188, since y 2^3 is
 * split into fp16 hi + lo -- a host call with a larger or non-finite sample in the read window returns
 * MMLA_E_RANGE, a device-pointer call reports it from the next mmla_range_check / mmla_synchronize): the
 * drop-in's path for what librosa.load(path, sr=None, mono=True) returns from a WAV that is not
 * 16-bit mono (stereo downmixed by the channel mean, 8/24/32-bit and float files) --
 * overlap_features_generator.py:72,93.  Zero crossings treat |y| <= 1e-10 as 0, as librosa. */
int mmla_od_features_f32(mmla_ctx* ctx, const float* y, int64_t n_clips, int64_t clip_stride,
                         const int32_t* lens, int32_t clip_len, float* db, float* norm_db,
                         float* zcr, uint8_t* img, uint32_t flags);

/*
 * SpeakerIdentification front-end, replaces input_feature_gen (speaker_identification.py:372-398):
 * psf.mfcc(winlen .025, winstep .01, nfft 512) -> delta(.,2) -> delta(delta,2) -> [T,39] ->
 * zero-pad / truncate to 256 frames.  Clips with lens < 4000 are 'silent': silent[c] = 1 and
 * feat[c] is all zeros.  feat [n,256,39] f32 (float64 arithmetic inside); silent [n] u8 (nullable).
 */
int mmla_si_features(mmla_ctx* ctx, const int16_t* pcm, int64_t n_clips, int64_t clip_stride,
                     const int32_t* lens, int32_t clip_len, float* feat, uint8_t* silent,
                     uint32_t flags);

/*
 * Whole-signal SI features cut into 256-frame windows, replaces the conversation-level MFCC +
 * deltas + chunking of speaker_identification_post_processing.py:255-269 and
 * make_feature_experiment (speaker_identification.py:340-353).  pcm [n_samples] int16; window s
 * holds global frames [256 s, 256 s + 256) (deltas edge-padded at the true sequence ends, zero
 * rows past the last frame).  n_windows must be ceil(T / 256), T = psf frame count of n_samples.
 * feat [n_windows, 256, 39] f32.
 */
int mmla_si_features_seq(mmla_ctx* ctx, const int16_t* pcm, int64_t n_samples, int64_t n_windows,
                         float* feat, uint32_t flags);

/* OD-NET predict on float NHWC [n,128,151,3] (values 0..255) -> probs [n,2]
 * (model.predict, record_on_pc.py:159). */
int mmla_od_forward(mmla_ctx* ctx, const float* x_nhwc, int64_t n, float* probs, uint32_t flags);
/* Same on the uint8 image produced by mmla_od_features. */
int mmla_od_forward_u8(mmla_ctx* ctx, const uint8_t* img, int64_t n, float* probs, uint32_t flags);

/* SI-NET predict on [n,256,39] -> probs [n,K] (SI record_on_pc.py:136;
 * speaker_identification_post_processing.py:272). */
int mmla_si_forward(mmla_ctx* ctx, const float* x, int64_t n, float* probs, uint32_t flags);

/* Fused WAV->class pipelines (no PNG, no host round trip): probs [n,K] f32 (nullable),
 * argmax [n] i32 (nullable; -1 for 'silent' clips), silent [n] u8 (nullable).  'silent' = fewer
 * than 4000 samples (lens[c], or clip_len without lens): OD record_on_pc.py:141-154 logs it and
 * skips predict, SI speaker_identification.py:375-376 returns the 'silent' sentinel; their probs
 * are still computed (on the zero-padded clip) but carry no meaning. */
int mmla_od_pipeline(mmla_ctx* ctx, const int16_t* pcm, int64_t n_clips, int64_t clip_stride,
                     const int32_t* lens, int32_t clip_len, float* probs, int32_t* argmax,
                     uint8_t* silent, uint32_t flags);
int mmla_si_pipeline(mmla_ctx* ctx, const int16_t* pcm, int64_t n_clips, int64_t clip_stride,
                     const int32_t* lens, int32_t clip_len, float* probs, int32_t* argmax,
                     uint8_t* silent, uint32_t flags);

/*
 * Stationary spectral-gate noise reduction, replaces nr.reduce_noise(y_noise=noise, y=y, sr=sr,
 * stationary=True) (OverlapDetection/scripts/record_on_pc.py:208-212,
 * SpeakerIdentification/scripts/record_on_pc.py:189, speaker_identification_post_processing.py:171)
 * with noisereduce 2.0.x defaults (n_fft 1024, hop 256, n_std 1.5, 500 Hz x 50 ms mask smoothing,
 * chunk_size 600000, padding 30000).  sr must be 16000.
 * mmla_nr_set_noise: noise [n_noise] f32 (librosa.load output; the first chunk_size samples are
 * used) -> per-bin threshold kept in the context.
 * mmla_nr_reduce: y [n_signals, stride] f32, each signal `len` samples -> out [n_signals, len] f32;
 * signals longer than chunk_size are gated chunk by chunk with `padding` samples of context.
 */
int mmla_nr_set_noise(mmla_ctx* ctx, const float* noise, int64_t n_noise, int32_t sr,
                      uint32_t flags);
int mmla_nr_reduce(mmla_ctx* ctx, const float* y, int64_t n_signals, int64_t stride, int64_t len,
                   float* out, uint32_t flags);

/*
 * Silence removal, replaces save_wave_file(silence_remove=True) (OverlapDetection/scripts/
 * record_on_pc.py:214-226, frame_generator :229-243, vad_collector :246-295; the same functions in
 * SpeakerIdentification/scripts/record_on_pc.py:196 and speaker_identification_post_processing.py:
 * 176-187,225-251).  Frames of 30 ms (480 samples) that END BEFORE the item's last sample,
 * webrtcvad.Vad(mode).is_speech per frame (py-webrtcvad / WebRTC fixed-point VAD, 16 kHz path),
 * the 10-frame ring-buffer trigger (> 90 % voiced / unvoiced), and the voiced frames written back
 * in order: item i -> out + i * stride, out_lens[i] samples (a multiple of 480).
 * mmla_vad_reset: (re)creates n_streams independent detectors in the context.  The reference keeps
 * ONE module-level Vad(3) whose GMM state carries across clips; a stream is that object: its items
 * are processed in order, and its state persists across calls until the next reset.
 * mmla_vad_remove_silence: n_items = n_streams * items_per_stream; stream s owns items
 * [s * items_per_stream, (s + 1) * items_per_stream).  speech [n_items][max_frames] u8 receives the
 * per-frame decisions (nullable); max_frames 0 = the frames of the widest item.
 * mmla_vad_collect: the collector and rewrite alone, on caller-supplied decisions `speech`.
 * mmla_pcm16: sf.write(path, y, 16000) of float audio as PCM_16 (:212): (short) lrintf(y * 32767).
 */
int mmla_vad_reset(mmla_ctx* ctx, int64_t n_streams, int32_t mode);
int mmla_vad_remove_silence(mmla_ctx* ctx, const int16_t* pcm, int64_t n_items, int64_t stride,
                            const int32_t* lens, int32_t clip_len, int64_t items_per_stream,
                            int16_t* out, int32_t* out_lens, uint8_t* speech, int32_t max_frames,
                            uint32_t flags);
int mmla_vad_collect(mmla_ctx* ctx, const int16_t* pcm, int64_t n_items, int64_t stride,
                     const int32_t* lens, int32_t clip_len, const uint8_t* speech, int32_t max_frames,
                     int16_t* out, int32_t* out_lens, uint32_t flags);
int mmla_pcm16(mmla_ctx* ctx, const float* y, int64_t n, int16_t* out, uint32_t flags);

/*
 * Rate conversion of the offline pre-conditioning (resample.hip).
 * mmla_ratecv: pydub AudioSegment.set_frame_rate(outrate) on 16-bit PCM, i.e.
 *   audioop.ratecv(data, 2, nch, inrate, outrate, None) (OverlapDetection/scripts/
 *   overlap_detection_post_processing.py:120-121; SpeakerIdentification/scripts/
 *   speaker_identification_post_processing.py:159-160), bit-identical to CPython's audioop.
 *   pcm [n_frames][nch] interleaved -> out [out_frames][nch]; out_frames must be
 *   (n_frames - 1) * (outrate / g) / (inrate / g) + 1 with g = gcd(inrate, outrate) (0 for no input).
 * mmla_resample_sinc: resampy.resample(x, sr_orig, sr_new, filter=<half window>) on one float32
 *   channel -- librosa.load(path) at its default 22050 Hz uses filter 'kaiser_best'
 *   (speaker_identification_post_processing.py:142).  half_window [window_len] float64 is the
 *   filter's right half sampled num_table times per zero crossing (resampy sinc_window); n_out must
 *   be int(n * sr_new / sr_orig).  resampy's float64 time register, filter interpolation and float32
 *   accumulation are reproduced (library absent here: parity against resampy itself unpinned).
 */
int mmla_ratecv(mmla_ctx* ctx, const int16_t* pcm, int64_t n_frames, int32_t nch, int32_t inrate,
                int32_t outrate, int16_t* out, int64_t out_frames, uint32_t flags);
int mmla_resample_sinc(mmla_ctx* ctx, const float* x, int64_t n, int32_t sr_orig, int32_t sr_new,
                       const double* half_window, int64_t window_len, int32_t num_table, float* y,
                       int64_t n_out, uint32_t flags);

/*
 * Kernel tracing (replaces the reference's time.time() prints, overlap_detector_run.py:49-104).
 * When enabled, every kernel launch is bracketed by hipEvents on the context stream and its device
 * time is accumulated per stage together with the stage's algorithmic work (bytes for the
 * front-ends, FLOPs for the networks).  mmla_profile_read waits for the recorded events.
 */
#define MMLA_NSTAGES 7
enum mmla_stage {
  MMLA_STAGE_OD_FE = 0, /* work = algorithmic HBM bytes */
  MMLA_STAGE_SI_FE = 1, /* work = algorithmic HBM bytes */
  MMLA_STAGE_CONV = 2,  /* work = FLOPs (2 * MACs, unpadded) */
  MMLA_STAGE_LSTM = 3,  /* work = FLOPs */
  MMLA_STAGE_GLUE = 4,  /* stem, pooling, mean: work = FLOPs */
  MMLA_STAGE_HEAD = 5,  /* dense + softmax / sigmoid: work = FLOPs */
  MMLA_STAGE_NR = 6     /* noise gate: work = algorithmic HBM bytes (signal in + out) */
};
int mmla_profile_enable(mmla_ctx* ctx, int on);

/* Layer-wise parity tap (tests): run OD-NET on host float NHWC x[n,128,151,3] up to `stage`
 * (0 = stem conv, 1..9 = after res_block 1..9 in NHWC, 10 = mean over H [n,19,128],
 * 11 = BiLSTM output [n,512]) and copy that tensor to host `out` (capacity out_floats). */
int mmla_debug_od_trace(mmla_ctx* ctx, const float* x, int64_t n, int stage, float* out,
                        int64_t out_floats);
/* Debug (tests, tools): device address and size of internal workspace slot `slot` (0 and 0 when the
 * slot was never allocated), e.g. to check that no kernel of another call writes into it. */
int mmla_debug_ws_slot(mmla_ctx* ctx, int slot, void** ptr, size_t* bytes);
/* Debug (tests): recovery counters of the context so far (each nullable): host-pointer micro-batches
 * re-run in exact f32 by the range guard, and host-pointer micro-batches re-run on the
 * one-workgroup-per-direction BiLSTM because a workgroup of the split BiLSTM (batches <= 128 clips)
 * timed out waiting for the others.  Env MMLA_DEBUG_LSTM_SPIN=<polls> at mmla_create bounds that
 * wait (tests force the timeout path with 1). */
int mmla_debug_counters(mmla_ctx* ctx, int64_t* f32_reruns, int64_t* lstm_split_reruns);
/* ms[MMLA_NSTAGES], launches[MMLA_NSTAGES], work[MMLA_NSTAGES] (each nullable); reset != 0 clears */
int mmla_profile_read(mmla_ctx* ctx, double* ms, int64_t* launches, double* work, int reset);

#ifdef __cplusplus
}
#endif

#endif /* MMLA_H_ */
