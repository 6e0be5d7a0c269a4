// OverlapDetection front-end: int16 PCM -> log-mel (librosa 0.8 semantics) + ZCR + model image.
//
// Replaces:
//   librosa.load + pad/trunc            overlap_features_generator.py:72-80,93-98
//   melspectrogram(n_fft 400, hop 160)  :81   (reflect-padded periodic-Hann STFT, Slaney mel)
//   power_to_db(ref=np.max, top_db=80)  :82
//   normalize_matrix                    :103-117
//   zero_crossing_rate(400, 160)        :100  (edge padding, signbit crossings)
//   generate_zcr_image + imsave + decode_png   :133-151, record_on_pc.py:156-158
//
// One persistent 1024-thread workgroup per CU loops over clips; the 400-point DFT runs as two
// matrix stages on the f16 MFMA in error-compensated 3xFP16 (the v3 kernel below; the earlier
// VALU-FFT kernels and their measurements are in DESIGN.md section 4).
//
// Built with the packed-FP32 target feature off (Makefile NO_PK_F32).  Today that is a no-op guard:
// the kernel below assembles to the same instructions with and without it (it emits no v_pk_*_f32).
// History: the deleted v2 VALU-FFT front-end, which did use half-swapped packed FMAs, returned wrong
// values in one 16-lane quarter of an instruction a few times per thousand waves while MFMA workgroups
// of another stream shared its CUs; built without packed FP32 the same co-run was bit-exact.  The
// hardware-side root cause was never isolated (co-run section); tests/test_gpu_corun.py
// stays the runtime guard.
//
// Accumulation is float32 (the reference runs the FFT in float64 and stores complex64; the measured
// deviation on the normalised log-mel is ~1e-5, tolerance 1e-4).  The scalar steps
// that the reference does in float64 (ref dB, image quantisation) are done in float64 here.
#include "common.h"
#include "od_fe.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <utility>

namespace {

constexpr int N_FFT = 400;
constexpr int HOP = 160;
constexpr int CLIP = 24000;
constexpr int NF = 151;
constexpr int NMEL = 128;
// ================================================================================================
// v3: the 400-point windowed real DFT as two matrix stages on the f16 MFMA, whole clips per
// persistent workgroup, the clip's mel-dB values in registers until its max / min are known (no
// HBM scratch: PCM in, outputs out).
//
//   n = n1 + 16 n2 (n1 < 16, n2 < 25),  k = 25 k1 + k2  =>  X[k] = sum_n1 W400^(n1 k) Y_n1[k2],
//   Y_n1[k2] = sum_n2 w[n] x[160 f - 200 + n] W25^(n2 k2)
//
//   stage 1 (wave = n1, 16 GEMMs per 32-frame tile):  D1[c][f] = sum_n2 A1[n1][c][n2] B1[n2][f]
//       c = 2 k2 + ri (k2 = 0..12; Y_n1[25 - k2] = conj Y_n1[k2] for the real input), the Hann window
//       folded into A1.  B1[n2][f] = x' at padded position 160 f + n1 + 16 n2: the tile's samples sit
//       in LDS transposed, T[n1][q] = x'[16 q + n1] (160 = 16 x 10 and 200 = 16 x 12.5 keep frame
//       starts at n1 = 0 or 8 of one q row ... so n2 runs contiguous: 16-B fragment reads)
//   stage 2 (wave = k2', 13 GEMMs): D2[row][f] = sum_k A2[k2'][row][k] Z[k2'][k][f], k = 2 n1 + ri,
//       rows = (re, im) of bins 25 i + k2' and 25 (i - 8) + 25 - k2' (i < 8; conj Y folded into A2)
//   power |X|^2 -> P[bin][f] (LDS) -> Slaney mel on the f32 MFMA (16-band x 4-bin A fragments)
//
// Arithmetic: error-compensated 3xFP16 with f32 accumulation (x' = x 2^-12 splits int16 exactly into
// fp16 hi + lo; A1 x 2^9, A2 x 2^7 so their lo halves stay normal (Z = 2 Y: |Z| < 51200, lo normal
// for |Y| > 2^-4); Z = stage-1 output split hi/lo before
// stage 2): acc += lo(a) hi(b) + hi(a) lo(b) + hi(a) hi(b).  The numpy model of this dataflow
// (tools/fe_mfma_model.py) is exact to 3.5e-15 in float64 and, in fp16/f32, flips 2.8e-5 of the image
// pixels against the float64 oracle (an fp32 FFT: ~8e-5).
namespace v3 {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t us2 __attribute__((ext_vector_type(2)));

constexpr int NWV = 16;                       // waves per workgroup (one workgroup per CU)
constexpr int NTH = 64 * NWV;
constexpr int TF = 32;                        // frames per tile = the MFMA's 32 columns
constexpr int NTILE = (NF + TF - 1) / TF;     // 5 (frames 151..159 are computed and dropped)
constexpr int TQ = 344;                       // q columns of T: p = 16 q + n1; q < 335 staged per tile,
constexpr int TQS = 335;                      //   q 335..343 (only multiplied by zero A1 columns) zeroed once
constexpr int TP = 346;                       // T row pitch (dwords, even: 8-B reads; rows 8 apart 16 banks apart)
constexpr int NCH = TQS * 16 / 8;             // 670 chunks of 8 samples staged per tile
constexpr int ZP = 36;                        // Z row pitch (halves): 18 dwords -- stage 1's dword stores
                                              // of 32 frame rows 2-way (free; 40 was 4-way, ~6 k LDS
                                              // conflict cycles per clip), stage 2's 8-B reads conflict-free
constexpr int PP = 32;                        // P row pitch (floats): frame f of bin b at column f ^ (16 (b & 1)),
                                              //   so the mel's 2 x 16-lane reads of bins b, b + 1 hit 32 banks
constexpr int PROWS = 212;                    // bins 0..200 + zero rows read by the last mel taps
constexpr int PTRASH = PROWS;                 // + one row that stage 2's unused lanes write
constexpr int G1 = 16 / NWV;                  // stage-1 GEMMs (n1) per wave
constexpr int G2 = (13 + NWV - 1) / NWV;      // stage-2 GEMMs (k2') per wave (the last round partial)
constexpr int MFRAG = 64;                     // mel A fragments (16 bands x 4 bins each)
constexpr int ROT4 = 9;                       // tile 4: chunk c is staged by thread c + ROT4
static_assert(NCH + ROT4 <= NTH, "one staged chunk per thread");
static_assert(G1 == 1, "stage 1: one GEMM per wave (16 waves)");
constexpr float X_SCALE = 1.0f / 4096.0f;     // x' = x 2^-12
constexpr float P_SCALE = 0x1p-38f;           // |X_ref|^2 = |D2|^2 2^-38 (x' 2^-12, A1 2^9, A2 2^7, y = x 2^-15),
                                              //   folded into the mel weights (power-of-two: exact)
static_assert(16 % NWV == 0 && 64 % NWV == 0, "work split over the waves");

struct Smem {
  // the buffers read at lane-dependent addresses plus constant offsets first: their offsets stay
  // below 64 KB, the ds instructions' immediate field (else a VALU add per read)
  float p[2][(PROWS + 1) * PP + 64];          // power [bin][frame] (+ the trash row), by step parity
  float ma[MFRAG * 64];                       // mel A fragments (OdFeTables::mel_a), x P_SCALE
  uint32_t ztrash[128];                       // stage 1's one unused (k2 = 14) word per lane, hi / lo
  uint32_t t[16 * TP];                        // staged samples, transposed: (hi, lo) fp16 pair of x'[16 q + n1]
  _Float16 z_hi[13 * TF * ZP], z_lo[13 * TF * ZP];   // stage-1 output
  uint8_t sgn[NCH + 16];                      // per chunk c at [c + 1]: sign bits of its 8 samples ([0] = 0)
  uint8_t cnt[NCH + 16];                      // per chunk: crossings (low 4 bits), one into its first sample (bit 4)
  int zc[2][NF + 1];                          // ZCR counts of the clip (double-buffered by clip)
  float red[2][NWV];                          // per-wave max / min of the finished clip's mel power
};
static_assert((TF - 1) * 10 + 24 < TQS && (TF - 1) * 10 + 16 + 8 + 8 <= TQ, "stage-1 reads: live / zero columns");
static_assert(20 * (TF - 1) + 50 <= NCH, "ZCR chunks of the tile's last frame are staged");

// (hi, lo) of one value in one dword: hi = f16(x) in bits 0-15, lo = f16(x - hi) in bits 16-31.
// The hi conversions are plain C (so the compiler's hazard tracking sees the first read of an MFMA
// result and pads it); the lo halves are v_fma_mix in inline asm, after their hi (which read the same
// registers), rounding the exact f32 difference once -- clang turns fma(x, 1, -hi) into cvt + sub + cvt
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));
MMLA_DEV uint32_t split1(float x) {   // x: a plain VALU result (staging), no MFMA hazard
  uint32_t u;
  asm("v_cvt_f16_f32 %0, %1\n\t"
      "v_fma_mixhi_f16 %0, %1, 1.0, -%0 op_sel_hi:[0,0,1]"
      : "=&v"(u) : "v"(x));
  return u;
}
// x' = x s with s a power of two in an SGPR (the staging's 2^-12), both halves by v_fma_mix: the
// scaling rides on the conversions (x s exact, rounded once to the hi half; x s - hi exact in f16)
MMLA_DEV uint32_t split1s(float x, float s) {
  uint32_t u;
  asm("v_fma_mixlo_f16 %0, %1, %2, 0\n\t"
      "v_fma_mixhi_f16 %0, %1, %2, -%0 op_sel_hi:[0,0,1]"
      : "=&v"(u) : "v"(x), "s"(s));
  return u;
}
// two values: hi = (f16(a), f16(b)), lo = (f16(a - hi.a), f16(b - hi.b))
MMLA_DEV void split2(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2v){a, b}, h2));
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %3, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(lo) : "v"(a), "v"(hi), "v"(b));
}

// raw buffer descriptor over [p, p + bytes): p must be wave-uniform (its halves are readfirstlane'd
// so the descriptor lives in SGPRs); a null p gives zero records (every access dropped)
MMLA_DEV __amdgpu_buffer_rsrc_t wave_rsrc(const void* p, uint32_t bytes) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)bytes, 0x00020000);
}

MMLA_DEV uint32_t pack_f16(_Float16 a, _Float16 b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}

// bin of output pair i of stage-2 GEMM k2 (-1: unused row pair)
MMLA_DEV int s2_bin(int k2, int i) {
  if (k2 == 0) return i <= 8 ? 25 * i : -1;
  return i < 8 ? 25 * i + k2 : 25 * (i - 8) + 25 - k2;
}

// log2 max(s, 1e-10) (the mel keeps this; the epilogue's fma applies 10 log10 2), the clamp as one
// med3 (fmaxf would add a NaN-quieting max; mel sums are never NaN)
MMLA_DEV float lg2m(float s) { return __log2f(__builtin_amdgcn_fmed3f(s, 1e-10f, __builtin_inff())); }
constexpr float DB_PER_LOG2 = 3.0102999566398120f;

// wave-wide max / min through DPP (quad_perm, row_ror) and four readlanes: no lane-index registers
template <bool MAX>
MMLA_DEV float wave_red(float v) {
  auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : fminf(a, b); };
#define FE3_DPP(ctrl)                                                                        \
  v = op(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v), \
                                                                  __builtin_bit_cast(int, v), \
                                                                  ctrl, 0xf, 0xf, false)))
  FE3_DPP(0xb1);    // quad_perm [1, 0, 3, 2]
  FE3_DPP(0x4e);    // quad_perm [2, 3, 0, 1]
  FE3_DPP(0x124);   // row_ror:4
  FE3_DPP(0x128);   // row_ror:8
#undef FE3_DPP
  const int b = __builtin_bit_cast(int, v);
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48));
  return op(op(r0, r1), op(r2, r3));
}

template <int T>
using tile_c = std::integral_constant<int, T>;
template <class F, int... I>
MMLA_DEV void for_tiles(F&& f, std::integer_sequence<int, I...>) {
  (f(tile_c<I>{}), ...);
}

// Software pipeline over the workgroup's (clip, tile) steps, two barriers per step:
//   interval A:  crossings(t), stage 1(t)  [T -> Z]      |  mel(previous step)  [P -> dB registers]
//   interval B:  stage 2(t)  [Z -> P], ZCR sum(t)        |  staging(next step)  [PCM -> T]
//                + at a clip's end (step (next clip, 0)): its max / min and the norm / dB / image
//                stores straight from the registers
// Every LDS buffer has one writer interval and one reader interval, separated by a barrier (T: B
// writes, A reads; Z: A / B; P: B / A; sgn: B / A; cnt: A / B; zc: double-buffered by clip).  The
// five tiles of a clip are unrolled (tile-dependent edges, offsets and dB register slots become
// compile-time); the loop runs over the workgroup's clips plus one drain pass.
#ifndef FE_TRACE
#define FE_TRACE 0
#endif
#if FE_TRACE
// dev phase timeline (FE_TRACE builds only, tools/fe_timeline.py): s_memtime at 8 points of every
// tile step of the third clip of the first 256 workgroups, per wave
__device__ unsigned long long fe_trace_buf[256 * 16 * 5 * 8];
#define FE_T(i) do { if (trace_on) tt[i] = __builtin_amdgcn_s_memtime(); } while (0)
#define FE_TFLUSH(t) do { if (trace_on && lane == 0) { for (int i_ = 0; i_ < 8; ++i_) fe_trace_buf[(((size_t)blockIdx.x * 16 + wid) * 5 + (t)) * 8 + i_] = tt[i_]; } } while (0)
#else
#define FE_T(i) do { } while (0)
#define FE_TFLUSH(t) do { } while (0)
#endif
template <bool DB, bool NM, bool IMG>
__global__ void __launch_bounds__(NTH, 1) od_fe3_kernel(OdFeArgs a, int64_t n_clips) {
  __shared__ __attribute__((aligned(16))) Smem sm;
  const OdFeTables& tb = *a.tables;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

  // this wave's A fragments for the whole launch: stage 1 n1 = G1 wid + g, stage 2 k2' = wid + NWV j
  f16x8 a1h[G1][2], a1l[G1][2], a2h[G2][2], a2l[G2][2];
#pragma unroll
  for (int g = 0; g < G1; ++g)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      a1h[g][s] = *reinterpret_cast<const f16x8*>(tb.a1[G1 * wid + g][s][0][lane]);
      a1l[g][s] = *reinterpret_cast<const f16x8*>(tb.a1[G1 * wid + g][s][1][lane]);
    }
#pragma unroll
  for (int j = 0; j < G2; ++j) {
    const int k2 = min(wid + NWV * j, 12);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      a2h[j][s] = *reinterpret_cast<const f16x8*>(tb.a2[k2][s][0][lane]);
      a2l[j][s] = *reinterpret_cast<const f16x8*>(tb.a2[k2][s][1][lane]);
    }
  }
  for (int i = tid; i < MFRAG * 64; i += NTH) sm.ma[i] = (&tb.mel_a[0][0])[i];
  for (int i = tid; i < 2 * (PROWS - 201) * PP; i += NTH) sm.p[i & 1][201 * PP + (i >> 1)] = 0.0f;
  for (int i = tid; i < 16 * (TP - TQS); i += NTH) sm.t[(i / (TP - TQS)) * TP + TQS + i % (TP - TQS)] = 0u;
  if (tid == 0) sm.sgn[0] = 0;

  // an opaque copy of the thread id per use: the tile-unrolled code otherwise hoists every
  // thread-derived address of all tiles out of the clip loop (hundreds of live registers -> spills)
  auto otid = [&]() {
    int v = tid;
    asm volatile("" : "+v"(v));
    return v;
  };
  // the staging thread order: chunk c is staged by thread c (starting at other waves, e.g. 13-15
  // first, measured 0.2936 vs 0.2899 ms with the mel in interval B)
  auto stid = [&]() { return otid(); };
  static_assert(NWV == 16, "staging order assumes 16 waves");

  // clip facts the staging needs, wave-uniform
  struct ClipIn {
    const int16_t* src;
    int len;
    bool fast;    // int16 PCM at a 16-B aligned start: 16-B chunk loads
  };
  auto clip_in = [&](int64_t clip) -> ClipIn {
    ClipIn ci;
    int len = a.lens ? a.lens[clip] : a.clip_len;
    // wave-uniform in an SGPR: the prefetch's buffer descriptor (num_records = 2 len) then needs no
    // waterfall loop over lanes
    len = __builtin_amdgcn_readfirstlane(len);
    ci.len = len < 0 ? 0 : (len > CLIP ? CLIP : len);
    ci.src = a.pcm + clip * a.clip_stride;
    ci.fast = !a.pcm_f32 && (reinterpret_cast<uintptr_t>(ci.src) & 15) == 0;
    return ci;
  };

  // the next staging's 8 samples of this thread's chunk, one step ahead: the 16-B load of the chunk
  // when it lies inside the clip's readable samples, else zeros (reflect-padded and partial chunks
  // are completed at staging time).  Tile 4 maps chunk c to thread c + 9 so that the reflected
  // chunks at its end and the chunks they mirror are lanes of one wave (tile 0: chunk c = thread c).
  uint32_t nx[4] = {0, 0, 0, 0};
  auto prefetch = [&](int64_t clip_, auto T_) {
    constexpr int t = decltype(T_)::value;
    nx[0] = nx[1] = nx[2] = nx[3] = 0u;
    if (clip_ >= n_clips) return;
    const ClipIn ci = clip_in(clip_);
    if (!ci.fast) return;
    // a buffer load over the clip's readable samples: chunks before sample 0 (negative offsets wrap
    // past the range) and past len read zeros with no per-lane bounds arithmetic; threads without a
    // chunk (c >= NCH) load harmlessly and never store
    const auto rs = wave_rsrc(ci.src, (uint32_t)ci.len * 2u);
    const int c = stid() - (t == NTILE - 1 ? ROT4 : 0);
    const uint32_t off = (uint32_t)(2 * (HOP * TF * t - N_FFT / 2 + 8 * c));
    typedef uint32_t u4v __attribute__((ext_vector_type(4)));
    const u4v v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    nx[0] = v.x;
    nx[1] = v.y;
    nx[2] = v.z;
    nx[3] = v.w;
  };

  // float PCM: y 2^3 is split into fp16 hi + lo, so |y| must stay below 65504 / 8 (a larger or
  // non-finite sample sets a.range_flag: the host call reports MMLA_E_RANGE)
  constexpr float F32_PCM_RANGE = 8188.0f;
  bool fbad = false;
  // ---- staging of (clip, t): chunk c holds p = 8c .. 8c + 7 (reflect-padded, zero past len), split
  //      x' = x 2^-12 into fp16 hi + lo, transposed store T[p & 15][p >> 4] = (hi, lo) ---------------
  auto stage = [&](int64_t clip, auto T_) {
    constexpr int t = decltype(T_)::value;
    const ClipIn ci = clip_in(clip);
    const int c = stid() - (t == NTILE - 1 ? ROT4 : 0);
    const int i0 = HOP * TF * t - N_FFT / 2 + 8 * c;
    const bool live = c >= 0 && c < NCH;
    uint32_t d[8];               // (hi, lo) of x' = x 2^-12 (int16 PCM) or y 2^3 (float PCM, y = x / 32768)
    uint32_t sg = 0;             // sign bits (librosa zero_crossings: |y| <= 1e-10 counts as 0)
    if (!ci.fast) {
      // float PCM or a clip start off 16-B alignment: per-sample loads (not the hot path)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        int i = i0 + j;
        i = i < 0 ? -i : i;
        i = i >= CLIP ? 2 * (CLIP - 1) - i : i;
        const bool in = live && i >= 0 && i < ci.len;
        if (a.pcm_f32) {
          const float y = in ? a.pcm_f32[clip * a.clip_stride + i] : 0.0f;
          fbad |= !(fabsf(y) < F32_PCM_RANGE);
          d[j] = split1(y * (32768.0f * X_SCALE));
          sg |= (uint32_t)(y < -1e-10f) << j;
        } else {
          const int16_t v = in ? ci.src[i] : (int16_t)0;
          d[j] = split1((float)v * X_SCALE);
          sg |= (uint32_t)(v < 0) << j;
        }
      }
    } else {
      uint32_t w[4] = {nx[0], nx[1], nx[2], nx[3]};
      if (ci.len < CLIP && live && i0 >= 0 && i0 < ci.len && i0 + 8 > ci.len) {
        // the clip's last, partial chunk: its samples one by one (short clips only)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t lo16 = i0 + 2 * k < ci.len ? (uint16_t)ci.src[i0 + 2 * k] : 0u;
          const uint32_t hi16 = i0 + 2 * k + 1 < ci.len ? (uint16_t)ci.src[i0 + 2 * k + 1] : 0u;
          w[k] = lo16 | (hi16 << 16);
        }
      }
      // reflect padding (center=True, pad_mode='reflect') of the zero-padded 24000 samples: the
      // chunks before sample 0 (tile 0, chunks 0..24) and past sample 23999 (tile 4, chunks
      // 465..489) take their samples from the chunks they mirror, lanes of the same wave:
      //   tile 0: p' = 400 - p  -> chunk 49 - c elements 8 - j (j >= 1), chunk 50 - c element 0
      //   tile 4: p' = 7438 - p -> chunk 929 - c elements 6 - j (j <= 6), chunk 928 - c element 7
      // (staging wave = first ? 0 : (465 + ROT4) / 64)
      if constexpr (t == 0 || t == NTILE - 1) {
        constexpr bool first = t == 0;
        if (wid == (first ? 0 : (465 + ROT4) / 64)) {
          const int pa = first ? 49 - c : 929 - c, pb = first ? 50 - c : 928 - c;
          const int la = (pa + (first ? 0 : ROT4)) & 63, lb = (pb + (first ? 0 : ROT4)) & 63;
          uint32_t ma[4], mb;
#pragma unroll
          for (int k = 0; k < 4; ++k) ma[k] = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * la, (int)w[k]);
          mb = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * lb, (int)w[first ? 0 : 3]);
          const bool refl = first ? (c < 25) : (c >= 465 && c < 490);
          if (refl) {
            auto el = [&](int e) -> uint32_t { return (ma[e >> 1] >> (16 * (e & 1))) & 0xffffu; };
            uint32_t v[8];
            if (first) {
              v[0] = mb & 0xffffu;
#pragma unroll
              for (int jj = 1; jj < 8; ++jj) v[jj] = el(8 - jj);
            } else {
#pragma unroll
              for (int jj = 0; jj < 7; ++jj) v[jj] = el(6 - jj);
              v[7] = mb >> 16;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) w[k] = v[2 * k] | (v[2 * k + 1] << 16);
          }
        }
      }
      if constexpr (t == NTILE - 1) {
        if (!live || i0 >= CLIP + N_FFT / 2) w[0] = w[1] = w[2] = w[3] = 0u;   // past the padded signal
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        d[2 * k] = split1s((float)(int16_t)(w[k] & 0xffffu), X_SCALE);
        d[2 * k + 1] = split1s((float)(int16_t)(w[k] >> 16), X_SCALE);
      }
      // sign bits: v_perm's selectors 8..11 give 0xff / 0x00 from the sign of bytes 1, 3, 5, 7 (the
      // samples' high bytes); a signed dot4 with weights -1, -2, -4, ... packs them (4 full-rate ops)
      const int s01 = (int)__builtin_amdgcn_perm(w[1], w[0], 0x0b0a0908u);
      const int s23 = (int)__builtin_amdgcn_perm(w[3], w[2], 0x0b0a0908u);
      sg = (uint32_t)__builtin_amdgcn_sdot4(s23, (int)0x80c0e0f0u,
                                            __builtin_amdgcn_sdot4(s01, (int)0xf8fcfeffu, 0, false), false);
    }
    if (live) {
      uint32_t* tq = sm.t + (c & 1) * 8 * TP + (c >> 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) tq[j * TP] = d[j];
      sm.sgn[c + 1] = (uint8_t)sg;
    }
  };

  // ---- crossings per chunk of tile t: transitions into its 8 samples, counted for samples
  //      1 <= i <= CLIP - 1 (edge padding repeats the clip's first / last sample: no crossing) ------
  auto crossings = [&](auto T_) {
    constexpr int t = decltype(T_)::value;
    const int ibase = HOP * TF * t - N_FFT / 2;
    static_assert(NCH <= NTH, "one chunk per thread");
    const int c = otid();
    if (c < NCH) {
      const uint32_t m = sm.sgn[c + 1];
      const uint32_t pv = (uint32_t)sm.sgn[c] >> 7;
      uint32_t tr = (m ^ ((m << 1) | pv)) & 0xffu;
      if constexpr (t == 0 || t == NTILE - 1) {
        const int i0 = ibase + 8 * c;
        if (i0 < 1 || i0 + 7 > CLIP - 1) {
          uint32_t vm = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) vm |= (uint32_t)(i0 + j >= 1 && i0 + j <= CLIP - 1) << j;
          tr &= vm;
        }
      }
      sm.cnt[c] = (uint8_t)(__builtin_popcount(tr) | ((tr & 1u) << 4));
    }
  };

  // ---- stage 1 (wave = n1 G1 wid .. + G1 - 1): D1 = A1[n1] (32 x 32) . B1 (32 n2 x 32 frames) ------
  auto stage1 = [&](int r, int hh) {
    f32x16 acc[G1];
#pragma unroll
    for (int g = 0; g < G1; ++g) {
      const int n1 = G1 * wid + g;
      // lane (frame r, half hh): q = 10 r + 16 s + 8 hh + j, j < 8 (two 8-B reads per 4 pairs)
      const uint2* tp = reinterpret_cast<const uint2*>(sm.t + n1 * TP + 10 * r + 8 * hh);
      acc[g] = f32x16{};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        uint32_t w[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint2 dd = tp[8 * s + i];
          w[2 * i] = dd.x;
          w[2 * i + 1] = dd.y;
        }
        uint32_t bh[4], bl[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {   // de-interleave (hi, lo) pairs: bytes 0-1 / 2-3 of each word
          bh[i] = __builtin_amdgcn_perm(w[2 * i + 1], w[2 * i], 0x05040100u);
          bl[i] = __builtin_amdgcn_perm(w[2 * i + 1], w[2 * i], 0x07060302u);
        }
        const f16x8 BH = __builtin_bit_cast(f16x8, bh), BL = __builtin_bit_cast(f16x8, bl);
        acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1l[g][s], BH, acc[g], 0, 0, 0);
        acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h[g][s], BL, acc[g], 0, 0, 0);
        acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h[g][s], BH, acc[g], 0, 0, 0);
      }
    }
    // registers 2 pi, 2 pi + 1 = (re, im) of Y_n1[k2], k2 = (pi & 1) + 4 (pi >> 1) + 2 hh, for
    // frame r: split hi / lo into Z[k2][r][2 n1 ..] (the wave's G1 n1 are 2 G1 consecutive k)
    uint32_t* zh = reinterpret_cast<uint32_t*>(sm.z_hi) + r * (ZP / 2) + G1 * wid;
    uint32_t* zl = reinterpret_cast<uint32_t*>(sm.z_lo) + r * (ZP / 2) + G1 * wid;
    // k2 < 13 except (pi 7: both halves) and (pi 6, hh 1: k2 14) -- that one goes to a trash word
#pragma unroll
    for (int pi = 0; pi < 7; ++pi) {
      const int k2 = (pi & 1) + 4 * (pi >> 1) + 2 * hh;
      uint32_t vh[G1], vl[G1];
#pragma unroll
      for (int g = 0; g < G1; ++g) split2(acc[g][2 * pi], acc[g][2 * pi + 1], vh[g], vl[g]);
      if (pi == 6) {
        uint32_t* th = hh ? &sm.ztrash[lane] : zh + 12 * TF * (ZP / 2);
        uint32_t* tl = hh ? &sm.ztrash[64 + lane] : zl + 12 * TF * (ZP / 2);
        *th = vh[0];
        *tl = vl[0];
      } else if constexpr (G1 == 2) {
        *reinterpret_cast<uint2*>(zh + k2 * TF * (ZP / 2)) = uint2{vh[0], vh[1]};
        *reinterpret_cast<uint2*>(zl + k2 * TF * (ZP / 2)) = uint2{vl[0], vl[1]};
      } else {
        zh[k2 * TF * (ZP / 2)] = vh[0];
        zl[k2 * TF * (ZP / 2)] = vl[0];
      }
    }
  };

  // ---- stage 2 (wave = k2' wid + NWV j): D2 = A2[k2'] (32 x 32) . Z[k2'] (32 k x 32 frames)
  //      -> |X|^2 (x 2^38: P_SCALE sits in the mel weights) -> P[bin][frame] ------------------------
  auto stage2 = [&](int r, int hh, float* P) {
#pragma unroll
    for (int j = 0; j < G2; ++j) {
      const int k2 = wid + NWV * j;
      if (k2 >= 13) continue;
      const uint2* zh = reinterpret_cast<const uint2*>(sm.z_hi + (k2 * TF + r) * ZP + 8 * hh);
      const uint2* zl = reinterpret_cast<const uint2*>(sm.z_lo + (k2 * TF + r) * ZP + 8 * hh);
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        // the fragment's 16 B as two 8-B reads (rows are 8-B, not 16-B, aligned)
        const uint2 h0 = zh[4 * s], h1 = zh[4 * s + 1], l0 = zl[4 * s], l1 = zl[4 * s + 1];
        const f16x8 BH = __builtin_bit_cast(f16x8, uint4{h0.x, h0.y, h1.x, h1.y});
        const f16x8 BL = __builtin_bit_cast(f16x8, uint4{l0.x, l0.y, l1.x, l1.y});
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2l[j][s], BH, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2h[j][s], BL, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2h[j][s], BH, acc, 0, 0, 0);
      }
      // pair i = c0 + 2 hh (c0 = (pi & 1) + 4 (pi >> 1)): bin 25 i + k2 (i < 8: c0 < 8), else
      // 25 (i - 8) + 25 - k2; GEMM 0 has bins 25 i for i <= 8 only (the other lanes write the
      // trash row).  Branch-free: the row offset is an immediate plus the wave-uniform k2
      // frame r of an even bin at column r, of an odd bin at r ^ 16 (PP above); a bin's parity is
      // that of c0 + k2 (rows 25 c0 + 50 hh + k2) or c0 + 1 + k2 (rows 25 (c0 - 8) + 50 hh + 25 - k2)
      float* const prow0 = P + 50 * PP * hh + r;
      float* const prow1 = P + 50 * PP * hh + (r ^ 16);
      // one scalar branch per GEMM (not per pair): the k2 = 0 GEMM's row pattern apart, so the other
      // twelve waves store each power with one immediate-offset write from two base registers
      if (k2 == 0) {
        float* trash = P + PTRASH * PP + lane;
#pragma unroll
        for (int pi = 0; pi < 8; ++pi) {
          const int c0 = (pi & 1) + 4 * (pi >> 1);
          if (c0 > 8) continue;
          const float pw = fmaf(acc[2 * pi], acc[2 * pi], acc[2 * pi + 1] * acc[2 * pi + 1]);
          *(c0 + 2 * hh <= 8 ? (c0 & 1 ? prow1 : prow0) + 25 * c0 * PP : trash) = pw;
        }
      } else {
        float* const qa = (k2 & 1) ? prow1 : prow0;  // rows of parity (c0 + k2) & 1 for even c0
        float* const qb = (k2 & 1) ? prow0 : prow1;
        float* const pa0 = qa + k2 * PP, * const pa1 = qb + k2 * PP;                // bins 25 c0 + k2 (c0 < 8)
        float* const pb0 = qb + (25 - k2) * PP, * const pb1 = qa + (25 - k2) * PP;  // bins 25 (c0 - 8) + 25 - k2
#pragma unroll
        for (int pi = 0; pi < 8; ++pi) {
          const int c0 = (pi & 1) + 4 * (pi >> 1);
          const float pw = fmaf(acc[2 * pi], acc[2 * pi], acc[2 * pi + 1] * acc[2 * pi + 1]);
          if (c0 < 8) (c0 & 1 ? pa1 : pa0)[25 * c0 * PP] = pw;
          else (c0 & 1 ? pb1 : pb0)[25 * (c0 - 8) * PP] = pw;
        }
      }
    }
  };

  // ---- ZCR of tile t (last wave): frame f0 + lane = the transitions into tile positions
  //      160 lane + 1 .. + 399 = chunks 20 lane .. 20 lane + 49 minus the one into chunk 20 lane's
  //      first sample ---------------------------------------------------------------------------------
  auto zsum = [&](auto T_, int par) {
    constexpr int t = decltype(T_)::value;
    if (wid == NWV - 1 && lane < TF) {
      const uint32_t* cw = reinterpret_cast<const uint32_t*>(sm.cnt) + 5 * lane;
      int s = 0;
#pragma unroll
      for (int k = 0; k < 13; ++k) {
        const uint32_t w = cw[k] & (k == 12 ? 0x0f0fu : 0x0f0f0f0fu);
        s = (int)__builtin_amdgcn_udot4(w, 0x01010101u, (uint32_t)s, false);   // the 4 byte counts
      }
      s -= (int)((cw[0] >> 4) & 1u);
      if (TF * t + lane < NF) sm.zc[par][TF * t + lane] = s;
    }
  };

  // this wave's mel unit: band tile bt (bands 16 bt ..), frame half fh of the 32-frame tile
  const int m_unit = __builtin_amdgcn_readfirstlane(tb.mel_unit[wid]);
  const int m_bt = m_unit >> 1, m_fh = m_unit & 1;
  const int m_bin0 = __builtin_amdgcn_readfirstlane(tb.mel_bt_bin0[m_bt]);
  const int m_nk = __builtin_amdgcn_readfirstlane(tb.mel_bt_nk[m_bt]);
  const int m_frag = __builtin_amdgcn_readfirstlane(tb.mel_bt_frag[m_bt]);
  // log2 S at band 16 bt + 4 (l >> 4) + i, frame 32 t + 16 fh + (l & 15)
  float dbv[NTILE][4];
  float smax = 0.0f, smin = INFINITY;
  typedef float f32x4 __attribute__((ext_vector_type(4)));

  // ---- mel of tile t on the f32 MFMA: S[16 bands][16 frames] = A (16 x 4 k-steps) . P (bins x frames),
  //      exact float32 products and sums (the reference's np.dot is float32); K-steps in batches of 4
  //      whose 8 LDS reads are issued before their MFMAs; A columns past a band's support are zero ----
  auto mel = [&](auto T_, const float* P) {
    constexpr int t = decltype(T_)::value;
    int l = lane;
    asm volatile("" : "+v"(l));
    const int mb = m_bin0 + (l >> 4);   // + 4 k per K-step: the same parity
    const float* pb = P + mb * PP + ((16 * m_fh + (l & 15)) ^ (16 * (mb & 1)));
    const float* ab = sm.ma + m_frag * 64 + l;
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    int nk = m_nk;
    asm volatile("" : "+s"(nk));
    constexpr int NK_MAX = 20;
#pragma unroll
    for (int j0 = 0; j0 < NK_MAX; j0 += 4) {
      if (j0 >= nk) break;
      float av[4], bv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        av[j] = ab[64 * (j0 + j)];
        bv[j] = pb[4 * PP * (j0 + j)];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bv[j], acc, 0, 0, 0);
      }
    }
    const bool live = TF * t + TF <= NF || TF * t + 16 * m_fh + (l & 15) < NF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      dbv[t][i] = lg2m(acc[i]);
      if (live) {
        smax = fmaxf(smax, acc[i]);
        smin = fminf(smin, acc[i]);
      }
    }
  };

  // ---- a clip's end: max / min of its mel power over the waves, power_to_db(ref=np.max, amin=1e-10,
  //      top_db=80) with numpy-1.21 dtypes, normalize_matrix (max / min of the dB matrix are the dB
  //      of max / min S), stores straight from the registers -----------------------------------
  auto epilogue = [&](int64_t clip, int par) {
#pragma clang fp contract(off)
    float mx = sm.red[0][0], mn = sm.red[1][0];
#pragma unroll
    for (int w = 1; w < NWV; ++w) {
      mx = fmaxf(mx, sm.red[0][w]);
      mn = fminf(mn, sm.red[1][w]);
    }
    // ref = np.max: numpy takes 10 log10 of the float32 max in float64 and subtracts it in float32.
    // Here every dB value is fma(log2 S, 10 log10 2, -ref) with ref = the rounded dB of the max, the
    // max and min taken through the same expression: d_max is within an ulp of 0 (the shift cancels
    // in the normalisation; the dB outputs move by ~1e-5 dB, tolerance 5e-3), the clip's min maps to
    // exactly 0, a constant spectrum (digital silence) to 0 / 0 = NaN as the reference
    const float lmx = lg2m(mx);
    const float nref = -(lmx * DB_PER_LOG2);
    const float d_max = fmaf(lmx, DB_PER_LOG2, nref);
    const float thr = d_max - 80.0f;
    const float d_min = fmaxf(fmaf(lg2m(mn), DB_PER_LOG2, nref), thr);
    const float diff = d_max - d_min;
    const float inv_diff = 1.0f / diff;
    const int tz = otid();
    if (a.zcr && tz < NF) a.zcr[clip * NF + tz] = (float)sm.zc[par][tz] * (1.0f / 400.0f);
    // norm / dB rows: lane l writes frame 32 t + 16 fh + (l & 15) of bands 16 bt + 4 (l >> 4) + i --
    // 64 B of one band row per 16 lanes.  Image (rows h = 127 - band, RGB bytes): R = trunc(255 zcr[w]),
    // G = B = trunc(255 (1 - norm)) in float64, NaN -> 0; three byte stores per pixel.
    // Buffer stores over the clip's output block: the lane's offset is one VGPR, the unit's band tile /
    // frame half an SGPR and (i, t) the immediate -- no per-store address arithmetic
    constexpr uint32_t FB = NMEL * NF * 4, IB = NMEL * NF * 3;
    const auto rn = wave_rsrc(NM ? a.norm + clip * (NMEL * NF) : nullptr, NM ? FB : 0);
    const auto rd = wave_rsrc(DB ? a.db + clip * (NMEL * NF) : nullptr, DB ? FB : 0);
    const auto ri = wave_rsrc(IMG ? a.img + clip * (NMEL * NF * 3) : nullptr, IMG ? IB : 0);
    int l = lane;
    asm volatile("" : "+v"(l));
    const int fr = 16 * m_fh + (l & 15);                          // frame within the 32-frame tile
    const uint32_t vf = (uint32_t)(4 * (l >> 4) * NF + (l & 15)) * 4u;
    const int sf = (16 * m_bt * NF + 16 * m_fh) * 4;
    // image row 127 - (16 bt + 4 (l >> 4) + i) = (112 - 16 bt) + (12 - 4 (l >> 4)) + (3 - i)
    const uint32_t vi = (uint32_t)((12 - 4 * (l >> 4)) * NF + (l & 15)) * 3u;
    const int si = ((112 - 16 * m_bt) * NF + 16 * m_fh) * 3;
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      if (TF * t + TF > NF && TF * t + fr >= NF) continue;
      uint32_t rr = 0;
      if (IMG) rr = (uint32_t)(int)(((double)sm.zc[par][TF * t + fr] / 400.0) * 255.0) & 255u;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = fmaxf(fmaf(dbv[t][i], DB_PER_LOG2, nref), thr);
        // (d - min) / (max - min) as a multiply by the reciprocal (<= 2 ulp); 0 * inf =
        // NaN keeps the digital-silence NaN.  The (i, t) part of the offset is wave-uniform: it
        // rides in soffset (a scalar add), the lane's part is the one VGPR vf
        const float nv = (d - d_min) * inv_diff;
        const int so = sf + (i * NF + TF * t) * 4;
        if (NM) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, nv), rn, vf, so, 0);
        if (DB) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, d), rd, vf, so, 0);
        if (IMG) {
          const double v = (1.0 - (double)nv) * 255.0;
          const uint32_t gb = (v >= 0.0) ? ((uint32_t)(int)v & 255u) : 0u;
          const int soi = si + ((3 - i) * NF + TF * t) * 3;
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)rr, ri, vi, soi, 0);
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)gb, ri, vi + 1, soi, 0);
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)gb, ri, vi + 2, soi, 0);
        }
      }
    }
  };

  const int64_t my_clips = (int64_t)blockIdx.x < n_clips ? (n_clips - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  if (my_clips > 0) {
    prefetch(blockIdx.x, tile_c<0>{});
    stage(blockIdx.x, tile_c<0>{});
    prefetch(blockIdx.x, tile_c<1>{});
  }
  __syncthreads();

#pragma unroll 1
  for (int64_t ci = 0; ci <= my_clips; ++ci) {
    const int64_t clip = blockIdx.x + ci * gridDim.x;
    const bool cur = ci < my_clips;
    const int par = (int)(ci & 1);
    for_tiles([&](auto T_) {
      constexpr int t = decltype(T_)::value;
      // the drain pass after the last clip: step 0's interval B (mel of the last tile, max / min) and
      // step 1's interval A (the last clip's epilogue)
      if (!cur && t > 1) return;
      // lane-derived offsets are recomputed per tile from an opaque copy of the lane id: hoisted,
      // the per-band store / LDS addresses of all five tiles stay live together and spill
      int lane_o = lane;
      asm volatile("" : "+v"(lane_o));
      const int r = lane_o & 31, hh = lane_o >> 5;
      // P by step parity: stage 2 of step s writes P[s & 1] while the mel of step s - 1 reads the other
      const int pw = (int)((ci * NTILE + t) & 1);
      float* const p_w = sm.p[pw];
      const float* const p_r = sm.p[pw ^ 1];
      // the mel of the previous step reads P[(s - 1) & 1], stable through intervals A and B of step s
      // (it runs in B on every wave: the youngest waves of each SIMD in A measured 0.2964 vs 0.2941 ms)
      auto mel_prev = [&]() {
        if constexpr (t > 0) {
          mel(tile_c<t - 1>{}, p_r);
        } else if (ci > 0) {
          mel(tile_c<NTILE - 1>{}, p_r);
        }
      };
#if FE_TRACE
      const bool trace_on = ci == 2 && blockIdx.x < 256;
      unsigned long long tt[8];
#endif
      FE_T(0);
      // ---- interval A ----
      if (cur) {
        crossings(T_);
        stage1(r, hh);
      }
      FE_T(1);
      if (t == 1 && ci > 0) {   // the previous clip: its last mel and max / min finished in step 0
        epilogue(clip - gridDim.x, par ^ 1);
      }
      FE_T(2);
      __syncthreads();
      FE_T(3);
      if (!cur && t == 1) return;
      // ---- interval B ----  (the mel of tile t - 1 first: its MFMAs then start on every wave at the
      // barrier instead of queueing behind stage 2's on waves 0-12 -- 0.2975 -> 0.2903 ms, A/B)
      mel_prev();   // (after the epilogue: tile 0's mel overwrites the dB registers it read)
      FE_T(4);
      if (t == 0 && ci > 0) {
        const float mx = wave_red<true>(smax), mn = wave_red<false>(smin);
        if (lane == 0) {
          sm.red[0][wid] = mx;
          sm.red[1][wid] = mn;
        }
        smax = 0.0f;
        smin = INFINITY;
      }
      if (cur) stage2(r, hh, p_w);
      FE_T(5);
      if (cur) {
        zsum(T_, par);
        if constexpr (t + 1 < NTILE) {
          stage(clip, tile_c<t + 1>{});
        } else if (ci + 1 < my_clips) {
          stage(clip + gridDim.x, tile_c<0>{});
        }
        if constexpr (t + 2 < NTILE) {
          prefetch(clip, tile_c<t + 2>{});
        } else {
          prefetch(ci + 1 < my_clips ? clip + gridDim.x : n_clips, tile_c<t + 2 - NTILE>{});
        }
      }
      FE_T(6);
      __syncthreads();
      FE_T(7);
      FE_TFLUSH(t);
    }, std::make_integer_sequence<int, NTILE>{});
  }
  if (fbad && a.range_flag) *a.range_flag = 1;
}

}  // namespace v3

}  // namespace

#if FE_TRACE
extern "C" int mmla_debug_fe_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(v3::fe_trace_buf), sizeof(v3::fe_trace_buf)) == hipSuccess ? 0 : -2;
}
#endif

bool od_fe_tables_ok(const OdFeTables& t) {
  for (int m = 0; m < 128; ++m) {
    if (t.mel_cnt[m] > 10) return false;   // the weights kept per band (mel_w)
    const int bt = m / 16;   // the band's support lies inside its tile's bins, read rows stay in P
    if (t.mel_cnt[m] > 0 && (t.mel_start[m] < t.mel_bt_bin0[bt] ||
                             t.mel_start[m] + t.mel_cnt[m] > t.mel_bt_bin0[bt] + 4 * t.mel_bt_nk[bt]))
      return false;
  }
  int frags = 0;
  for (int bt = 0; bt < 8; ++bt) {
    if (t.mel_bt_nk[bt] % 4 || t.mel_bt_nk[bt] > 20 || t.mel_bt_bin0[bt] < 0 ||
        t.mel_bt_bin0[bt] + 4 * t.mel_bt_nk[bt] > v3::PROWS || t.mel_bt_frag[bt] != frags)
      return false;
    frags += t.mel_bt_nk[bt];
  }
  if (frags > v3::MFRAG) return false;
  return true;
}

static void launch_v3(const OdFeArgs& a, int64_t n, hipStream_t s) {
  // persistent: one 1024-thread workgroup per CU (LDS ~119 KB), each looping over clips
  static int n_cu = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  const dim3 g((unsigned)std::min<int64_t>(n, n_cu)), b(v3::NTH);
  const int k = (a.db ? 4 : 0) | (a.norm ? 2 : 0) | (a.img ? 1 : 0);
  switch (k) {
    case 0: hipLaunchKernelGGL((v3::od_fe3_kernel<false, false, false>), g, b, 0, s, a, n); break;
    case 1: hipLaunchKernelGGL((v3::od_fe3_kernel<false, false, true>), g, b, 0, s, a, n); break;
    case 2: hipLaunchKernelGGL((v3::od_fe3_kernel<false, true, false>), g, b, 0, s, a, n); break;
    case 3: hipLaunchKernelGGL((v3::od_fe3_kernel<false, true, true>), g, b, 0, s, a, n); break;
    case 4: hipLaunchKernelGGL((v3::od_fe3_kernel<true, false, false>), g, b, 0, s, a, n); break;
    case 5: hipLaunchKernelGGL((v3::od_fe3_kernel<true, false, true>), g, b, 0, s, a, n); break;
    case 6: hipLaunchKernelGGL((v3::od_fe3_kernel<true, true, false>), g, b, 0, s, a, n); break;
    default: hipLaunchKernelGGL((v3::od_fe3_kernel<true, true, true>), g, b, 0, s, a, n); break;
  }
}

hipError_t od_fe_launch(const OdFeArgs& a, int64_t n_clips, hipStream_t stream) {
  if (n_clips <= 0) return hipSuccess;
  launch_v3(a, n_clips, stream);
  return hipGetLastError();
}

void od_fe_build_tables(OdFeTables* t) {
  const double PI = 3.14159265358979323846;
  // librosa.filters.mel(16000, 400, n_mels=128, fmin=0, fmax=8000, htk=False, norm='slaney'):
  // float64 triangles stored float32, then float32 * float64 enorm -> float32.
  auto hz_to_mel = [](double f) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = 1000.0 / f_sp;
    const double logstep = log(6.4) / 27.0;
    return f >= min_log_hz ? min_log_mel + log(f / min_log_hz) / logstep : f / f_sp;
  };
  auto mel_to_hz = [](double m) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = 1000.0 / f_sp;
    const double logstep = log(6.4) / 27.0;
    return m >= min_log_mel ? min_log_hz * exp(logstep * (m - min_log_mel)) : f_sp * m;
  };
  double mel_f[NMEL + 2];
  const double mmin = hz_to_mel(0.0), mmax = hz_to_mel(8000.0);
  for (int i = 0; i < NMEL + 2; ++i) {
    // np.linspace(min, max, n): start + i * step, last element exactly max
    const double step = (mmax - mmin) / (NMEL + 1);
    const double m = (i == NMEL + 1) ? mmax : mmin + i * step;
    mel_f[i] = mel_to_hz(m);
  }
  t->zero16 = 0;
  for (int m = 0; m < NMEL; ++m) {
    int st = -1, cnt = 0;
    float w[16] = {0};
    const double enorm = 2.0 / (mel_f[m + 2] - mel_f[m]);
    const double fd0 = mel_f[m + 1] - mel_f[m], fd1 = mel_f[m + 2] - mel_f[m + 1];
    for (int k = 0; k <= N_FFT / 2; ++k) {
      const double fk = 8000.0 * k / (N_FFT / 2);     // np.linspace(0, 8000, 201)
      const double lower = -(mel_f[m] - fk) / fd0;
      const double upper = (mel_f[m + 2] - fk) / fd1;
      double v = fmin(lower, upper);
      v = v > 0.0 ? v : 0.0;
      const float v32 = (float)v;
      const float wv = (float)((double)v32 * enorm);
      if (wv != 0.0f) {
        if (st < 0) st = k;
        if (k - st < 16) w[k - st] = wv;
        cnt = k - st + 1;
      }
    }
    t->mel_start[m] = st < 0 ? 0 : st;
    t->mel_cnt[m] = cnt;
    for (int j = 0; j < 10; ++j) t->mel_w[m][j] = j < cnt ? w[j] : 0.0f;
  }

  // v3 mel schedule: band tile bt = bands 16 bt .. 16 bt + 15 reads the bins of their union, in
  // k-steps of 4 bins, padded to batches of 4 k-steps and kept inside the P rows (start moved down)
  std::memset(t->mel_a, 0, sizeof(t->mel_a));
  int frag = 0;
  for (int bt = 0; bt < 8; ++bt) {
    int lo = 1 << 30, hi = -1;
    for (int m = 16 * bt; m < 16 * bt + 16; ++m)
      if (t->mel_cnt[m] > 0) {
        lo = std::min(lo, t->mel_start[m]);
        hi = std::max(hi, t->mel_start[m] + t->mel_cnt[m] - 1);
      }
    if (hi < 0) lo = hi = 0;
    const int nk = ((hi - lo + 1 + 3) / 4 + 3) / 4 * 4;
    const int b0 = std::max(0, std::min(lo, v3::PROWS - 4 * nk));
    t->mel_bt_bin0[bt] = b0;
    t->mel_bt_nk[bt] = nk;
    t->mel_bt_frag[bt] = frag;
    for (int j = 0; j < nk && frag + j < v3::MFRAG; ++j)
      for (int l = 0; l < 64; ++l) {
        const int m = 16 * bt + (l & 15), bin = b0 + 4 * j + (l >> 4);
        const int jj = bin - t->mel_start[m];
        if (jj >= 0 && jj < t->mel_cnt[m] && jj < 10) t->mel_a[frag + j][l] = t->mel_w[m][jj] * v3::P_SCALE;
      }
    frag += nk;
  }
  // units (bt, frame half) onto waves: longest first onto the SIMD with the least MFMA work so far,
  // four units per SIMD (a SIMD runs waves s, s + 4, s + 8, s + 12).  The mel shares interval B with
  // stage 2, whose 13 GEMMs (6 MFMAs of the mel K-step's 32 cycles each) sit on waves 0-12: SIMD 0
  // starts with 4 of them, the others with 3 (1 0: mel work alone)
  {
    int order[16];
    for (int u = 0; u < 16; ++u) order[u] = u;
    std::stable_sort(order, order + 16, [&](int x, int y) { return t->mel_bt_nk[x >> 1] > t->mel_bt_nk[y >> 1]; });
    int load[4] = {0, 0, 0, 0}, fill[4] = {0, 0, 0, 0};
    for (int w = 0; w < 13; ++w) load[w % 4] += 6;
    for (int k = 0; k < 16; ++k) {
      int best = -1;
      for (int s_ = 0; s_ < 4; ++s_)
        if (fill[s_] < 4 && (best < 0 || load[s_] < load[best])) best = s_;
      t->mel_unit[best + 4 * fill[best]++] = order[k];
      load[best] += t->mel_bt_nk[order[k] >> 1];
    }
  }

  // v3 MFMA A fragments (tools/fe_mfma_model.py restates these matrices): element j of lane l in
  // k-step s is A[row l & 31][k = 16 s + 8 (l >> 5) + j]; each value is rounded to float32, then
  // split hi = fp16(v), lo = fp16(v - hi)
  auto put = [](uint16_t (*dst)[2][2][64][8], int g, double (*A)[32]) {
    for (int s = 0; s < 2; ++s)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const float v = (float)A[l & 31][16 * s + 8 * (l >> 5) + j];
          const _Float16 hi = (_Float16)v;
          const _Float16 lo = (_Float16)(v - (float)hi);
          dst[g][s][0][l][j] = __builtin_bit_cast(uint16_t, hi);
          dst[g][s][1][l][j] = __builtin_bit_cast(uint16_t, lo);
        }
  };
  static double A[32][32];
  for (int n1 = 0; n1 < 16; ++n1) {   // stage 1: rows c = 2 k2 + ri, k = n2; window x W25 x 2^9
    for (int i = 0; i < 32; ++i)
      for (int k = 0; k < 32; ++k) A[i][k] = 0.0;
    for (int k2 = 0; k2 < 13; ++k2)
      for (int n2 = 0; n2 < 25; ++n2) {
        const double th = 2.0 * PI * n2 * k2 / 25.0;
        const double w = 0.5 - 0.5 * cos(2.0 * PI * (n1 + 16 * n2) / N_FFT);
        A[2 * k2][n2] = w * cos(th) * 512.0;
        A[2 * k2 + 1][n2] = k2 ? -w * sin(th) * 512.0 : 0.0;
      }
    put(t->a1, n1, A);
  }
  for (int k2 = 0; k2 < 13; ++k2) {   // stage 2: rows 2 i + ro, k = 2 n1 + ri; W400^(n1 bin) x 2^7
    for (int i = 0; i < 32; ++i)
      for (int k = 0; k < 32; ++k) A[i][k] = 0.0;
    for (int i = 0; i < 16; ++i) {
      const int bin = k2 == 0 ? (i <= 8 ? 25 * i : -1) : (i < 8 ? 25 * i + k2 : 25 * (i - 8) + 25 - k2);
      if (bin < 0) continue;
      const double sg = (k2 != 0 && i >= 8) ? -1.0 : 1.0;   // these bins read conj(Y_n1[k2])
      for (int n1 = 0; n1 < 16; ++n1) {
        const double th = 2.0 * PI * n1 * bin / 400.0;
        const double C = cos(th), S = (n1 * bin) % 200 == 0 ? 0.0 : -sin(th);
        A[2 * i][2 * n1] = C * 128.0;                // re = C a - sg S b  (x 2^7: Z carries 2^1 of A1's 2^9)
        A[2 * i][2 * n1 + 1] = -sg * S * 128.0;
        A[2 * i + 1][2 * n1] = S * 128.0;            // im = S a + sg C b
        A[2 * i + 1][2 * n1 + 1] = sg * C * 128.0;
      }
    }
    put(t->a2, k2, A);
  }
}
