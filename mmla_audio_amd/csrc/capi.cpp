// libmmla C ABI: context, weights, and the OD / SI pipelines over the HIP kernels.
// See include/mmla.h for the contract and the reference call site each entry point replaces.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <numeric>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mmla.h"
#include "conv.h"
#include "conv_h3.h"
#include "nets.h"
#include "resblk.h"
#include "od_fe.h"
#include <type_traits>
#include "si_fe.h"
#include "nr.h"
#include "vad.h"
#include "resample.h"
#include "siu.h"
#include "odu.h"

namespace {

constexpr int OD_H = 128, OD_W = 151, OD_PIX = OD_H * OD_W;
constexpr int OD_IMG = OD_PIX * 3;
constexpr int SI_T = 256, SI_D = 39;
constexpr int SI_NEED_SAMPLES = 160 * 259 + 400;   // frames 0..259 (delta-delta reach)
constexpr int CH[9] = {32, 32, 32, 64, 64, 64, 128, 128, 128};
constexpr bool POOL[9] = {true, false, false, true, false, false, true, false, false};

struct ConvW {
  float* wt = nullptr;
  float* bias = nullptr;
  uint16_t* wh = nullptr;   // 3xFP16 split weights [tap][cout_pad][cin_pad] (spatial convs only)
  uint16_t* wl = nullptr;
  uint16_t* fh = nullptr;   // fused res_block layout [cout][kpad], k = tap * cin + ci (resblk.hip)
  uint16_t* fl = nullptr;
  int kh = 0, kw = 0, cin = 0, cout = 0, cout_pad = 0, cin_pad = 0, kpad = 0;
  float wscale = 256.0f;    // power-of-two scale of the fp16 hi/lo split (pick_wscale)
  float unscale() const { return 1.0f / (16.0f * wscale); }   // x the 2^4 activation scale
};
struct BnW {
  float* scale = nullptr;
  float* shift = nullptr;
  int c = 0;
};
struct LstmW {
  float* wcat[2] = {nullptr, nullptr};
  float* bias[2] = {nullptr, nullptr};
  uint16_t* wth[2] = {nullptr, nullptr};   // 3xFP16 split, transposed [1024][256 + D] (nets.hip)
  uint16_t* wtl[2] = {nullptr, nullptr};
  float ws[2] = {256.0f, 256.0f};          // per-direction split scale (pick_wscale)
};
struct OdBlock {
  BnW bn_in, bn_mid;
  ConvW c3, c4, sc;
};
struct SiUnit {
  BnW bn_in, bn_mid;
  ConvW ca, cb, sc;
};
struct OdNet {
  ConvW stem;
  OdBlock blk[9];
  LstmW lstm;
  float* head_w = nullptr;
  float* head_b = nullptr;
};
struct SiNet {
  ConvW stem;
  SiUnit unit[9];
  BnW final_bn;
  LstmW lstm;
  ConvW dense;
  int k = 0, head = 0;
};

struct ProfRec {
  int stage;
  hipEvent_t a, b;
  double work;
};

}  // namespace

// Micro-batch caps (clips per internal pass).  The default (mmla_set_microbatch 0) is sized from
// the device's free memory at call time, capped here: 16384 OD clips = 124 GB of activations
// (4096: -2.4 % clips/s), 65536 SI clips = 9 GB (16384: -4 %).  A micro-batch whose workspace
// allocation fails is halved and retried (down to kMinMicrobatch) instead of failing the call.
constexpr int64_t kOdMicrobatch = 16384;
constexpr int64_t kSiMicrobatch = 65536;
constexpr int64_t kMinMicrobatch = 64;
// device bytes per clip of one micro-batch (workspace slots of run_od_net / run_si_net + FE I/O)
constexpr double kOdBytesPerClip = 3.0 * 128 * 151 * 32 * 4 + 128 * 151 * 3 + 128 * 151 * 4 +
                                   19 * 128 * 4 + 512 * 4 + 64;
constexpr double kSiBytesPerClip = 4.0 * 256 * 32 * 4 + 256 * 39 * 4 + 8 * 128 * 4 + 512 * 4 +
                                   1024 * 4 + 64;

struct mmla_ctx {
  bool prof_on = false;
  std::vector<ProfRec> prof_pending;
  std::vector<hipEvent_t> prof_pool;
  double prof_ms[MMLA_NSTAGES] = {0};
  double prof_work[MMLA_NSTAGES] = {0};
  int64_t prof_n[MMLA_NSTAGES] = {0};
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t own_stream = nullptr;
  std::string err;
  OdFeTables* od_tables = nullptr;
  SiFeTables* si_tables = nullptr;
  bool od_loaded = false, si_loaded = false;
  OdNet od;
  SiNet si;
  std::vector<void*> od_allocs, si_allocs;
  std::vector<void*> ws;
  std::vector<size_t> ws_size;
  std::vector<size_t> ws_guard;   // MMLA_WS_GUARD: guard bytes before and after each slot (0 = none)
  int64_t od_mb = 0, si_mb = 0;            // user caps (0 = sized from free memory)
  int64_t od_mb_cap = kOdMicrobatch, si_mb_cap = kSiMicrobatch;   // default caps of the automatic size
  int debug_fail_allocs = 0;   // test hook (env MMLA_DEBUG_FAIL_ALLOC at create): fail this many workspace allocations
  int precision = MMLA_PREC_F16X3;
  // SI res units without pooling as one fused kernel each (siu.hip); env MMLA_NO_SIU=1 at create:
  // the two conv_h3 launches (A/B)
  bool siu = true;
  // ... and the pool units too (siu.hip POOL); env MMLA_NO_SIPU=1 at create: the conv_h3 pair
  bool sipu = true;
  // ... and the last one with the final BN + ReLU + AvgPool4 (siu.hip FIN); env MMLA_NO_SIFIN=1: the
  // unit writes its output and bn_relu_avgpool4 runs as its own launch
  bool sifin = true;
  // ... and two consecutive units without pooling (2-3, 5-6, 8-9) as one kernel (siu.hip
  // siu_chain_kernel without a pool unit: the first unit's output stays on chip); env MMLA_NO_SIPAIR=1:
  // one launch each
  bool sipair = true;
  // ... and a pool unit with the two units after it (1-3, 4-6, 7-9) as one kernel (siu.hip
  // siu_chain_kernel POOL); env MMLA_NO_SICHAIN=1: the pool unit alone, then the pair
  bool sichain = true;
  // fused SI pipeline: si_fe writes 40-float feature rows for the stem (env MMLA_NO_SIPAD=1: 39)
  bool si_pad_feat = true;
  // OD blocks 4-9 as one fused kernel each (odu.hip: t1 on chip); env MMLA_NO_ODU=1 at create: the
  // conv_h3 pairs (A/B, bit-identical)
  bool odu = true;
  // OD blocks 1-3 as rolling column strips (rbs.hip); env MMLA_RB_TILE=1 at create: the 16 x 16 tile
  // kernels of resblk.hip instead
  bool rbs = true;
  // batches of <= lstm_split_max clips: the 3xFP16 BiLSTM with each direction's hidden units on eight workgroups
  // (nets.hip bilstm_h3_split_kernel); env MMLA_NO_LSTM_SPLIT=1 at create: one workgroup per direction
  bool lstm_split = true;
  // measured (tools/lat_split_sweep.py): OD 1.62 -> 1.53 ms at 128 clips, even at 192, +1 % at 256
  int lstm_split_max = 128;   // env MMLA_LSTM_SPLIT_MAX (A/B; the kernel takes up to 256)
  // test hook (env MMLA_DEBUG_LSTM_SPIN at create): the split BiLSTM's wait bound in polls (0 = default,
  // < 0 = give up at the first wait)
  int lstm_spin = 0;
  // 3xFP16 range guard: kernels set range_dev[0] (device-pointer calls; sticky until
  // mmla_range_check) or range_dev[1] (host-pointer micro-batches: re-run in exact f32) when an
  // operand they split into fp16 is >= 65504 in magnitude or not finite.  The split BiLSTM's wait
  // timeout (bilstm_h3_split_kernel) likewise: range_dev[3] (device-pointer calls, sticky) or
  // range_dev[2] (host-pointer micro-batches: re-run on the one-workgroup-per-direction kernel)
  int* range_dev = nullptr;
  int* range_host = nullptr;                // pinned copy of range_dev[1..2]
  // small host-pointer calls (the real-time loops' batch-1 case): the range flag and the outputs live
  // in host-mapped coherent memory that the kernels write over the bus, so a micro-batch ends with one
  // stream synchronisation and host memcpys instead of three or four device-to-host copies, a flag
  // memset and a second synchronisation (each copy ≈ 20 µs of a 0.55 ms call).  env MMLA_NO_PIN_OUT=1
  // at create: staging slots in HBM + hipMemcpyAsync (A/B)
  bool pin_small = true;
  int* range_map = nullptr;       // host view: [0] range flag, [1] split-BiLSTM timeout
  int* range_map_dev = nullptr;   // device view of the same words
  char* pin_out = nullptr;        // kPinSlots x kPinSlotBytes, host view
  char* pin_out_dev = nullptr;
  char* pin_in = nullptr;         // kPinInBytes of pinned input staging: one DMA for PCM + lens
  int* range_ptr = nullptr;                 // what the current launches write (null: unguarded)
  int* timeout_ptr = nullptr;               // where the split BiLSTM reports a timeout (null: nowhere)
  int64_t lstm_split_reruns = 0;
  int64_t range_reruns = 0;
  bool od_f32_only = false, si_f32_only = false;   // weights outside the fp16 range
  bool loading_f16_bad = false;                     // mmla_load_weights scratch
  VadState* vad_state = nullptr;   // mmla_vad_reset: webrtcvad.Vad(mode) per stream (device)
  int64_t vad_streams = 0;
  NrTables* nr_tables = nullptr;   // noise gate (nr.hip): tables + the noise profile's threshold
  float* nr_thresh = nullptr;
  bool nr_ready = false;
};

namespace {

int fail(mmla_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIPCHK(ctx, expr)                                                                    \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return fail(ctx, MMLA_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),   \
                  __FILE__, __LINE__);                                                       \
  } while (0)

#define CHK(expr)              \
  do {                         \
    int r_ = (expr);           \
    if (r_ != MMLA_OK) return r_; \
  } while (0)

// ---- tracing: hipEvents around each launch when enabled ---------------------------------------
hipEvent_t prof_event(mmla_ctx* c) {
  if (!c->prof_pool.empty()) {
    hipEvent_t e = c->prof_pool.back();
    c->prof_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

int prof_begin(mmla_ctx* c, int stage) {
  if (!c->prof_on) return -1;
  ProfRec r{stage, prof_event(c), prof_event(c), 0.0};
  (void)hipEventRecord(r.a, c->stream);
  c->prof_pending.push_back(r);
  return (int)c->prof_pending.size() - 1;
}

void prof_end(mmla_ctx* c, int idx, double work) {
  if (idx < 0) return;
  ProfRec& r = c->prof_pending[idx];
  r.work = work;
  (void)hipEventRecord(r.b, c->stream);
}

int prof_collect(mmla_ctx* c) {
  for (ProfRec& r : c->prof_pending) {
    HIPCHK(c, hipEventSynchronize(r.b));
    float ms = 0.0f;
    HIPCHK(c, hipEventElapsedTime(&ms, r.a, r.b));
    c->prof_ms[r.stage] += ms;
    c->prof_work[r.stage] += r.work;
    c->prof_n[r.stage] += 1;
    c->prof_pool.push_back(r.a);
    c->prof_pool.push_back(r.b);
  }
  c->prof_pending.clear();
  return MMLA_OK;
}

// launch `expr` (a hipError_t-returning launcher) as stage `st` with algorithmic work `wk`
#define LAUNCH(c, st, wk, expr)            \
  do {                                     \
    const int pi_ = prof_begin((c), (st)); \
    HIPCHK((c), (expr));                   \
    prof_end((c), pi_, (wk));              \
  } while (0)

// growable device workspace slots
// Debug aid: with MMLA_WS_GUARD=1 in the environment each slot allocated from then on is framed by
// 4 MiB guard bands filled with kGuardByte, and finish() fails the call if a kernel wrote into one
// (out-of-bounds stores that would otherwise land silently in a neighbouring allocation).
constexpr size_t kGuardBytes = 4u << 20;
constexpr int kGuardByte = 0xA5;

int ws_get(mmla_ctx* c, int slot, size_t bytes, void** out) {
  if ((int)c->ws.size() <= slot) {
    c->ws.resize(slot + 1, nullptr);
    c->ws_size.resize(slot + 1, 0);
    c->ws_guard.resize(slot + 1, 0);
  }
  const char* ge = std::getenv("MMLA_WS_GUARD");
  const size_t guard = ge && ge[0] == '1' ? kGuardBytes : 0;
  // guarded slots are re-framed whenever the size changes, so the trailing band always sits right
  // behind the live tensor (not behind the largest one ever requested)
  if (c->ws_size[slot] < bytes || (guard && c->ws_size[slot] != bytes)) {
    if (c->ws[slot]) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      HIPCHK(c, hipFree(static_cast<char*>(c->ws[slot]) - c->ws_guard[slot]));
      c->ws[slot] = nullptr;
      c->ws_size[slot] = 0;
    }
    void* p = nullptr;
    if (c->debug_fail_allocs > 0) {
      --c->debug_fail_allocs;
      return fail(c, MMLA_E_OOM, "workspace slot %d: injected allocation failure (MMLA_DEBUG_FAIL_ALLOC)", slot);
    }
    if (hipMalloc(&p, bytes + 2 * guard) != hipSuccess) {
      (void)hipGetLastError();   // clear the sticky allocation error
      return fail(c, MMLA_E_OOM, "hipMalloc(%zu) failed for workspace slot %d", bytes, slot);
    }
    if (guard) {   // on the context stream: ordered before the kernels that follow
      HIPCHK(c, hipMemsetAsync(p, kGuardByte, guard, c->stream));
      HIPCHK(c, hipMemsetAsync(static_cast<char*>(p) + guard + bytes, kGuardByte, guard, c->stream));
    }
    // Debug aid: MMLA_WS_POISON=<byte> fills every new slot with that byte (0xff: float NaN), so a
    // kernel that reads workspace memory no earlier launch wrote shows up in its results
    const char* pe = std::getenv("MMLA_WS_POISON");
    if (pe && pe[0])
      HIPCHK(c, hipMemsetAsync(static_cast<char*>(p) + guard, (int)std::strtol(pe, nullptr, 0) & 255,
                               bytes, c->stream));
    c->ws[slot] = static_cast<char*>(p) + guard;
    c->ws_size[slot] = bytes;
    c->ws_guard[slot] = guard;
  }
  *out = c->ws[slot];
  return MMLA_OK;
}

// free every workspace slot (after the stream drains)
int ws_release(mmla_ctx* c) {
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < c->ws.size(); ++i)
    if (c->ws[i]) {
      HIPCHK(c, hipFree(static_cast<char*>(c->ws[i]) - c->ws_guard[i]));
      c->ws[i] = nullptr;
      c->ws_size[i] = 0;
      c->ws_guard[i] = 0;
    }
  return MMLA_OK;
}

int ws_check_guards(mmla_ctx* c) {
  std::vector<unsigned char> h(kGuardBytes);
  for (size_t slot = 0; slot < c->ws.size(); ++slot) {
    const size_t g = c->ws_guard[slot];
    if (!c->ws[slot] || !g) continue;
    for (int side = 0; side < 2; ++side) {
      const char* d = static_cast<const char*>(c->ws[slot]) + (side ? c->ws_size[slot] : -(ptrdiff_t)g);
      HIPCHK(c, hipMemcpy(h.data(), d, g, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < g; ++i)
        if (h[i] != kGuardByte)
          return fail(c, MMLA_E_HIP, "workspace slot %zu: %s guard overwritten at byte %zu", slot,
                      side ? "trailing" : "leading", side ? i : g - i);
    }
  }
  return MMLA_OK;
}

enum Slot {
  S_PCM = 0, S_LENS, S_IMG, S_X, S_T1, S_T2, S_T3, S_SEQ, S_HOUT, S_LOGIT, S_FEAT, S_SILENT,
  S_OUT0, S_OUT1, S_OUT2, S_OUT3, S_IN,
  S_NR_S, S_NR_BITS, S_NR_FMAX, S_NR_FRAMES, S_NR_ITEMS, S_NR_Y, S_NR_ROWS,
  S_VAD_SPEECH, S_VAD_OUT, S_VAD_LENS, S_RS_TR, S_RS_WIN, S_LSTM
};

// ---- weights -------------------------------------------------------------------------------------

struct Cursor {
  const float* p;
  int64_t left;
  bool ok = true;
  const float* take(int64_t n) {
    if (n > left) {
      ok = false;
      return nullptr;
    }
    const float* r = p;
    p += n;
    left -= n;
    return r;
  }
};

int upload(mmla_ctx* c, std::vector<void*>& allocs, const void* host, size_t bytes, float** out) {
  void* d = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess) return fail(c, MMLA_E_OOM, "weight hipMalloc failed");
  allocs.push_back(d);
  HIPCHK(c, hipMemcpy(d, host, bytes, hipMemcpyHostToDevice));
  *out = static_cast<float*>(d);
  return MMLA_OK;
}

// The power-of-two scale at which a weight tensor is split into fp16 hi + lo for the 3xFP16 MFMA
// paths (one fixed 2^8 sent a whole model to exact f32 as soon as one weight
// reached 255.9).  2^8 for the usual max |w| in [1/16, 255.9) -- the arithmetic of earlier rounds,
// bit for bit -- else the scale that puts max |w| in [2^13, 2^14): far from the fp16 overflow and
// with the lo halves of the large weights normal.  The kernels multiply by its inverse (exact).
// false in *finite for a tensor holding inf / NaN (that model runs exact f32).
static float pick_wscale(const float* w, size_t n, bool* finite) {
  float m = 0.0f;
  *finite = true;
  for (size_t i = 0; i < n; ++i) {
    const float a = std::fabs(w[i]);
    if (!(a <= 3.4e38f)) *finite = false;
    else m = std::max(m, a);
  }
  if (m == 0.0f || (m < 255.9f && m >= 0.0625f)) return 256.0f;
  // e >= -126: the largest finite max |w| (< 2^128) needs e = -114, so after the clamp
  // m * 2^e < 2^14 for every finite tensor and its fp16 hi half never overflows
  const int e = std::max(-126, std::min(100, (int)std::floor(std::log2(16384.0 / m))));
  return std::ldexp(1.0f, e);
}

int take_conv(mmla_ctx* c, Cursor& cur, std::vector<void*>& al, int kh, int kw, int cin, int cout,
              ConvW* w) {
  const float* k = cur.take((int64_t)kh * kw * cin * cout);
  const float* b = cur.take(cout);
  if (!cur.ok) return fail(c, MMLA_E_SHAPE, "weight blob too short");
  // 3xFP16: any finite tensor fits the fp16 split at its own power-of-two scale
  bool finite = true;
  w->wscale = pick_wscale(k, (size_t)kh * kw * cin * cout, &finite);
  if (!finite) c->loading_f16_bad = true;
  w->kh = kh;
  w->kw = kw;
  w->cin = cin;
  w->cout = cout;
  w->cout_pad = (cout + 31) / 32 * 32;
  if (w->cout_pad > 128) w->cout_pad = (cout + 127) / 128 * 128;
  std::vector<float> kp((size_t)kh * kw * cin * w->cout_pad, 0.0f), bp(w->cout_pad, 0.0f);
  for (int64_t r = 0; r < (int64_t)kh * kw * cin; ++r)
    memcpy(&kp[r * w->cout_pad], k + r * cout, sizeof(float) * cout);
  memcpy(bp.data(), b, sizeof(float) * cout);
  CHK(upload(c, al, kp.data(), kp.size() * sizeof(float), &w->wt));
  CHK(upload(c, al, bp.data(), bp.size() * sizeof(float), &w->bias));
  // spatial conv: also the 3xFP16 operand layout (cin % 4 != 0: only the SI stem's 4-tap Conv1D,
  // conv_h3.hip stages it element-wise)
  // (1x1 convs with 16-channel steps too: the OD pool blocks' shortcut, fused into the pooled conv(4,1))
  if ((kh * kw > 1 && (cin % 4 == 0 || (kh == 4 && kw == 1 && cout <= 32))) || (kh * kw == 1 && cin % 16 == 0)) {
    w->cin_pad = (cin + 15) / 16 * 16;
    const size_t n = (size_t)kh * kw * w->cout_pad * w->cin_pad;
    std::vector<uint16_t> hi(n), lo(n);
    conv_h3_split_weights(k, kh, kw, cin, cout, w->cin_pad, w->cout_pad, hi.data(), lo.data(),
                          w->wscale);
    float* p = nullptr;
    CHK(upload(c, al, hi.data(), n * sizeof(uint16_t), &p));
    w->wh = reinterpret_cast<uint16_t*>(p);
    CHK(upload(c, al, lo.data(), n * sizeof(uint16_t), &p));
    w->wl = reinterpret_cast<uint16_t*>(p);
  }
  if (cin % 16 == 0 && cout % 16 == 0) {   // fused res_block layout (resblk.hip)
    w->kpad = (kh * kw * cin + 31) / 32 * 32;
    const size_t n = (size_t)cout * w->kpad;
    std::vector<uint16_t> hi(n), lo(n);
    // the 3x3 (GEMM 1) and conv(4,1) (GEMM 2) weights in MFMA fragment order; the 1x1 shortcut
    // keeps [co][k] rows
    resblk_split_weights(k, kh * kw, cin, cout, w->kpad, hi.data(), lo.data(), kh > 1, w->wscale);
    float* p = nullptr;
    CHK(upload(c, al, hi.data(), n * sizeof(uint16_t), &p));
    w->fh = reinterpret_cast<uint16_t*>(p);
    CHK(upload(c, al, lo.data(), n * sizeof(uint16_t), &p));
    w->fl = reinterpret_cast<uint16_t*>(p);
  }
  return MMLA_OK;
}

int take_bn(mmla_ctx* c, Cursor& cur, std::vector<void*>& al, int ch, BnW* bn) {
  const float* g = cur.take(ch);
  const float* be = cur.take(ch);
  const float* m = cur.take(ch);
  const float* v = cur.take(ch);
  if (!cur.ok) return fail(c, MMLA_E_SHAPE, "weight blob too short");
  std::vector<float> sc(ch), sh(ch);
  for (int i = 0; i < ch; ++i) {   // Keras BN(eps=1e-3) inference: x * s + (beta - mean * s)
    const double s = (double)g[i] / std::sqrt((double)v[i] + 1e-3);
    sc[i] = (float)s;
    sh[i] = (float)((double)be[i] - (double)m[i] * s);
  }
  bn->c = ch;
  CHK(upload(c, al, sc.data(), ch * sizeof(float), &bn->scale));
  CHK(upload(c, al, sh.data(), ch * sizeof(float), &bn->shift));
  return MMLA_OK;
}

int take_lstm(mmla_ctx* c, Cursor& cur, std::vector<void*>& al, int d, LstmW* l) {
  for (int dir = 0; dir < 2; ++dir) {
    const float* k = cur.take((int64_t)d * 1024);
    const float* r = cur.take(256 * 1024);
    const float* b = cur.take(1024);
    if (!cur.ok) return fail(c, MMLA_E_SHAPE, "weight blob too short");
    std::vector<float> wc((size_t)(256 + d) * 1024);
    memcpy(wc.data(), r, sizeof(float) * 256 * 1024);
    memcpy(wc.data() + 256 * 1024, k, sizeof(float) * d * 1024);
    CHK(upload(c, al, wc.data(), wc.size() * sizeof(float), &l->wcat[dir]));
    CHK(upload(c, al, b, 1024 * sizeof(float), &l->bias[dir]));
    bool finite = true;
    l->ws[dir] = pick_wscale(wc.data(), wc.size(), &finite);
    if (!finite) c->loading_f16_bad = true;
    std::vector<uint16_t> hi(wc.size()), lo(wc.size());
    bilstm_h3_split_weights(wc.data(), d, hi.data(), lo.data(), l->ws[dir]);
    float* p = nullptr;
    CHK(upload(c, al, hi.data(), hi.size() * sizeof(uint16_t), &p));
    l->wth[dir] = reinterpret_cast<uint16_t*>(p);
    CHK(upload(c, al, lo.data(), lo.size() * sizeof(uint16_t), &p));
    l->wtl[dir] = reinterpret_cast<uint16_t*>(p);
  }
  return MMLA_OK;
}

void free_allocs(std::vector<void*>& al) {
  for (void* p : al) (void)hipFree(p);
  al.clear();
}

// ---- PCM staging -------------------------------------------------------------------------------

// host-pinned staging of small host-pointer calls (mmla_ctx::pin_small)
constexpr size_t kPinSlotBytes = 64u << 10;
constexpr size_t kPinInBytes = 1u << 20;

template <typename T>
struct PcmT {
  const T* p;
  int64_t stride;
  const int32_t* lens;
  int32_t clip_len;
};
using Pcm = PcmT<int16_t>;

// Device view of clips [c0, c0 + cnt): offsets in device mode, a dense copy of the first
// `need` samples per clip in host mode.
template <typename T>
int stage_pcm(mmla_ctx* c, const T* pcm, int64_t c0, int64_t cnt, int64_t stride,
              const int32_t* lens, int32_t clip_len, int need, bool dev, PcmT<T>* out) {
  if (dev) {
    *out = {pcm + c0 * stride, stride, lens ? lens + c0 : nullptr, clip_len};
    return MMLA_OK;
  }
  int64_t width = lens ? std::min<int64_t>(need, stride) : std::min<int64_t>(need, clip_len);
  if (width < 1) width = 1;
  void* dp = nullptr;
  const bool overlap = !lens && stride < width;
  const size_t pbytes = (size_t)(overlap ? (cnt - 1) * stride + width : cnt * width) * sizeof(T);
  const size_t loff = (pbytes + 255) & ~(size_t)255;
  if (c->pin_small && c->pin_in && loff + (lens ? cnt * sizeof(int32_t) : 0) <= kPinInBytes) {
    // small calls: gather into pinned memory on the host, one asynchronous DMA (host-mode bodies
    // end with a stream synchronisation, so the staging is free again when the next one starts)
    if (overlap) {
      std::memcpy(c->pin_in, pcm + c0 * stride, pbytes);
    } else {
      for (int64_t i = 0; i < cnt; ++i)
        std::memcpy(c->pin_in + (size_t)i * width * sizeof(T), pcm + (c0 + i) * stride, width * sizeof(T));
    }
    const size_t tot = loff + (lens ? cnt * sizeof(int32_t) : 0);
    if (lens) std::memcpy(c->pin_in + loff, lens + c0, cnt * sizeof(int32_t));
    CHK(ws_get(c, S_PCM, tot, &dp));
    HIPCHK(c, hipMemcpyAsync(dp, c->pin_in, tot, hipMemcpyHostToDevice, c->stream));
    const int32_t* dl = lens ? reinterpret_cast<const int32_t*>(static_cast<char*>(dp) + loff) : nullptr;
    *out = {static_cast<T*>(dp), overlap ? stride : width, dl, (int32_t)std::min<int64_t>(clip_len, width)};
    return MMLA_OK;
  }
  if (!lens && stride < width) {
    // overlapping windows of one signal (segmentation with step < window): copy the covered span
    // once and let the kernels read window c at c * stride
    const int64_t span = (cnt - 1) * stride + width;
    CHK(ws_get(c, S_PCM, (size_t)span * sizeof(T), &dp));
    HIPCHK(c, hipMemcpyAsync(dp, pcm + c0 * stride, span * sizeof(T), hipMemcpyHostToDevice,
                             c->stream));
    *out = {static_cast<T*>(dp), stride, nullptr, (int32_t)std::min<int64_t>(clip_len, width)};
    return MMLA_OK;
  }
  CHK(ws_get(c, S_PCM, (size_t)cnt * width * sizeof(T), &dp));
  HIPCHK(c, hipMemcpy2DAsync(dp, width * sizeof(T), pcm + c0 * stride, stride * sizeof(T),
                             width * sizeof(T), cnt, hipMemcpyHostToDevice, c->stream));
  int32_t* dl = nullptr;
  if (lens) {
    void* lp = nullptr;
    CHK(ws_get(c, S_LENS, (size_t)cnt * sizeof(int32_t), &lp));
    HIPCHK(c, hipMemcpyAsync(lp, lens + c0, cnt * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    dl = static_cast<int32_t*>(lp);
  }
  *out = {static_cast<T*>(dp), width, dl, (int32_t)std::min<int64_t>(clip_len, width)};
  return MMLA_OK;
}

// device destination for an output chunk: the caller's pointer (device mode), a host-mapped slot
// (small host-mode outputs, mmla_ctx::pin_small) or a staging slot in HBM
constexpr int kPinSlots = 4;   // S_OUT0 .. S_OUT3
template <typename T>
int out_ptr(mmla_ctx* c, T* user, int64_t off, size_t count, bool dev, int slot, T** d) {
  if (!user) {
    *d = nullptr;
    return MMLA_OK;
  }
  if (dev) {
    *d = user + off;
    return MMLA_OK;
  }
  if (c->pin_small && c->pin_out_dev && slot >= S_OUT0 && slot < S_OUT0 + kPinSlots &&
      count * sizeof(T) <= kPinSlotBytes) {
    *d = reinterpret_cast<T*>(c->pin_out_dev + (size_t)(slot - S_OUT0) * kPinSlotBytes);
    return MMLA_OK;
  }
  void* p = nullptr;
  CHK(ws_get(c, slot, count * sizeof(T), &p));
  *d = static_cast<T*>(p);
  return MMLA_OK;
}

template <typename T>
int copy_back(mmla_ctx* c, T* user, int64_t off, const T* d, size_t count, bool dev) {
  if (!user || dev) return MMLA_OK;
  const char* dc = reinterpret_cast<const char*>(d);
  if (c->pin_out_dev && dc >= c->pin_out_dev && dc < c->pin_out_dev + kPinSlots * kPinSlotBytes) {
    HIPCHK(c, hipStreamSynchronize(c->stream));   // the kernels wrote host memory: wait, then copy
    std::memcpy(user + off, c->pin_out + (dc - c->pin_out_dev), count * sizeof(T));
    return MMLA_OK;
  }
  HIPCHK(c, hipMemcpyAsync(user + off, d, count * sizeof(T), hipMemcpyDeviceToHost, c->stream));
  return MMLA_OK;
}

int finish(mmla_ctx* c, bool dev) {
  HIPCHK(c, hipGetLastError());
  bool guarded = false;
  for (size_t g : c->ws_guard) guarded |= g != 0;
  if (!dev || guarded) HIPCHK(c, hipStreamSynchronize(c->stream));
  if (guarded) return ws_check_guards(c);
  return MMLA_OK;
}

// ---- micro-batching and the 3xFP16 range guard -------------------------------------------------

// clips per micro-batch: the user's cap, else what the device's free memory holds (the slots this
// context already owns count as free), capped at the default
int64_t microbatch(mmla_ctx* c, bool od) {
  const int64_t user = od ? c->od_mb : c->si_mb;
  if (user > 0) return user;
  const int64_t cap = od ? c->od_mb_cap : c->si_mb_cap;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
    (void)hipGetLastError();
    return cap;
  }
  double held = 0;
  for (size_t b : c->ws_size) held += (double)b;
  int64_t fit = (int64_t)(((double)fr + held) * 0.9 / (od ? kOdBytesPerClip : kSiBytesPerClip));
  fit = fit / kMinMicrobatch * kMinMicrobatch;
  return std::max(kMinMicrobatch, std::min(cap, fit));
}

// body(c0, cnt) over clips [0, n) in micro-batches.  A workspace allocation failure (MMLA_E_OOM)
// frees the context's workspaces, halves the micro-batch (unless the caller fixed it with
// mmla_set_microbatch) and retries the same clips; the halving holds for the rest of this call only
// (a transient OOM, e.g. while another context held memory, must not cap every later call).
template <class F>
int for_microbatches(mmla_ctx* c, bool od, int64_t n, F&& body) {
  int64_t c0 = 0;
  int64_t mb = microbatch(c, od);   // fixed for the call (unless an allocation fails)
  while (c0 < n) {
    const int64_t cnt = std::min(mb, n - c0);
    const int rc = body(c0, cnt);
    if (rc == MMLA_E_OOM && (od ? c->od_mb : c->si_mb) == 0 && cnt > kMinMicrobatch) {
      CHK(ws_release(c));
      mb = std::max(kMinMicrobatch, cnt / 2);   // this call only: the next call re-reads free memory
      continue;
    }
    CHK(rc);
    c0 += cnt;
  }
  return MMLA_OK;
}

// one micro-batch of a network call under the 3xFP16 range guard.  Device-pointer calls let the
// kernels flag into range_dev[0] (sticky, reported by mmla_range_check / mmla_synchronize);
// host-pointer calls check range_dev[1] after the micro-batch and re-run it in exact f32 when an
// operand left the fp16 range.  f32_only: the model's weights are outside the fp16 range.
template <class F>
int guarded(mmla_ctx* c, bool dev, bool f32_only, F&& body) {
  struct Restore {   // precision, split switch and flag targets of the context, restored on every return
    mmla_ctx* c;
    int prec;
    bool split;
    ~Restore() {
      c->precision = prec;
      c->lstm_split = split;
      c->range_ptr = nullptr;
      c->timeout_ptr = nullptr;
    }
  } restore{c, c->precision, c->lstm_split};
  if (f32_only) c->precision = MMLA_PREC_F32;
  if (c->precision != MMLA_PREC_F16X3) {
    c->range_ptr = nullptr;
    return body();
  }
  if (dev) {
    c->range_ptr = c->range_dev;
    c->timeout_ptr = c->range_dev + 3;
    return body();
  }
  // one pass of the micro-batch; -> its range flag and split-BiLSTM timeout flag
  auto pass = [&](bool* flagged, bool* timed_out) -> int {
    if (c->pin_small && c->range_map) {   // the flags in host-mapped memory: no memset, no copy
      c->range_ptr = c->range_map_dev;
      c->timeout_ptr = c->range_map_dev + 1;
      reinterpret_cast<volatile int*>(c->range_map)[0] = 0;   // host calls leave the stream idle
      reinterpret_cast<volatile int*>(c->range_map)[1] = 0;
      CHK(body());
      HIPCHK(c, hipStreamSynchronize(c->stream));
      *flagged = reinterpret_cast<volatile int*>(c->range_map)[0] != 0;
      *timed_out = reinterpret_cast<volatile int*>(c->range_map)[1] != 0;
    } else {
      c->range_ptr = c->range_dev + 1;
      c->timeout_ptr = c->range_dev + 2;
      HIPCHK(c, hipMemsetAsync(c->range_ptr, 0, 2 * sizeof(int), c->stream));
      CHK(body());
      HIPCHK(c, hipMemcpyAsync(c->range_host, c->range_ptr, 2 * sizeof(int), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      *flagged = c->range_host[0] != 0;
      *timed_out = c->range_host[1] != 0;
    }
    return MMLA_OK;
  };
  bool flagged = false, timed_out = false;
  CHK(pass(&flagged, &timed_out));
  if (timed_out) {   // a split-BiLSTM workgroup gave up waiting (NaN outputs): the unsplit kernel,
    c->lstm_split = false;   // the same arithmetic bit for bit
    c->lstm_split_reruns += 1;
    CHK(pass(&flagged, &timed_out));
    if (timed_out) return fail(c, MMLA_E_HIP, "BiLSTM timed out without the split kernel");
  }
  if (flagged) {
    c->precision = MMLA_PREC_F32;
    c->range_ptr = nullptr;
    c->timeout_ptr = nullptr;
    c->range_reruns += 1;
    CHK(body());
  }
  return MMLA_OK;
}

// ---- network runners (device pointers, one micro-batch) -----------------------------------------

ConvArgs conv_args(const ConvW& w, const float* x, float* y, int n, int h, int wd, int stride,
                   const BnW* bn, int pro, int epi, const float* res) {
  ConvArgs a{};
  a.x = x;
  a.wt = w.wt;
  a.bias = w.bias;
  a.scale = bn ? bn->scale : nullptr;
  a.shift = bn ? bn->shift : nullptr;
  a.res = res;
  a.y = y;
  a.n = n;
  a.h = h;
  a.w = wd;
  a.cin = w.cin;
  a.ho = (h + stride - 1) / stride;
  a.wo = (wd + stride - 1) / stride;
  a.cout = w.cout;
  a.cout_pad = w.cout_pad;
  a.ldy = w.cout;
  a.kh = w.kh;
  a.kw = w.kw;
  a.stride = stride;
  const int th = std::max((a.ho - 1) * stride + w.kh - h, 0);
  const int tw = std::max((a.wo - 1) * stride + w.kw - wd, 0);
  a.pad_h = th / 2;   // Keras 'same': extra padding goes after
  a.pad_w = tw / 2;
  a.pro = pro;
  a.epi = epi;
  return a;
}

double conv_flops(const ConvArgs& a) {
  return 2.0 * (double)a.n * a.ho * a.wo * a.kh * a.kw * a.cin * a.cout;
}

int conv_run(mmla_ctx* c, const ConvArgs& a, int stage = MMLA_STAGE_CONV) {
  LAUNCH(c, stage, conv_flops(a), conv_launch(a, c->stream));
  return MMLA_OK;
}

// spatial conv on the 3xFP16 path when enabled (falls back to the exact-f32 kernel otherwise);
// pool_out: write MaxPool2D(2,'same') of the output instead of the output (OD pool blocks).
// sc / sc_x (pool_out only): the block's shortcut Conv2D(1x1, stride 2) of sc_x, added to the pooled
// output inside the same launch
int conv_spatial(mmla_ctx* c, const ConvW& w, const float* x, float* y, int n, int h, int wd,
                 const BnW* bn, int pro, int epi, const float* res, bool pool_out = false,
                 int pool_in_h = 0, const ConvW* sc = nullptr, const float* sc_x = nullptr,
                 int sc_h = 0) {
  if (c->precision == MMLA_PREC_F16X3 && w.wh) {
    ConvH3Args a{};
    double sc_flops = 0.0;
    if (sc && sc_x) {
      a.sc_x = sc_x;
      a.sc_wh = sc->wh;
      a.sc_wl = sc->wl;
      a.sc_bias = sc->bias;
      a.sc_cin = sc->cin;
      a.sc_h = sc_h;
      a.sc_unscale = sc->unscale();
      // pooled 2-D blocks: one output per pooled pixel; Conv1D: one per output row (h = rows)
      sc_flops = sc_h > 0 ? 2.0 * n * h * sc->cin * sc->cout
                          : 2.0 * n * ((h + 1) / 2) * ((wd + 1) / 2) * sc->cin * sc->cout;
    }
    a.pool_in = pool_in_h > 0;   // x = the unpooled [n, pool_in_h, 1, cin] (MaxPool1D fused)
    a.h_in = pool_in_h;
    a.x = x;
    a.wh = w.wh;
    a.wl = w.wl;
    a.unscale = w.unscale();
    a.bias = w.bias;
    a.scale = bn ? bn->scale : nullptr;
    a.shift = bn ? bn->shift : nullptr;
    a.res = res;
    a.y = y;
    a.n = n;
    a.h = h;
    a.w = wd;
    a.cin = w.cin;
    a.cin_pad = w.cin_pad;
    a.cout = w.cout;
    a.cout_pad = w.cout_pad;
    a.kh = w.kh;
    a.kw = w.kw;
    a.pad_h = (w.kh - 1) / 2;   // Keras 'same', stride 1: extra padding after
    a.pad_w = (w.kw - 1) / 2;
    a.pro = pro;
    a.epi = epi;
    a.pool_out = pool_out ? 1 : 0;
    a.range_flag = c->range_ptr;
    LAUNCH(c, MMLA_STAGE_CONV, 2.0 * n * h * wd * w.kh * w.kw * w.cin * w.cout + sc_flops,
           conv_h3_launch(a, c->stream));
    return MMLA_OK;
  }
  ConvArgs a = conv_args(w, x, y, n, h, wd, 1, bn, pro, epi, res);
  if (!pool_out) return conv_run(c, a);
  return fail(c, MMLA_E_INVALID, "pooled epilogue needs the 3xFP16 conv path");
}

double lstm_flops(int64_t n, int T, int D) { return 2.0 * n * T * 2 * (256.0 + D) * 1024.0; }

// BiLSTM on the 3xFP16 path when enabled (exact-f32 MFMA kernel otherwise)
hipError_t lstm_run(mmla_ctx* c, const LstmW& L, const float* seq, int64_t n, int T, float* out) {
  if (c->precision == MMLA_PREC_F16X3 && L.wth[0] && c->lstm_split &&
      n <= std::min(c->lstm_split_max, bilstm_h3_split_max_clips())) {
    void* ws = nullptr;   // small batches (the real-time calls): each direction over eight CUs
    if (ws_get(c, S_LSTM, bilstm_h3_split_ws_bytes(), &ws) != MMLA_OK) return hipErrorOutOfMemory;
    return bilstm_h3_split_launch(seq, (int)n, T, 128, L.wth[0], L.wtl[0], L.wth[1], L.wtl[1],
                                  L.bias[0], L.bias[1], out, c->range_ptr, L.ws[0], L.ws[1], ws,
                                  c->timeout_ptr, c->lstm_spin, c->stream);
  }
  if (c->precision == MMLA_PREC_F16X3 && L.wth[0])
    return bilstm_h3_launch(seq, (int)n, T, 128, L.wth[0], L.wtl[0], L.wth[1], L.wtl[1], L.bias[0],
                            L.bias[1], out, c->range_ptr, L.ws[0], L.ws[1], c->stream);
  return bilstm_launch(seq, (int)n, T, 128, L.wcat[0], L.wcat[1], L.bias[0], L.bias[1], out,
                       c->stream);
}

// the OD 'silent' gate (record_on_pc.py:141-154) of one micro-batch: device lens (nullable) or
// clip_len; silent output (nullable)
struct OdGate {
  const int32_t* lens = nullptr;
  int clip_len = -1;   // < 0: no gate (network-only calls)
  uint8_t* silent = nullptr;
};

// OD-NET on a device batch; input = uint8 image (img_u8) or float NHWC (img_f32).
// `stop` >= 0 (debug trace): return after stage `stop` (0 stem, 1..9 res blocks, 10 mean, 11
// BiLSTM) with *tap / *tap_n set to that stage's output tensor.
int run_od_net(mmla_ctx* c, const uint8_t* img_u8, const float* img_f32, int64_t n, float* probs,
               int32_t* argmax, OdGate gate = OdGate(), int stop = -1, const float** tap = nullptr,
               int64_t* tap_n = nullptr) {
  const OdNet& W = c->od;
  const size_t big = (size_t)n * OD_PIX * 32 * sizeof(float);
  void *px, *pt1, *pt2, *pseq, *ph;
  CHK(ws_get(c, S_X, big, &px));
  CHK(ws_get(c, S_T1, big, &pt1));
  CHK(ws_get(c, S_T2, big, &pt2));
  CHK(ws_get(c, S_SEQ, (size_t)n * 19 * 128 * sizeof(float), &pseq));
  CHK(ws_get(c, S_HOUT, (size_t)n * 512 * sizeof(float), &ph));
  float* X = static_cast<float*>(px);
  float* T1 = static_cast<float*>(pt1);
  float* T2 = static_cast<float*>(pt2);
  // Conv2D(16, 1x1) on the PNG image (overlap_detector_temp.py:282): computed inside block 1's
  // staging when block 1 runs fused (resblk.hip STEM), else its own launch
  // blocks 1-3 as rolling strips (rbs.hip) on the conv_h3 weight layout
  auto rbs_ok = [&](int b, int hh, int ww) {
    const OdBlock& B = W.blk[b];
    return c->rbs && c->precision == MMLA_PREC_F16X3 && B.c3.wh && B.c4.wh && (!POOL[b] || B.sc.wh) &&
           B.c3.cin_pad == B.c3.cin && B.c3.cout_pad == 32 && B.c4.cin_pad == 32 && B.c4.cout_pad == 32 &&
           B.c4.kh == 4 && B.c4.kw == 1 && (!POOL[b] || (B.sc.cin_pad == B.c3.cin && B.sc.cout_pad == 32)) &&
           rbs_supported(hh, ww, B.c3.cin, B.c3.cout, POOL[b]);
  };
  const bool rbs_stem = stop != 0 && rbs_ok(0, OD_H, OD_W);
  const bool fuse_stem = c->precision == MMLA_PREC_F16X3 && stop != 0 &&
                         (rbs_stem || (W.blk[0].c3.fh && W.blk[0].c4.fh && W.blk[0].sc.fh &&
                                       resblk_supported(W.blk[0].c3.cin, W.blk[0].c3.cout, POOL[0])));
  if (!fuse_stem)
    LAUNCH(c, MMLA_STAGE_GLUE, 2.0 * n * OD_PIX * 3 * 16,
           od_stem_launch(img_u8, img_f32, n * OD_PIX, W.stem.cout_pad, W.stem.wt, W.stem.bias, X,
                          c->stream));
  int h = OD_H, w = OD_W;
  if (stop == 0) {
    *tap = X;
    *tap_n = n * OD_PIX * 16;
    return MMLA_OK;
  }
  for (int b = 0; b < 9; ++b) {   // res_block, overlap_detector_temp.py:253-277
    const OdBlock& B = W.blk[b];
    if ((b == 0 ? rbs_stem && fuse_stem : rbs_ok(b, h, w))) {
      // whole block in one launch, rolling down 16-column strips: t1 stays in LDS (rbs.hip)
      ResBlkArgs r{};
      r.x = X;
      r.w1h = B.c3.wh;
      r.w1l = B.c3.wl;
      r.b1 = B.c3.bias;
      r.u1 = B.c3.unscale();
      r.u2 = B.c4.unscale();
      r.us = POOL[b] ? B.sc.unscale() : 0.0f;
      r.s1 = B.bn_in.scale;
      r.t1 = B.bn_in.shift;
      r.w2h = B.c4.wh;
      r.w2l = B.c4.wl;
      r.b2 = B.c4.bias;
      r.s2 = B.bn_mid.scale;
      r.t2 = B.bn_mid.shift;
      if (POOL[b]) {
        r.wsh = B.sc.wh;
        r.wsl = B.sc.wl;
        r.bs = B.sc.bias;
      }
      r.y = T1;
      if (b == 0) {
        r.x = nullptr;
        r.img8 = img_u8;
        r.imgf = img_u8 ? nullptr : img_f32;
        r.wst = W.stem.wt;
        r.bst = W.stem.bias;
        r.ldst = W.stem.cout_pad;
      }
      r.n = (int)n;
      r.h = h;
      r.w = w;
      r.range_flag = c->range_ptr;
      LAUNCH(c, MMLA_STAGE_CONV,
             (b == 0 ? 2.0 * n * h * w * 3 * 16 : 0.0) +
             2.0 * n * h * w * (9.0 * B.c3.cin * B.c3.cout + 4.0 * B.c4.cin * B.c4.cout) +
                 (POOL[b] ? 2.0 * n * ((h + 1) / 2) * ((w + 1) / 2) * B.sc.cin * B.sc.cout : 0.0),
             rbs_launch(r, B.c3.cin, B.c3.cout, POOL[b], c->stream));
      if (POOL[b]) {
        h = (h + 1) / 2;
        w = (w + 1) / 2;
      }
      std::swap(X, T1);
      if (stop == b + 1) {
        *tap = X;
        *tap_n = n * h * w * CH[b];
        return MMLA_OK;
      }
      continue;
    }
    if (c->precision == MMLA_PREC_F16X3 && B.c3.fh && B.c4.fh && B.c4.kpad == 4 * B.c4.cin &&
        (!POOL[b] || B.sc.fh) &&
        resblk_supported(B.c3.cin, B.c3.cout, POOL[b])) {
      // whole block in one launch: t1 stays in LDS (resblk.hip)
      ResBlkArgs r{};
      r.x = X;
      r.w1h = B.c3.fh;
      r.w1l = B.c3.fl;
      r.b1 = B.c3.bias;
      r.u1 = B.c3.unscale();
      r.u2 = B.c4.unscale();
      r.us = POOL[b] ? B.sc.unscale() : 0.0f;
      r.s1 = B.bn_in.scale;
      r.t1 = B.bn_in.shift;
      r.w2h = B.c4.fh;
      r.w2l = B.c4.fl;
      r.b2 = B.c4.bias;
      r.s2 = B.bn_mid.scale;
      r.t2 = B.bn_mid.shift;
      if (POOL[b]) {
        r.wsh = B.sc.fh;
        r.wsl = B.sc.fl;
        r.bs = B.sc.bias;
      }
      r.y = T1;
      if (b == 0 && fuse_stem) {
        r.x = nullptr;
        r.img8 = img_u8;
        r.imgf = img_u8 ? nullptr : img_f32;
        r.wst = W.stem.wt;
        r.bst = W.stem.bias;
        r.ldst = W.stem.cout_pad;
      }
      r.n = (int)n;
      r.h = h;
      r.w = w;
      r.range_flag = c->range_ptr;
      LAUNCH(c, MMLA_STAGE_CONV,
             (b == 0 && fuse_stem ? 2.0 * n * h * w * 3 * 16 : 0.0) +
             2.0 * n * h * w * (9.0 * B.c3.cin * B.c3.cout + 4.0 * B.c4.cin * B.c4.cout) +
                 (POOL[b] ? 2.0 * n * ((h + 1) / 2) * ((w + 1) / 2) * B.sc.cin * B.sc.cout : 0.0),
             resblk_launch(r, B.c3.cin, B.c3.cout, POOL[b], c->stream));
      if (POOL[b]) {
        h = (h + 1) / 2;
        w = (w + 1) / 2;
      }
      std::swap(X, T1);
      if (stop == b + 1) {
        *tap = X;
        *tap_n = n * h * w * CH[b];
        return MMLA_OK;
      }
      continue;
    }
    if (c->odu && c->precision == MMLA_PREC_F16X3 && B.c3.wh && B.c4.wh && (!POOL[b] || B.sc.wh) &&
        odu_supported(h, w, B.c3.cin, B.c3.cout, POOL[b]) && B.c3.cin_pad == B.c3.cin &&
        B.c3.cout_pad == B.c3.cout && B.c4.cin == B.c3.cout && B.c4.cout == B.c3.cout &&
        B.c4.cin_pad == B.c4.cin && B.c4.cout_pad == B.c4.cout && B.c4.kh == 4 && B.c4.kw == 1 &&
        (!POOL[b] || (B.sc.cin == B.c3.cin && B.sc.cout == B.c3.cout && B.sc.cout_pad == B.sc.cout))) {
      // the whole block in one launch: t1 stays in LDS (odu.hip), bit-identical to the pair below
      OduArgs o{};
      o.x = X;
      o.y = T1;
      o.wah = B.c3.wh;
      o.wal = B.c3.wl;
      o.wbh = B.c4.wh;
      o.wbl = B.c4.wl;
      o.ba = B.c3.bias;
      o.bb = B.c4.bias;
      o.s_in = B.bn_in.scale;
      o.t_in = B.bn_in.shift;
      o.s_mid = B.bn_mid.scale;
      o.t_mid = B.bn_mid.shift;
      o.ua = B.c3.unscale();
      o.ub = B.c4.unscale();
      o.n = (int)n;
      o.range_flag = c->range_ptr;
      if (POOL[b]) {
        o.wsh = B.sc.wh;
        o.wsl = B.sc.wl;
        o.bs = B.sc.bias;
        o.us = B.sc.unscale();
      }
      LAUNCH(c, MMLA_STAGE_CONV,
             2.0 * n * h * w * (9.0 * B.c3.cin * B.c3.cout + 4.0 * B.c4.cin * B.c4.cout) +
                 (POOL[b] ? 2.0 * n * (h / 2) * (w / 2) * B.sc.cin * B.sc.cout : 0.0),
             odu_launch(o, h, w, B.c3.cin, B.c3.cout, POOL[b], c->stream));
      if (POOL[b]) {
        h /= 2;
        w /= 2;
      }
      std::swap(X, T1);
      if (stop == b + 1) {
        *tap = X;
        *tap_n = n * h * w * CH[b];
        return MMLA_OK;
      }
      continue;
    }
    CHK(conv_spatial(c, B.c3, X, T1, (int)n, h, w, &B.bn_in, PRO_BN_ELU, EPI_BIAS, nullptr));
    if (POOL[b]) {
      if (c->precision == MMLA_PREC_F16X3) {
        if (B.sc.wh && B.sc.cout == B.c4.cout && B.c4.cout_pad == B.sc.cout_pad) {
          // conv(4,1) + MaxPool2D(2,'same') + the shortcut Conv2D(1x1, stride 2) of X + Add, one launch
          CHK(conv_spatial(c, B.c4, T1, T2, (int)n, h, w, &B.bn_mid, PRO_BN_ELU, EPI_BIAS, nullptr,
                           true, 0, &B.sc, X));
          std::swap(T1, T2);
        } else {
          // conv(4,1) with MaxPool2D(2,'same') fused into its epilogue -> T2 at half resolution;
          // then shortcut Conv2D(1x1, stride 2) + pooled T2
          CHK(conv_spatial(c, B.c4, T1, T2, (int)n, h, w, &B.bn_mid, PRO_BN_ELU, EPI_BIAS, nullptr,
                           true));
          CHK(conv_run(c, conv_args(B.sc, X, T1, (int)n, h, w, 2, nullptr, PRO_NONE, EPI_ADD, T2)));
        }
      } else {
        CHK(conv_spatial(c, B.c4, T1, T2, (int)n, h, w, &B.bn_mid, PRO_BN_ELU, EPI_BIAS, nullptr));
        // shortcut Conv2D(1x1, stride 2) + MaxPool2D(2, 'same')(t2), fused
        ConvArgs s = conv_args(B.sc, X, T1, (int)n, h, w, 2, nullptr, PRO_NONE, EPI_ADD_POOL, T2);
        s.hp = h;
        s.wp = w;
        CHK(conv_run(c, s));
      }
      std::swap(X, T1);
      h = (h + 1) / 2;
      w = (w + 1) / 2;
    } else {
      CHK(conv_spatial(c, B.c4, T1, X, (int)n, h, w, &B.bn_mid, PRO_BN_ELU, EPI_ADD, X));
    }
    if (stop == b + 1) {
      *tap = X;
      *tap_n = n * h * w * CH[b];
      return MMLA_OK;
    }
  }
  // h = 16, w = 19, c = 128: Lambda(K.mean(x, axis=1)) -> [n, 19, 128]
  LAUNCH(c, MMLA_STAGE_GLUE, (double)n * h * w * 128,
         mean_h_launch(X, (int)n, h, w, 128, static_cast<float*>(pseq), c->stream));
  if (stop == 10) {
    *tap = static_cast<float*>(pseq);
    *tap_n = n * w * 128;
    return MMLA_OK;
  }
  LAUNCH(c, MMLA_STAGE_LSTM, lstm_flops(n, w, 128),
         lstm_run(c, W.lstm, static_cast<float*>(pseq), n, w, static_cast<float*>(ph)));
  if (stop == 11) {
    *tap = static_cast<float*>(ph);
    *tap_n = n * 512;
    return MMLA_OK;
  }
  LAUNCH(c, MMLA_STAGE_HEAD, 2.0 * n * 512 * 2,
         od_head_launch(static_cast<float*>(ph), (int)n, W.head_w, W.head_b, probs, argmax,
                        gate.lens, gate.clip_len, gate.silent, c->stream));
  return MMLA_OK;
}

// a res unit without pooling that siu.hip runs (3xFP16 weights of the exact widths)
bool siu_ok(const SiUnit& U, int cin) {
  return U.ca.wh && U.cb.wh && siu_supported(cin) && U.ca.cin == cin && U.ca.cout == cin && U.cb.cin == cin &&
         U.cb.cout == cin && U.ca.cin_pad == cin && U.ca.cout_pad == cin && U.cb.cout_pad == cin;
}

SiuArgs siu_args(const SiUnit& U, const float* x, float* y, int64_t n, int t, int* range_flag) {
  SiuArgs s{};
  s.n = (int)n;
  s.t = t;
  s.range_flag = range_flag;
  s.x = x;
  s.y = y;
  s.wah = U.ca.wh;
  s.wal = U.ca.wl;
  s.wbh = U.cb.wh;
  s.wbl = U.cb.wl;
  s.ba = U.ca.bias;
  s.bb = U.cb.bias;
  s.s_in = U.bn_in.scale;
  s.t_in = U.bn_in.shift;
  s.s_mid = U.bn_mid.scale;
  s.t_mid = U.bn_mid.shift;
  s.ua = U.ca.unscale();
  s.ub = U.cb.unscale();
  return s;
}

// ldx: the features' row stride (39, or 40 from si_fe with a zero 40th column: the stem then stages
// 16-B aligned rows, conv_h3's float4 path, bit-identical -- its weights' padded channels are zero)
int run_si_net(mmla_ctx* c, const float* x, int64_t n, float* probs, int32_t* argmax,
               const uint8_t* silent, int ldx = SI_D) {
  const SiNet& W = c->si;
  const size_t big = (size_t)n * SI_T * 32 * sizeof(float);
  void *px, *pt1, *pt2, *pt3, *pseq, *ph, *pl;
  CHK(ws_get(c, S_X, big, &px));
  CHK(ws_get(c, S_T1, big, &pt1));
  CHK(ws_get(c, S_T2, big, &pt2));
  CHK(ws_get(c, S_T3, big, &pt3));
  CHK(ws_get(c, S_SEQ, (size_t)n * 8 * 128 * sizeof(float), &pseq));
  CHK(ws_get(c, S_HOUT, (size_t)n * 512 * sizeof(float), &ph));
  CHK(ws_get(c, S_LOGIT, (size_t)n * W.dense.cout_pad * sizeof(float), &pl));
  float* X = static_cast<float*>(px);
  float* T1 = static_cast<float*>(pt1);
  float* XP = static_cast<float*>(pt2);
  float* R = static_cast<float*>(pt3);
  int t = SI_T;
  bool fused_final = false;   // the last unit wrote BN + ReLU + AvgPool4 itself (siu FIN)
  // Conv1D(32, 4, same): [n, 256, 1, 39] -> [n, 256, 1, 32] (speaker_identification.py:195)
  ConvW stem = W.stem;
  if (ldx == SI_D + 1 && c->precision == MMLA_PREC_F16X3 && stem.wh && stem.cin_pad > SI_D) stem.cin = ldx;
  else if (ldx != SI_D) return fail(c, MMLA_E_INVALID, "padded SI features need the 3xFP16 stem");
  CHK(conv_spatial(c, stem, x, X, (int)n, t, 1, nullptr, PRO_NONE, EPI_BIAS, nullptr));
  for (int u = 0; u < 9; ++u) {   // res_unit, speaker_identification.py:168-190
    const SiUnit& U = W.unit[u];
    const int cin = U.ca.cin;
    if (POOL[u] && c->siu && c->sipu && c->precision == MMLA_PREC_F16X3 && U.ca.wh && U.cb.wh && U.sc.wh &&
        sipu_supported(cin, U.ca.cout) && U.ca.cin_pad == cin && U.ca.cout_pad == U.ca.cout &&
        U.cb.cin == U.ca.cout && U.cb.cout == U.ca.cout && U.cb.cout_pad == U.ca.cout &&
        U.sc.cin == cin && U.sc.cout == U.ca.cout && U.sc.cout_pad == U.ca.cout) {
      // the whole pool unit in one launch: MaxPool1D in the staging, t1 on chip, the shortcut in the
      // epilogue (siu.hip POOL), bit-identical to the two conv_h3 launches below
      const int tp = (t + 1) / 2;
      SiuArgs s{};
      s.x = X;
      s.y = R;
      s.wah = U.ca.wh;
      s.wal = U.ca.wl;
      s.wbh = U.cb.wh;
      s.wbl = U.cb.wl;
      s.ba = U.ca.bias;
      s.bb = U.cb.bias;
      s.s_in = U.bn_in.scale;
      s.t_in = U.bn_in.shift;
      s.s_mid = U.bn_mid.scale;
      s.t_mid = U.bn_mid.shift;
      s.ua = U.ca.unscale();
      s.ub = U.cb.unscale();
      s.n = (int)n;
      s.t = tp;
      s.t_src = t;
      s.wsh = U.sc.wh;
      s.wsl = U.sc.wl;
      s.bs = U.sc.bias;
      s.us = U.sc.unscale();
      s.range_flag = c->range_ptr;
      const int C = U.ca.cout;
      const double pool_flops = 2.0 * n * tp * (3.0 * cin * C + 3.0 * C * C + cin * C);
      // ... with the two units after it (siu.hip chain: both intermediates stay on chip)
      if (c->sichain && u + 2 < 9 && !POOL[u + 1] && !POOL[u + 2] && siu_triple_supported(cin, C) &&
          siu_ok(W.unit[u + 1], C) && siu_ok(W.unit[u + 2], C)) {
        SiuArgs sa = siu_args(W.unit[u + 1], nullptr, nullptr, n, tp, c->range_ptr);
        SiuArgs sb = siu_args(W.unit[u + 2], nullptr, R, n, tp, c->range_ptr);
        if (u + 2 == 8 && c->sifin && siu_final_supported(C) && tp % 4 == 0) {
          sb.y = nullptr;
          sb.seq = static_cast<float*>(pseq);
          sb.fs = W.final_bn.scale;
          sb.ft = W.final_bn.shift;
          fused_final = true;
        }
        s.y = nullptr;
        LAUNCH(c, MMLA_STAGE_CONV, pool_flops + 2.0 * 2.0 * 2.0 * n * tp * 3 * C * C,
               siu_triple_launch(s, sa, sb, cin, C, c->stream));
        u += 2;
      } else {
        LAUNCH(c, MMLA_STAGE_CONV, pool_flops, sipu_launch(s, cin, U.ca.cout, c->stream));
      }
      std::swap(X, R);
      t = tp;
    } else if (POOL[u]) {
      const int tp = (t + 1) / 2;
      if (c->precision == MMLA_PREC_F16X3 && U.ca.wh) {
        // MaxPool1D(2, same) taken inside the conv's staging (conv_h3.hip PIN)
        CHK(conv_spatial(c, U.ca, X, T1, (int)n, tp, 1, &U.bn_in, PRO_BN_RELU, EPI_BIAS, nullptr,
                         false, t));
      } else {
        LAUNCH(c, MMLA_STAGE_GLUE, (double)n * t * cin,
               maxpool_t2_launch(X, (int)n, t, cin, XP, c->stream));
        CHK(conv_spatial(c, U.ca, XP, T1, (int)n, tp, 1, &U.bn_in, PRO_BN_RELU, EPI_BIAS, nullptr));
      }
      if (c->precision == MMLA_PREC_F16X3 && U.cb.wh && U.sc.wh && U.sc.cout == U.cb.cout &&
          U.sc.cout_pad == U.cb.cout_pad) {
        // Conv1D(3) + the shortcut Conv1D(1, stride 2) of X as its residual + Add, one launch
        CHK(conv_spatial(c, U.cb, T1, R, (int)n, tp, 1, &U.bn_mid, PRO_BN_RELU, EPI_ADD, nullptr, false,
                         0, &U.sc, X, t));
      } else {
        CHK(conv_run(c, conv_args(U.sc, X, R, (int)n, t, 1, 2, nullptr, PRO_NONE, EPI_BIAS, nullptr)));
        CHK(conv_spatial(c, U.cb, T1, R, (int)n, tp, 1, &U.bn_mid, PRO_BN_RELU, EPI_ADD, R));
      }
      std::swap(X, R);
      t = tp;
    } else if (c->siu && c->precision == MMLA_PREC_F16X3 && siu_ok(U, cin)) {
      // the whole unit in one launch, t1 kept on chip (siu.hip), bit-identical to the pair below
      SiuArgs s = siu_args(U, X, R, n, t, c->range_ptr);
      SiuArgs s2{};
      const bool pair = c->sipair && u + 1 < 9 && !POOL[u + 1] && siu_pair_supported(cin) &&
                        siu_ok(W.unit[u + 1], cin);
      if (pair) s2 = siu_args(W.unit[u + 1], nullptr, R, n, t, c->range_ptr);
      SiuArgs& last = pair ? s2 : s;
      if (u + (pair ? 1 : 0) == 8 && c->sifin && siu_final_supported(cin) && cin == 128 && t % 4 == 0) {
        // + the final BN + ReLU + AveragePooling1D(4) in the epilogue: the unit's output never
        // reaches HBM (bit-identical to bn_relu_avgpool4_launch below)
        last.y = nullptr;
        last.seq = static_cast<float*>(pseq);
        last.fs = W.final_bn.scale;
        last.ft = W.final_bn.shift;
        fused_final = true;
      }
      if (pair) {
        s.y = nullptr;
        LAUNCH(c, MMLA_STAGE_CONV, 2.0 * 2.0 * 2.0 * n * t * 3 * cin * cin, siu_pair_launch(s, s2, cin, c->stream));
        ++u;
      } else {
        LAUNCH(c, MMLA_STAGE_CONV, 2.0 * 2.0 * n * t * 3 * cin * cin, siu_launch(s, cin, c->stream));
      }
      std::swap(X, R);
    } else {
      CHK(conv_spatial(c, U.ca, X, T1, (int)n, t, 1, &U.bn_in, PRO_BN_RELU, EPI_BIAS, nullptr));
      CHK(conv_spatial(c, U.cb, T1, X, (int)n, t, 1, &U.bn_mid, PRO_BN_RELU, EPI_ADD, X));
    }
  }
  // t = 32, c = 128 -> BN -> ReLU -> AvgPool1D(4) -> [n, 8, 128] (speaker_identification.py:208-212)
  if (!fused_final)
    LAUNCH(c, MMLA_STAGE_GLUE, 3.0 * n * t * 128,
           bn_relu_avgpool4_launch(X, (int)n, t, 128, W.final_bn.scale, W.final_bn.shift,
                                   static_cast<float*>(pseq), c->stream));
  LAUNCH(c, MMLA_STAGE_LSTM, lstm_flops(n, t / 4, 128),
         lstm_run(c, W.lstm, static_cast<float*>(pseq), n, t / 4, static_cast<float*>(ph)));
  if (c->precision == MMLA_PREC_F16X3 && W.dense.wh && W.dense.cin % 32 == 0) {
    // Dense(K) as a 1x1 conv over the clips on the 3xFP16 path (conv_h3 Conv1D tiles of 128 clips):
    // all cout_pad columns are written (the padding columns: zero weights and bias), so the logits
    // keep the cout_pad row stride the head reads
    ConvH3Args a{};
    a.x = static_cast<float*>(ph);
    a.wh = W.dense.wh;
    a.wl = W.dense.wl;
    a.unscale = W.dense.unscale();
    a.bias = W.dense.bias;
    a.y = static_cast<float*>(pl);
    a.n = (int)n;
    a.h = 1;
    a.w = 1;
    a.cin = a.cin_pad = W.dense.cin;
    a.cout = a.cout_pad = W.dense.cout_pad;
    a.kh = a.kw = 1;
    a.pro = PRO_NONE;
    a.epi = EPI_BIAS;
    a.range_flag = c->range_ptr;
    LAUNCH(c, MMLA_STAGE_HEAD, 2.0 * n * W.dense.cin * W.dense.cout, conv_h3_launch(a, c->stream));
  } else {
    ConvArgs d = conv_args(W.dense, static_cast<float*>(ph), static_cast<float*>(pl), (int)n, 1, 1, 1,
                           nullptr, PRO_NONE, EPI_BIAS, nullptr);
    d.ldy = W.dense.cout_pad;
    CHK(conv_run(c, d, MMLA_STAGE_HEAD));
  }
  LAUNCH(c, MMLA_STAGE_HEAD, 4.0 * n * W.k,
         si_head_launch(static_cast<float*>(pl), (int)n, W.k, W.dense.cout_pad, W.head, probs,
                        argmax, silent, c->stream));
  return MMLA_OK;
}

// algorithmic HBM bytes of one front-end launch: PCM actually consumed + outputs
double od_fe_bytes(int64_t n, const OdFeArgs& a) {
  const double in = a.lens ? (double)MMLA_OD_CLIP * 2 : (double)std::min(a.clip_len, MMLA_OD_CLIP) * 2;
  const double out = (a.db ? OD_PIX * 4.0 : 0) + (a.norm ? OD_PIX * 4.0 : 0) +
                     (a.zcr ? OD_W * 4.0 : 0) + (a.img ? (double)OD_IMG : 0);
  return (double)n * (in + out);
}

double si_fe_bytes(int64_t n, const SiFeArgs& a) {
  const double in = a.lens ? (double)SI_NEED_SAMPLES * 2 : (double)std::min(a.clip_len, SI_NEED_SAMPLES) * 2;
  return (double)n * (in + SI_T * SI_D * 4.0 + (a.silent ? 1.0 : 0.0));
}

bool bad_pcm_args(const int16_t* pcm, int64_t n, int64_t stride, const int32_t* lens,
                  int32_t clip_len) {
  if (n < 0 || (n > 0 && !pcm)) return true;
  if (!lens && clip_len < 0) return true;
  if (!lens && n > 1 && stride < 1) return true;   // stride < clip_len: overlapping windows
  return false;
}

}  // namespace

// ==== C ABI =========================================================================================

extern "C" {

int mmla_abi_version(void) { return MMLA_ABI_VERSION; }

// CRC-32C (Castagnoli, reflected polynomial 0x82F63B78), slice-by-8 tables built once
static uint32_t g_crc_tab[8][256];
static void crc32c_tables() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    g_crc_tab[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t) g_crc_tab[t][i] = (g_crc_tab[t - 1][i] >> 8) ^ g_crc_tab[0][g_crc_tab[t - 1][i] & 255];
}

int mmla_crc32c(const void* data, int64_t n, uint32_t* crc) {
  if ((!data && n > 0) || n < 0 || !crc) return MMLA_E_INVALID;
  static const bool ready = (crc32c_tables(), true);
  (void)ready;
  const unsigned char* p = static_cast<const unsigned char*>(data);
  uint32_t c = 0xFFFFFFFFu;
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint32_t lo, hi;
    memcpy(&lo, p + i, 4);
    memcpy(&hi, p + i + 4, 4);
    lo ^= c;
    c = g_crc_tab[7][lo & 255] ^ g_crc_tab[6][(lo >> 8) & 255] ^ g_crc_tab[5][(lo >> 16) & 255] ^
        g_crc_tab[4][lo >> 24] ^ g_crc_tab[3][hi & 255] ^ g_crc_tab[2][(hi >> 8) & 255] ^
        g_crc_tab[1][(hi >> 16) & 255] ^ g_crc_tab[0][hi >> 24];
  }
  for (; i < n; ++i) c = g_crc_tab[0][(c ^ p[i]) & 255] ^ (c >> 8);
  *crc = c ^ 0xFFFFFFFFu;
  return MMLA_OK;
}

int mmla_png_unfilter(const uint8_t* raw, int64_t h, int64_t row_bytes, int32_t bpp, uint8_t* out) {
  if (h < 0 || row_bytes < 0 || bpp < 1 || bpp > 8 || ((!raw || !out) && h * row_bytes > 0))
    return MMLA_E_INVALID;
  const uint8_t* prev = nullptr;  // row above (all zero for the first row)
  for (int64_t r = 0; r < h; ++r) {
    const uint8_t* in = raw + r * (row_bytes + 1);
    uint8_t* cur = out + r * row_bytes;
    const int ft = in[0];
    ++in;
    switch (ft) {
      case 0:
        memcpy(cur, in, (size_t)row_bytes);
        break;
      case 1:  // Sub
        for (int64_t i = 0; i < row_bytes; ++i)
          cur[i] = (uint8_t)(in[i] + (i >= bpp ? cur[i - bpp] : 0));
        break;
      case 2:  // Up
        for (int64_t i = 0; i < row_bytes; ++i) cur[i] = (uint8_t)(in[i] + (prev ? prev[i] : 0));
        break;
      case 3:  // Average (floor of the 9-bit sum)
        for (int64_t i = 0; i < row_bytes; ++i) {
          const int a = i >= bpp ? cur[i - bpp] : 0, b = prev ? prev[i] : 0;
          cur[i] = (uint8_t)(in[i] + ((a + b) >> 1));
        }
        break;
      case 4:  // Paeth
        for (int64_t i = 0; i < row_bytes; ++i) {
          const int a = i >= bpp ? cur[i - bpp] : 0, b = prev ? prev[i] : 0;
          const int c = (prev && i >= bpp) ? prev[i - bpp] : 0;
          const int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
          cur[i] = (uint8_t)(in[i] + ((pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c)));
        }
        break;
      default:
        return MMLA_E_INVALID;
    }
    prev = cur;
  }
  return MMLA_OK;
}

int mmla_create(int device, mmla_ctx** out) {
  if (!out) return MMLA_E_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return MMLA_E_HIP;
  if (device < 0 || device >= ndev) return MMLA_E_INVALID;
  if (hipSetDevice(device) != hipSuccess) return MMLA_E_HIP;
  mmla_ctx* c = new mmla_ctx();
  c->device = device;
  if (const char* fa = std::getenv("MMLA_DEBUG_FAIL_ALLOC")) c->debug_fail_allocs = std::atoi(fa);
  if (const char* su = std::getenv("MMLA_NO_SIU")) c->siu = std::atoi(su) == 0;
  if (const char* sp = std::getenv("MMLA_NO_SIPU")) c->sipu = std::atoi(sp) == 0;
  if (const char* sf = std::getenv("MMLA_NO_SIFIN")) c->sifin = std::atoi(sf) == 0;
  if (const char* sq = std::getenv("MMLA_NO_SIPAIR")) c->sipair = std::atoi(sq) == 0;
  if (const char* sc = std::getenv("MMLA_NO_SICHAIN")) c->sichain = std::atoi(sc) == 0;
  if (const char* ls = std::getenv("MMLA_NO_LSTM_SPLIT")) c->lstm_split = std::atoi(ls) == 0;
  if (const char* lm = std::getenv("MMLA_LSTM_SPLIT_MAX")) c->lstm_split_max = std::atoi(lm);
  if (const char* sp = std::getenv("MMLA_DEBUG_LSTM_SPIN")) c->lstm_spin = std::atoi(sp);
  if (const char* sd = std::getenv("MMLA_NO_SIPAD")) c->si_pad_feat = std::atoi(sd) == 0;
  if (const char* ou = std::getenv("MMLA_NO_ODU")) c->odu = std::atoi(ou) == 0;
  if (const char* rt = std::getenv("MMLA_RB_TILE")) c->rbs = std::atoi(rt) == 0;
  // a BLOCKING stream: it orders with the legacy default (NULL) stream, on which PyTorch's default
  // stream enqueues -- so a device-pointer call sees tensors a torch kernel or copy just produced
  // without an explicit synchronisation (a non-blocking stream raced them: a 65 536-clip call read
  // the last clips before torch had written them)
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamDefault) != hipSuccess) {
    delete c;
    return MMLA_E_HIP;
  }
  c->stream = c->own_stream;
  if (hipMalloc(&c->range_dev, 4 * sizeof(int)) != hipSuccess ||
      hipMemset(c->range_dev, 0, 4 * sizeof(int)) != hipSuccess ||
      hipHostMalloc(&c->range_host, 2 * sizeof(int), hipHostMallocDefault) != hipSuccess) {
    mmla_destroy(c);
    return MMLA_E_HIP;
  }
  if (const char* po = std::getenv("MMLA_NO_PIN_OUT")) c->pin_small = std::atoi(po) == 0;
  if (c->pin_small) {
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    if (hipHostMalloc(reinterpret_cast<void**>(&c->range_map), 64, fl) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&c->range_map_dev), c->range_map, 0) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&c->pin_out), kPinSlots * kPinSlotBytes, fl) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&c->pin_out_dev), c->pin_out, 0) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&c->pin_in), kPinInBytes, hipHostMallocDefault) != hipSuccess) {
      mmla_destroy(c);
      return MMLA_E_HIP;
    }
    c->range_map[0] = c->range_map[1] = 0;
  }
  OdFeTables ot;
  od_fe_build_tables(&ot);
  if (!od_fe_tables_ok(ot)) {   // the mel schedule exceeds the front-end kernel's LDS rows / fragments
    mmla_destroy(c);
    return MMLA_E_INVALID;
  }
  SiFeTables st;
  si_fe_build_tables(&st);
  if (!si_fe_tables_ok(st)) {   // filterbank segments exceed the front-end kernel's unrolled loops
    mmla_destroy(c);
    return MMLA_E_INVALID;
  }
  if (hipMalloc(&c->od_tables, sizeof(OdFeTables)) != hipSuccess ||
      hipMalloc(&c->si_tables, sizeof(SiFeTables)) != hipSuccess ||
      hipMemcpy(c->od_tables, &ot, sizeof(ot), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->si_tables, &st, sizeof(st), hipMemcpyHostToDevice) != hipSuccess) {
    mmla_destroy(c);
    return MMLA_E_HIP;
  }
  *out = c;
  return MMLA_OK;
}

int mmla_destroy(mmla_ctx* c) {
  if (!c) return MMLA_E_INVALID;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  free_allocs(c->od_allocs);
  free_allocs(c->si_allocs);
  for (size_t i = 0; i < c->ws.size(); ++i)
    if (c->ws[i]) (void)hipFree(static_cast<char*>(c->ws[i]) - c->ws_guard[i]);
  if (c->od_tables) (void)hipFree(c->od_tables);
  if (c->si_tables) (void)hipFree(c->si_tables);
  if (c->nr_tables) (void)hipFree(c->nr_tables);
  if (c->nr_thresh) (void)hipFree(c->nr_thresh);
  if (c->range_dev) (void)hipFree(c->range_dev);
  if (c->vad_state) (void)hipFree(c->vad_state);
  if (c->range_host) (void)hipHostFree(c->range_host);
  if (c->range_map) (void)hipHostFree(c->range_map);
  if (c->pin_out) (void)hipHostFree(c->pin_out);
  if (c->pin_in) (void)hipHostFree(c->pin_in);
  (void)prof_collect(c);
  for (hipEvent_t e : c->prof_pool) (void)hipEventDestroy(e);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
  return MMLA_OK;
}

// ---- stationary noise gate ----------------------------------------------------

namespace {
constexpr int64_t kNrChunk = 600000, kNrPadding = 30000;   // noisereduce 2.0 defaults
constexpr int64_t kNrItemsPerLaunch = 512;                  // ~3.4 GB of scratch per launch (2.5 s)
}  // namespace

int mmla_nr_set_noise(mmla_ctx* c, const float* noise, int64_t n_noise, int32_t sr, uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (!noise || n_noise < 2) return fail(c, MMLA_E_INVALID, "noise clip needs >= 2 samples");
  if (sr != 16000) return fail(c, MMLA_E_INVALID, "noise gate supports sr = 16000 (got %d)", sr);
  HIPCHK(c, hipSetDevice(c->device));
  const bool dev = flags & MMLA_DEVICE_PTR;
  if (!c->nr_tables) {
    NrTables t;
    nr_build_tables(&t, sr);
    if (t.ngf != NR_NGF || t.ngt != NR_NGT) return fail(c, MMLA_E_INVALID, "smoothing filter shape");
    HIPCHK(c, hipMalloc(&c->nr_tables, sizeof(NrTables)));
    HIPCHK(c, hipMalloc(&c->nr_thresh, (NR_NFFT / 2 + 1) * sizeof(float)));
    HIPCHK(c, hipMemcpy(c->nr_tables, &t, sizeof(t), hipMemcpyHostToDevice));
  }
  const int64_t m = std::min(n_noise, kNrChunk);   // clip_noise_stationary: y_noise[:chunk_size]
  const int64_t Tn = 1 + m / NR_HOP;
  const float* dn = noise;
  void *pdb = nullptr, *pmx = nullptr;
  if (!dev) {
    void* p = nullptr;
    CHK(ws_get(c, S_IN, m * sizeof(float), &p));
    HIPCHK(c, hipMemcpyAsync(p, noise, m * sizeof(float), hipMemcpyHostToDevice, c->stream));
    dn = static_cast<const float*>(p);
  }
  CHK(ws_get(c, S_NR_FRAMES, (size_t)Tn * (NR_NFFT / 2 + 1) * sizeof(float), &pdb));
  CHK(ws_get(c, S_NR_FMAX, (size_t)Tn * sizeof(float), &pmx));
  LAUNCH(c, MMLA_STAGE_NR, (double)m * 4,
         nr_noise_launch(dn, m, c->nr_tables, static_cast<float*>(pdb), static_cast<float*>(pmx),
                         1.5f, c->nr_thresh, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->nr_ready = true;
  return MMLA_OK;
}

int mmla_nr_reduce(mmla_ctx* c, const float* y, int64_t n_signals, int64_t stride, int64_t len,
                   float* out, uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (n_signals < 0 || len < 0 || (n_signals > 0 && (!y || !out)) ||
      (n_signals > 1 && stride < len))
    return fail(c, MMLA_E_INVALID, "bad nr_reduce args");
  if (!c->nr_ready) return fail(c, MMLA_E_INVALID, "mmla_nr_set_noise must be called first");
  if (n_signals == 0 || len == 0) return MMLA_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const bool dev = flags & MMLA_DEVICE_PTR;
  // SpectralGate.get_traces: one chunk of `len` when len <= chunk_size, else chunk_size pieces
  const int64_t keep = len <= kNrChunk ? len : kNrChunk;
  const int64_t per = (len + keep - 1) / keep;
  const int64_t L = keep + 2 * kNrPadding;
  const int T = (int)(1 + L / NR_HOP);
  const int64_t bins = NR_NFFT / 2 + 1;
  const int64_t cap = std::max<int64_t>(1, std::min<int64_t>(kNrItemsPerLaunch, (int64_t)(2e10 / ((double)T * (bins * 25 + NR_NFFT * 8 + 8)))));
  std::vector<NrItem> items;
  items.reserve(n_signals * per);
  for (int64_t sgl = 0; sgl < n_signals; ++sgl)
    for (int64_t k = 0; k < per; ++k)
      items.push_back(NrItem{sgl * stride, len, k * keep - kNrPadding, sgl * len + k * keep,
                             std::min(keep, len - k * keep)});
  // signals: the caller's device pointer, or one host copy per call
  const float* dy = y;
  if (!dev) {
    void* p = nullptr;
    const int64_t span = (n_signals - 1) * stride + len;
    CHK(ws_get(c, S_NR_Y, span * sizeof(float), &p));
    HIPCHK(c, hipMemcpyAsync(p, y, span * sizeof(float), hipMemcpyHostToDevice, c->stream));
    dy = static_cast<const float*>(p);
  }
  float* dout = out;
  if (!dev) {
    void* p = nullptr;
    CHK(ws_get(c, S_OUT0, (size_t)n_signals * len * sizeof(float), &p));
    dout = static_cast<float*>(p);
  }
  for (size_t i0 = 0; i0 < items.size(); i0 += cap) {
    const int64_t ni = std::min<int64_t>(cap, (int64_t)items.size() - (int64_t)i0);
    void *pS, *pB, *pM, *pF, *pI, *pR;
    CHK(ws_get(c, S_NR_S, (size_t)ni * T * bins * sizeof(double2), &pS));
    CHK(ws_get(c, S_NR_BITS, (size_t)ni * T * bins, &pB));
    CHK(ws_get(c, S_NR_FMAX, (size_t)ni * (T + 1) * sizeof(double), &pM));
    CHK(ws_get(c, S_NR_FRAMES, (size_t)ni * T * NR_NFFT * sizeof(double), &pF));
    CHK(ws_get(c, S_NR_ITEMS, (size_t)ni * sizeof(NrItem), &pI));
    CHK(ws_get(c, S_NR_ROWS, (size_t)ni * T * bins * sizeof(double), &pR));
    HIPCHK(c, hipMemcpyAsync(pI, items.data() + i0, ni * sizeof(NrItem), hipMemcpyHostToDevice,
                             c->stream));
    NrArgs a{};
    a.y = dy;
    a.items = static_cast<const NrItem*>(pI);
    a.n_items = ni;
    a.L = L;
    a.T = T;
    a.keep0 = kNrPadding;
    a.keep_len = keep;
    int t_hi = T - 1;
    nr_frame_range(items.data() + i0, ni, L, T, a.keep0, a.keep_len, &a.t_lo, &t_hi);
    a.t_n = t_hi - a.t_lo + 1;
    a.tables = c->nr_tables;
    a.thresh = c->nr_thresh;
    a.prop_decrease = 1.0;
    a.S = static_cast<double2*>(pS);
    a.bits = static_cast<uint8_t*>(pB);
    a.fmax = static_cast<double*>(pM);
    a.gmax = static_cast<double*>(pM) + ni * T;
    a.frames = static_cast<double*>(pF);
    a.rows = static_cast<double*>(pR);
    a.out = dout;
    double bytes = 0;
    for (int64_t i = 0; i < ni; ++i) bytes += 8.0 * items[i0 + i].out_len;   // f32 in + f32 out
    LAUNCH(c, MMLA_STAGE_NR, bytes, nr_gate_launch(a, c->stream));
    // the item table / scratch of this launch must not be overwritten by the next one's upload
    if (i0 + cap < items.size()) HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  CHK(copy_back(c, out, 0, dout, (size_t)n_signals * len, dev));
  return finish(c, dev);
}

const char* mmla_last_error(const mmla_ctx* c) { return c ? c->err.c_str() : "null context"; }

int mmla_set_stream(mmla_ctx* c, void* s) {
  if (!c) return MMLA_E_INVALID;
  hipStream_t ns = s ? static_cast<hipStream_t>(s) : c->own_stream;
  if (ns != c->stream) {
    // work already enqueued on the old stream still reads and writes this context's workspaces:
    // the new stream waits for it before the next call reuses them
    HIPCHK(c, hipSetDevice(c->device));
    hipEvent_t e = nullptr;
    HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const hipError_t r1 = hipEventRecord(e, c->stream);
    const hipError_t r2 = r1 == hipSuccess ? hipStreamWaitEvent(ns, e, 0) : r1;
    (void)hipEventDestroy(e);
    HIPCHK(c, r2);
  }
  c->stream = ns;
  return MMLA_OK;
}

int mmla_range_check(mmla_ctx* c, int64_t* f32_reruns) {
  if (!c) return MMLA_E_INVALID;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (f32_reruns) *f32_reruns = c->range_reruns;
  int flag = 0, timeout = 0;
  HIPCHK(c, hipMemcpy(&flag, c->range_dev, sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(&timeout, c->range_dev + 3, sizeof(int), hipMemcpyDeviceToHost));
  if (timeout) {
    HIPCHK(c, hipMemset(c->range_dev + 3, 0, sizeof(int)));
    return fail(c, MMLA_E_HIP,
                "a device-pointer call since the last check ran the split BiLSTM and one of its "
                "workgroups timed out waiting for the others: its probabilities are NaN; re-run it");
  }
  if (flag) {
    HIPCHK(c, hipMemset(c->range_dev, 0, sizeof(int)));
    return fail(c, MMLA_E_RANGE,
                "a device-pointer call since the last check split an operand outside the fp16 "
                "range (|x| >= 65504): its results are not valid; re-run it with MMLA_PREC_F32");
  }
  return MMLA_OK;
}

int mmla_debug_counters(mmla_ctx* c, int64_t* f32_reruns, int64_t* lstm_split_reruns) {
  if (!c) return MMLA_E_INVALID;
  if (f32_reruns) *f32_reruns = c->range_reruns;
  if (lstm_split_reruns) *lstm_split_reruns = c->lstm_split_reruns;
  return MMLA_OK;
}

int mmla_synchronize(mmla_ctx* c) {
  if (!c) return MMLA_E_INVALID;
  return mmla_range_check(c, nullptr);
}

int mmla_get_microbatch(mmla_ctx* c, int64_t* od_clips, int64_t* si_clips) {
  if (!c) return MMLA_E_INVALID;
  HIPCHK(c, hipSetDevice(c->device));
  if (od_clips) *od_clips = microbatch(c, true);
  if (si_clips) *si_clips = microbatch(c, false);
  return MMLA_OK;
}

int mmla_release_workspace(mmla_ctx* c) {
  if (!c) return MMLA_E_INVALID;
  HIPCHK(c, hipSetDevice(c->device));
  return ws_release(c);
}

int mmla_set_precision(mmla_ctx* c, int mode) {
  if (!c || (mode != MMLA_PREC_F32 && mode != MMLA_PREC_F16X3)) return MMLA_E_INVALID;
  c->precision = mode;
  return MMLA_OK;
}

int mmla_set_microbatch(mmla_ctx* c, int64_t od, int64_t si) {
  if (!c || od < 0 || si < 0) return MMLA_E_INVALID;
  c->od_mb = od;   // 0 = sized from free memory (mmla.h)
  c->si_mb = si;
  c->od_mb_cap = kOdMicrobatch;
  c->si_mb_cap = kSiMicrobatch;
  return MMLA_OK;
}

int mmla_load_weights(mmla_ctx* c, int kind, const float* packed, int64_t n_floats,
                      int32_t n_classes, int32_t head) {
  if (!c) return MMLA_E_INVALID;
  if (!packed || n_floats <= 0) return fail(c, MMLA_E_INVALID, "null weight blob");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  Cursor cur{packed, n_floats};
  c->loading_f16_bad = false;
  if (kind == MMLA_MODEL_OD) {
    if (n_classes != 2) return fail(c, MMLA_E_INVALID, "OD model has 2 classes, got %d", n_classes);
    free_allocs(c->od_allocs);
    c->od_loaded = false;
    OdNet& W = c->od;
    auto& al = c->od_allocs;
    CHK(take_conv(c, cur, al, 1, 1, 3, 16, &W.stem));
    int cin = 16;
    for (int b = 0; b < 9; ++b) {
      const int ch = CH[b];
      CHK(take_bn(c, cur, al, cin, &W.blk[b].bn_in));
      CHK(take_conv(c, cur, al, 3, 3, cin, ch, &W.blk[b].c3));
      CHK(take_bn(c, cur, al, ch, &W.blk[b].bn_mid));
      CHK(take_conv(c, cur, al, 4, 1, ch, ch, &W.blk[b].c4));
      if (POOL[b]) CHK(take_conv(c, cur, al, 1, 1, cin, ch, &W.blk[b].sc));
      cin = ch;
    }
    CHK(take_lstm(c, cur, al, 128, &W.lstm));
    const float* hw = cur.take(512 * 2);
    const float* hb = cur.take(2);
    if (!cur.ok) return fail(c, MMLA_E_SHAPE, "OD weight blob too short");
    CHK(upload(c, al, hw, 512 * 2 * sizeof(float), &W.head_w));
    CHK(upload(c, al, hb, 2 * sizeof(float), &W.head_b));
    if (cur.left != 0)
      return fail(c, MMLA_E_SHAPE, "OD weight blob has %lld extra floats", (long long)cur.left);
    c->od_f32_only = c->loading_f16_bad;   // some weight outside the fp16 range: exact f32 only
    c->od_loaded = true;
    return MMLA_OK;
  }
  if (kind == MMLA_MODEL_SI) {
    if (n_classes < 1) return fail(c, MMLA_E_INVALID, "SI n_classes must be >= 1");
    if (head != MMLA_HEAD_SOFTMAX && head != MMLA_HEAD_SIGMOID)
      return fail(c, MMLA_E_INVALID, "unknown head %d", head);
    free_allocs(c->si_allocs);
    c->si_loaded = false;
    SiNet& W = c->si;
    auto& al = c->si_allocs;
    CHK(take_conv(c, cur, al, 4, 1, 39, 32, &W.stem));
    int cin = 32;
    for (int u = 0; u < 9; ++u) {
      const int ch = CH[u];
      CHK(take_bn(c, cur, al, cin, &W.unit[u].bn_in));
      CHK(take_conv(c, cur, al, 3, 1, cin, ch, &W.unit[u].ca));
      CHK(take_bn(c, cur, al, ch, &W.unit[u].bn_mid));
      if (POOL[u]) CHK(take_conv(c, cur, al, 1, 1, cin, ch, &W.unit[u].sc));
      CHK(take_conv(c, cur, al, 3, 1, ch, ch, &W.unit[u].cb));
      cin = ch;
    }
    CHK(take_bn(c, cur, al, 128, &W.final_bn));
    CHK(take_lstm(c, cur, al, 128, &W.lstm));
    CHK(take_conv(c, cur, al, 1, 1, 512, n_classes, &W.dense));
    if (cur.left != 0)
      return fail(c, MMLA_E_SHAPE, "SI weight blob has %lld extra floats", (long long)cur.left);
    W.k = n_classes;
    W.head = head;
    c->si_f32_only = c->loading_f16_bad;
    c->si_loaded = true;
    return MMLA_OK;
  }
  return fail(c, MMLA_E_INVALID, "unknown model kind %d", kind);
}

}  // extern "C"

template <typename T>
static int od_features_common(mmla_ctx* c, const T* pcm, int64_t n, int64_t stride,
                              const int32_t* lens, int32_t clip_len, float* db, float* norm,
                              float* zcr, uint8_t* img, uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (bad_pcm_args(reinterpret_cast<const int16_t*>(pcm), n, stride, lens, clip_len))
    return fail(c, MMLA_E_INVALID, "bad pcm args");
  HIPCHK(c, hipSetDevice(c->device));
  const bool dev = flags & MMLA_DEVICE_PTR;
  // float PCM: the front-end splits y 2^3 into fp16 hi + lo, so the kernel checks every sample it
  // reads (the first min(len, 24000) of each clip) into a range word: device-pointer calls into the
  // sticky word (mmla_range_check / mmla_synchronize report it), host-pointer calls into their own
  // word, read after the micro-batch's synchronisation; only then is the micro-batch re-scanned on
  // the host, to name the first offending sample
  auto host_range_error = [&](int64_t c0, int64_t cnt) -> int {
    if constexpr (std::is_same<T, float>::value) {
      for (int64_t i = c0; i < c0 + cnt; ++i) {
        const int64_t len = std::min<int64_t>(lens ? lens[i] : clip_len, MMLA_OD_CLIP);
        for (int64_t j = 0; j < len; ++j)
          if (!(std::fabs(pcm[i * stride + j]) < 8188.0f))
            return fail(c, MMLA_E_RANGE,
                        "float PCM clip %lld sample %lld = %g: the front-end needs |y| < 8188 (y * 8 is "
                        "split into fp16)", (long long)i, (long long)j, (double)pcm[i * stride + j]);
      }
    }
    return fail(c, MMLA_E_RANGE, "float PCM outside |y| < 8188 in clips %lld..%lld", (long long)c0,
                (long long)(c0 + cnt - 1));
  };
  auto body = [&](int64_t c0, int64_t cnt) -> int {
    PcmT<T> p;
    CHK(stage_pcm(c, pcm, c0, cnt, stride, lens, clip_len, MMLA_OD_CLIP, dev, &p));
    OdFeArgs a{};
    if constexpr (std::is_same<T, float>::value) {
      a.pcm_f32 = p.p;
      a.range_flag = dev ? c->range_dev : c->range_dev + 1;
      if (!dev) HIPCHK(c, hipMemsetAsync(a.range_flag, 0, sizeof(int), c->stream));
    } else {
      a.pcm = p.p;
    }
    a.clip_stride = p.stride;
    a.lens = p.lens;
    a.clip_len = p.clip_len;
    a.tables = c->od_tables;
    CHK(out_ptr(c, db, c0 * OD_PIX, cnt * OD_PIX, dev, S_OUT0, &a.db));
    CHK(out_ptr(c, norm, c0 * OD_PIX, cnt * OD_PIX, dev, S_OUT1, &a.norm));
    CHK(out_ptr(c, zcr, c0 * OD_W, cnt * OD_W, dev, S_OUT2, &a.zcr));
    CHK(out_ptr(c, img, c0 * OD_IMG, cnt * OD_IMG, dev, S_OUT3, &a.img));
    LAUNCH(c, MMLA_STAGE_OD_FE, od_fe_bytes(cnt, a), od_fe_launch(a, cnt, c->stream));
    CHK(copy_back(c, db, c0 * OD_PIX, a.db, cnt * OD_PIX, dev));
    CHK(copy_back(c, norm, c0 * OD_PIX, a.norm, cnt * OD_PIX, dev));
    CHK(copy_back(c, zcr, c0 * OD_W, a.zcr, cnt * OD_W, dev));
    CHK(copy_back(c, img, c0 * OD_IMG, a.img, cnt * OD_IMG, dev));
    if (!dev) HIPCHK(c, hipStreamSynchronize(c->stream));
    if (std::is_same<T, float>::value && !dev) {
      int flag = 0;
      HIPCHK(c, hipMemcpy(&flag, c->range_dev + 1, sizeof(int), hipMemcpyDeviceToHost));
      if (flag) return host_range_error(c0, cnt);
    }
    return MMLA_OK;
  };
  if (dev) {   // one launch over the caller's device buffers
    if (n > 0) CHK(body(0, n));
  } else {
    CHK(for_microbatches(c, true, n, body));
  }
  return finish(c, dev);
}

extern "C" {

int mmla_od_features(mmla_ctx* c, const int16_t* pcm, int64_t n, int64_t stride,
                     const int32_t* lens, int32_t clip_len, float* db, float* norm, float* zcr,
                     uint8_t* img, uint32_t flags) {
  return od_features_common(c, pcm, n, stride, lens, clip_len, db, norm, zcr, img, flags);
}

int mmla_od_features_f32(mmla_ctx* c, const float* y, int64_t n, int64_t stride,
                         const int32_t* lens, int32_t clip_len, float* db, float* norm, float* zcr,
                         uint8_t* img, uint32_t flags) {
  return od_features_common(c, y, n, stride, lens, clip_len, db, norm, zcr, img, flags);
}

int mmla_si_features(mmla_ctx* c, const int16_t* pcm, int64_t n, int64_t stride,
                     const int32_t* lens, int32_t clip_len, float* feat, uint8_t* silent,
                     uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (bad_pcm_args(pcm, n, stride, lens, clip_len) || (n > 0 && !feat))
    return fail(c, MMLA_E_INVALID, "bad pcm/feat args");
  HIPCHK(c, hipSetDevice(c->device));
  const bool dev = flags & MMLA_DEVICE_PTR;
  auto body = [&](int64_t c0, int64_t cnt) -> int {
    Pcm p;
    CHK(stage_pcm(c, pcm, c0, cnt, stride, lens, clip_len, SI_NEED_SAMPLES, dev, &p));
    SiFeArgs a{};
    a.pcm = p.p;
    a.clip_stride = p.stride;
    a.lens = p.lens;
    a.clip_len = lens ? 0 : clip_len;   // true length decides T even if fewer samples are staged
    a.tables = c->si_tables;
    CHK(out_ptr(c, feat, c0 * SI_T * SI_D, cnt * SI_T * SI_D, dev, S_OUT0, &a.feat));
    CHK(out_ptr(c, silent, c0, cnt, dev, S_OUT1, &a.silent));
    LAUNCH(c, MMLA_STAGE_SI_FE, si_fe_bytes(cnt, a), si_fe_launch(a, cnt, c->stream));
    CHK(copy_back(c, feat, c0 * SI_T * SI_D, a.feat, cnt * SI_T * SI_D, dev));
    CHK(copy_back(c, silent, c0, a.silent, cnt, dev));
    if (!dev) HIPCHK(c, hipStreamSynchronize(c->stream));
    return MMLA_OK;
  };
  if (dev) {
    if (n > 0) CHK(body(0, n));
  } else {
    CHK(for_microbatches(c, false, n, body));
  }
  return finish(c, dev);
}

int mmla_si_features_seq(mmla_ctx* c, const int16_t* pcm, int64_t n_samples, int64_t n_windows,
                         float* feat, uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (n_samples < 1 || !pcm || !feat) return fail(c, MMLA_E_INVALID, "bad si_features_seq args");
  const int64_t T = n_samples <= 400 ? 1 : 1 + (n_samples - 400 + 159) / 160;
  if (n_windows != (T + SI_T - 1) / SI_T)
    return fail(c, MMLA_E_INVALID, "n_windows must be ceil(T/256) = %lld", (long long)((T + 255) / 256));
  HIPCHK(c, hipSetDevice(c->device));
  const bool dev = flags & MMLA_DEVICE_PTR;
  const int16_t* dp = pcm;
  if (!dev) {
    void* p = nullptr;
    CHK(ws_get(c, S_PCM, n_samples * sizeof(int16_t), &p));
    HIPCHK(c, hipMemcpyAsync(p, pcm, n_samples * sizeof(int16_t), hipMemcpyHostToDevice, c->stream));
    dp = static_cast<int16_t*>(p);
  }
  SiFeArgs a{};
  a.pcm = dp;
  a.seq_len = n_samples;
  a.tables = c->si_tables;
  CHK(out_ptr(c, feat, 0, n_windows * SI_T * SI_D, dev, S_OUT0, &a.feat));
  LAUNCH(c, MMLA_STAGE_SI_FE, (double)n_samples * 2 + (double)n_windows * SI_T * SI_D * 4,
         si_fe_launch(a, n_windows, c->stream));
  CHK(copy_back(c, feat, 0, a.feat, n_windows * SI_T * SI_D, dev));
  return finish(c, dev);
}

// OD-NET over float NHWC (x_f32) or uint8 (x_u8) images
static int od_forward_common(mmla_ctx* c, const float* x_f32, const uint8_t* x_u8, int64_t n, float* probs,
                      uint32_t flags) {
  if (n < 0 || (n > 0 && ((!x_f32 && !x_u8) || !probs)))
    return fail(c, MMLA_E_INVALID, "bad od_forward args");
  if (!c->od_loaded) return fail(c, MMLA_E_NOWEIGHTS, "OD weights not loaded");
  HIPCHK(c, hipSetDevice(c->device));
  const bool dev = flags & MMLA_DEVICE_PTR;
  CHK(for_microbatches(c, true, n, [&](int64_t c0, int64_t cnt) -> int {
    return guarded(c, dev, c->od_f32_only, [&]() -> int {
      const float* df = x_f32 ? x_f32 + c0 * OD_IMG : nullptr;
      const uint8_t* du = x_u8 ? x_u8 + c0 * OD_IMG : nullptr;
      if (!dev) {
        void* p = nullptr;
        const size_t bytes = cnt * OD_IMG * (x_f32 ? sizeof(float) : 1);
        CHK(ws_get(c, x_f32 ? S_IN : S_IMG, bytes, &p));
        HIPCHK(c, hipMemcpyAsync(p, x_f32 ? (const void*)df : (const void*)du, bytes,
                                 hipMemcpyHostToDevice, c->stream));
        if (x_f32) df = static_cast<float*>(p);
        else du = static_cast<uint8_t*>(p);
      }
      float* dp;
      CHK(out_ptr(c, probs, c0 * 2, cnt * 2, dev, S_OUT0, &dp));
      CHK(run_od_net(c, du, df, cnt, dp, nullptr));
      CHK(copy_back(c, probs, c0 * 2, dp, cnt * 2, dev));
      if (!dev) HIPCHK(c, hipStreamSynchronize(c->stream));
      return MMLA_OK;
    });
  }));
  return finish(c, dev);
}

int mmla_od_forward(mmla_ctx* c, const float* x, int64_t n, float* probs, uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (n > 0 && !x) return fail(c, MMLA_E_INVALID, "bad od_forward args");
  return od_forward_common(c, x, nullptr, n, probs, flags);
}

int mmla_od_forward_u8(mmla_ctx* c, const uint8_t* img, int64_t n, float* probs, uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (n > 0 && !img) return fail(c, MMLA_E_INVALID, "bad od_forward args");
  return od_forward_common(c, nullptr, img, n, probs, flags);
}

int mmla_si_forward(mmla_ctx* c, const float* x, int64_t n, float* probs, uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (n < 0 || (n > 0 && (!x || !probs))) return fail(c, MMLA_E_INVALID, "bad si_forward args");
  if (!c->si_loaded) return fail(c, MMLA_E_NOWEIGHTS, "SI weights not loaded");
  HIPCHK(c, hipSetDevice(c->device));
  const bool dev = flags & MMLA_DEVICE_PTR;
  const int k = c->si.k;
  CHK(for_microbatches(c, false, n, [&](int64_t c0, int64_t cnt) -> int {
    return guarded(c, dev, c->si_f32_only, [&]() -> int {
      const float* dx = x + c0 * SI_T * SI_D;
      if (!dev) {
        void* p = nullptr;
        CHK(ws_get(c, S_IN, cnt * SI_T * SI_D * sizeof(float), &p));
        HIPCHK(c, hipMemcpyAsync(p, dx, cnt * SI_T * SI_D * sizeof(float), hipMemcpyHostToDevice,
                                 c->stream));
        dx = static_cast<float*>(p);
      }
      float* dp;
      CHK(out_ptr(c, probs, c0 * k, cnt * k, dev, S_OUT0, &dp));
      CHK(run_si_net(c, dx, cnt, dp, nullptr, nullptr));
      CHK(copy_back(c, probs, c0 * k, dp, cnt * k, dev));
      if (!dev) HIPCHK(c, hipStreamSynchronize(c->stream));
      return MMLA_OK;
    });
  }));
  return finish(c, dev);
}

int mmla_od_pipeline(mmla_ctx* c, const int16_t* pcm, int64_t n, int64_t stride,
                     const int32_t* lens, int32_t clip_len, float* probs, int32_t* argmax,
                     uint8_t* silent, uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (bad_pcm_args(pcm, n, stride, lens, clip_len)) return fail(c, MMLA_E_INVALID, "bad pcm args");
  if (!c->od_loaded) return fail(c, MMLA_E_NOWEIGHTS, "OD weights not loaded");
  HIPCHK(c, hipSetDevice(c->device));
  const bool dev = flags & MMLA_DEVICE_PTR;
  CHK(for_microbatches(c, true, n, [&](int64_t c0, int64_t cnt) -> int {
    return guarded(c, dev, c->od_f32_only, [&]() -> int {
      Pcm p;
      CHK(stage_pcm(c, pcm, c0, cnt, stride, lens, clip_len, MMLA_OD_CLIP, dev, &p));
      void* pimg = nullptr;
      CHK(ws_get(c, S_IMG, cnt * OD_IMG, &pimg));
      OdFeArgs a{};
      a.pcm = p.p;
      a.clip_stride = p.stride;
      a.lens = p.lens;
      a.clip_len = p.clip_len;
      a.tables = c->od_tables;
      a.img = static_cast<uint8_t*>(pimg);
      LAUNCH(c, MMLA_STAGE_OD_FE, od_fe_bytes(cnt, a), od_fe_launch(a, cnt, c->stream));
      float* dp;
      int32_t* da;
      uint8_t* ds;
      CHK(out_ptr(c, probs, c0 * 2, cnt * 2, dev, S_OUT0, &dp));
      CHK(out_ptr(c, argmax, c0, cnt, dev, S_OUT1, &da));
      CHK(out_ptr(c, silent, c0, cnt, dev, S_OUT2, &ds));
      OdGate g;
      g.lens = p.lens;
      g.clip_len = lens ? 0 : clip_len;   // the true length decides, not the staged width
      g.silent = ds;
      CHK(run_od_net(c, a.img, nullptr, cnt, dp, da, g));
      CHK(copy_back(c, probs, c0 * 2, dp, cnt * 2, dev));
      CHK(copy_back(c, argmax, c0, da, cnt, dev));
      CHK(copy_back(c, silent, c0, ds, cnt, dev));
      if (!dev) HIPCHK(c, hipStreamSynchronize(c->stream));
      return MMLA_OK;
    });
  }));
  return finish(c, dev);
}

int mmla_si_pipeline(mmla_ctx* c, const int16_t* pcm, int64_t n, int64_t stride,
                     const int32_t* lens, int32_t clip_len, float* probs, int32_t* argmax,
                     uint8_t* silent, uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (bad_pcm_args(pcm, n, stride, lens, clip_len)) return fail(c, MMLA_E_INVALID, "bad pcm args");
  if (!c->si_loaded) return fail(c, MMLA_E_NOWEIGHTS, "SI weights not loaded");
  HIPCHK(c, hipSetDevice(c->device));
  const bool dev = flags & MMLA_DEVICE_PTR;
  const int k = c->si.k;
  CHK(for_microbatches(c, false, n, [&](int64_t c0, int64_t cnt) -> int {
    return guarded(c, dev, c->si_f32_only, [&]() -> int {
      Pcm p;
      CHK(stage_pcm(c, pcm, c0, cnt, stride, lens, clip_len, SI_NEED_SAMPLES, dev, &p));
      void *pf, *ps;
      // the features stay on the device: rows of 40 floats when the 3xFP16 stem reads them
      const int ldf = c->precision == MMLA_PREC_F16X3 && c->si.stem.wh && c->si.stem.cin_pad > SI_D &&
                              c->si_pad_feat ? SI_D + 1 : SI_D;
      CHK(ws_get(c, S_FEAT, cnt * SI_T * ldf * sizeof(float), &pf));
      uint8_t* pso = nullptr;   // host mode: the caller's 'silent' flags through an output slot
      if (!dev && silent) CHK(out_ptr(c, silent, c0, cnt, dev, S_OUT2, &pso));
      if (pso)
        ps = pso;
      else
        CHK(ws_get(c, S_SILENT, cnt, &ps));
      SiFeArgs a{};
      a.pcm = p.p;
      a.clip_stride = p.stride;
      a.lens = p.lens;
      a.clip_len = lens ? 0 : clip_len;
      a.tables = c->si_tables;
      a.feat = static_cast<float*>(pf);
      a.ldf = ldf;
      a.silent = static_cast<uint8_t*>(ps);
      LAUNCH(c, MMLA_STAGE_SI_FE, si_fe_bytes(cnt, a), si_fe_launch(a, cnt, c->stream));
      float* dp;
      int32_t* da;
      CHK(out_ptr(c, probs, c0 * k, cnt * k, dev, S_OUT0, &dp));
      CHK(out_ptr(c, argmax, c0, cnt, dev, S_OUT1, &da));
      CHK(run_si_net(c, a.feat, cnt, dp, da, a.silent, ldf));
      CHK(copy_back(c, probs, c0 * k, dp, cnt * k, dev));
      CHK(copy_back(c, argmax, c0, da, cnt, dev));
      if (silent) {
        if (dev)
          HIPCHK(c, hipMemcpyAsync(silent + c0, a.silent, cnt, hipMemcpyDeviceToDevice, c->stream));
        else
          CHK(copy_back(c, silent, c0, pso, cnt, dev));
      }
      if (!dev) HIPCHK(c, hipStreamSynchronize(c->stream));
      return MMLA_OK;
    });
  }));
  return finish(c, dev);
}

// ---- silence removal: webrtcvad + vad_collector, soundfile PCM_16 ------------

int mmla_vad_reset(mmla_ctx* c, int64_t n_streams, int32_t mode) {
  if (!c) return MMLA_E_INVALID;
  if (n_streams < 1) return fail(c, MMLA_E_INVALID, "n_streams must be >= 1");
  VadState init;
  if (!vad_init_state(&init, mode)) return fail(c, MMLA_E_INVALID, "VAD mode must be 0..3, got %d", mode);
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->vad_state) HIPCHK(c, hipFree(c->vad_state));
  c->vad_state = nullptr;
  c->vad_streams = 0;
  if (hipMalloc(&c->vad_state, n_streams * sizeof(VadState)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(c, MMLA_E_OOM, "VAD state for %lld streams", (long long)n_streams);
  }
  std::vector<VadState> h(n_streams, init);
  HIPCHK(c, hipMemcpy(c->vad_state, h.data(), n_streams * sizeof(VadState), hipMemcpyHostToDevice));
  c->vad_streams = n_streams;
  return MMLA_OK;
}

// shared body: speech == nullptr -> decisions from the context's VAD states, else the caller's
static int vad_run(mmla_ctx* c, const int16_t* pcm, int64_t n, int64_t stride, const int32_t* lens,
                   int32_t clip_len, int64_t items_per_stream, const uint8_t* speech_in,
                   uint8_t* speech_out, int32_t max_frames, int16_t* out, int32_t* out_lens,
                   uint32_t flags) {
  if (n < 0 || (n > 0 && (!pcm || !out || !out_lens)) || (!lens && clip_len < 0) ||
      (n > 1 && stride < (lens ? 1 : clip_len)) || (n > 0 && lens && stride < 1))
    return fail(c, MMLA_E_INVALID, "bad VAD args");
  if (n == 0) return MMLA_OK;
  // with lens the row width is the stride: an item longer than its row would read the next item
  // and its rewrite would run past the output; device-pointer lens are clamped in the
  // kernels instead
  if (lens && !(flags & MMLA_DEVICE_PTR))
    for (int64_t i = 0; i < n; ++i)
      if (lens[i] > stride)
        return fail(c, MMLA_E_INVALID, "lens[%lld] = %d exceeds the row width (stride %lld)",
                    (long long)i, lens[i], (long long)stride);
  const int64_t width = lens ? stride : std::max<int64_t>(clip_len, 1);
  if (max_frames <= 0) max_frames = std::max(1, vad_frames(width));
  if (max_frames > 4096) return fail(c, MMLA_E_INVALID, "more than 4096 frames (2 min) per item");
  HIPCHK(c, hipSetDevice(c->device));
  const bool dev = flags & MMLA_DEVICE_PTR;
  VadArgs a{};
  a.stride = n > 1 ? stride : width;
  a.clip_len = clip_len;
  a.n_items = n;
  a.items_per_stream = items_per_stream;
  a.max_frames = max_frames;
  a.state = c->vad_state;
  const size_t samples = (size_t)(n - 1) * a.stride + width;
  a.pcm = pcm;
  a.lens = lens;
  if (!dev) {
    void *pp = nullptr, *pl = nullptr;
    CHK(ws_get(c, S_PCM, samples * sizeof(int16_t), &pp));
    HIPCHK(c, hipMemcpyAsync(pp, pcm, samples * sizeof(int16_t), hipMemcpyHostToDevice, c->stream));
    a.pcm = static_cast<int16_t*>(pp);
    if (lens) {
      CHK(ws_get(c, S_LENS, n * sizeof(int32_t), &pl));
      HIPCHK(c, hipMemcpyAsync(pl, lens, n * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
      a.lens = static_cast<int32_t*>(pl);
    }
  }
  void* ps = nullptr;
  const size_t sbytes = (size_t)n * max_frames;
  if (speech_in && dev) {
    a.speech = const_cast<uint8_t*>(speech_in);
  } else if (speech_out && dev) {
    a.speech = speech_out;
  } else {
    CHK(ws_get(c, S_VAD_SPEECH, sbytes, &ps));
    a.speech = static_cast<uint8_t*>(ps);
    if (speech_in) HIPCHK(c, hipMemcpyAsync(ps, speech_in, sbytes, hipMemcpyHostToDevice, c->stream));
  }
  CHK(out_ptr(c, out, 0, samples, dev, S_VAD_OUT, &a.out));
  CHK(out_ptr(c, out_lens, 0, n, dev, S_VAD_LENS, &a.out_lens));
  if (!speech_in) {
    if (!c->vad_state) return fail(c, MMLA_E_INVALID, "mmla_vad_reset must be called first");
    if (items_per_stream < 1 || n % items_per_stream || n / items_per_stream != c->vad_streams)
      return fail(c, MMLA_E_INVALID, "%lld items are not %lld streams x items_per_stream %lld",
                  (long long)n, (long long)c->vad_streams, (long long)items_per_stream);
    // the rewrite keeps a frame's bytes or drops it: outputs are never longer than inputs
    LAUNCH(c, MMLA_STAGE_GLUE, (double)n * width, vad_speech_launch(a, c->stream));
  }
  LAUNCH(c, MMLA_STAGE_GLUE, (double)n * width, vad_collect_launch(a, c->stream));
  CHK(copy_back(c, out, 0, a.out, samples, dev));
  CHK(copy_back(c, out_lens, 0, a.out_lens, n, dev));
  if (speech_out && !dev)
    HIPCHK(c, hipMemcpyAsync(speech_out, a.speech, sbytes, hipMemcpyDeviceToHost, c->stream));
  return finish(c, dev);
}

int mmla_vad_remove_silence(mmla_ctx* c, const int16_t* pcm, int64_t n_items, int64_t stride,
                            const int32_t* lens, int32_t clip_len, int64_t items_per_stream,
                            int16_t* out, int32_t* out_lens, uint8_t* speech, int32_t max_frames,
                            uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  return vad_run(c, pcm, n_items, stride, lens, clip_len, items_per_stream, nullptr, speech,
                 max_frames, out, out_lens, flags);
}

int mmla_vad_collect(mmla_ctx* c, const int16_t* pcm, int64_t n_items, int64_t stride,
                     const int32_t* lens, int32_t clip_len, const uint8_t* speech, int32_t max_frames,
                     int16_t* out, int32_t* out_lens, uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (n_items > 0 && !speech) return fail(c, MMLA_E_INVALID, "speech flags required");
  return vad_run(c, pcm, n_items, stride, lens, clip_len, 1, speech, nullptr, max_frames, out,
                 out_lens, flags);
}

int mmla_pcm16(mmla_ctx* c, const float* y, int64_t n, int16_t* out, uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (n < 0 || (n > 0 && (!y || !out))) return fail(c, MMLA_E_INVALID, "bad pcm16 args");
  if (n == 0) return MMLA_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const bool dev = flags & MMLA_DEVICE_PTR;
  const float* dy = y;
  if (!dev) {
    void* p = nullptr;
    CHK(ws_get(c, S_IN, n * sizeof(float), &p));
    HIPCHK(c, hipMemcpyAsync(p, y, n * sizeof(float), hipMemcpyHostToDevice, c->stream));
    dy = static_cast<float*>(p);
  }
  int16_t* d;
  CHK(out_ptr(c, out, 0, n, dev, S_VAD_OUT, &d));
  LAUNCH(c, MMLA_STAGE_GLUE, (double)n * 6, pcm16_launch(dy, n, d, c->stream));
  CHK(copy_back(c, out, 0, d, n, dev));
  return finish(c, dev);
}

// ---- rate conversion of the offline pre-conditioning (resample.hip) ------------------------------

int mmla_ratecv(mmla_ctx* c, const int16_t* pcm, int64_t n_frames, int32_t nch, int32_t inrate,
                int32_t outrate, int16_t* out, int64_t out_frames, uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (n_frames < 0 || nch < 1 || nch > 64 || inrate < 1 || outrate < 1 ||
      (n_frames > 0 && (!pcm || !out)))
    return fail(c, MMLA_E_INVALID, "bad ratecv args");
  const int g = std::gcd(inrate, outrate);
  const int64_t ir = inrate / g, orr = outrate / g;
  const int64_t want = n_frames > 0 ? (n_frames - 1) * orr / ir + 1 : 0;
  if (out_frames != want)
    return fail(c, MMLA_E_INVALID, "ratecv of %lld frames %d -> %d Hz gives %lld frames, not %lld",
                (long long)n_frames, inrate, outrate, (long long)want, (long long)out_frames);
  if (n_frames == 0) return MMLA_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const bool dev = flags & MMLA_DEVICE_PTR;
  const int16_t* din = pcm;
  if (!dev) {
    void* p = nullptr;
    CHK(ws_get(c, S_PCM, (size_t)n_frames * nch * sizeof(int16_t), &p));
    HIPCHK(c, hipMemcpyAsync(p, pcm, (size_t)n_frames * nch * sizeof(int16_t), hipMemcpyHostToDevice,
                             c->stream));
    din = static_cast<const int16_t*>(p);
  }
  int16_t* d;
  CHK(out_ptr(c, out, 0, (size_t)want * nch, dev, S_VAD_OUT, &d));
  LAUNCH(c, MMLA_STAGE_GLUE, 2.0 * nch * (double)(n_frames + want),
         ratecv_launch(din, n_frames, nch, (int)ir, (int)orr, d, want, c->stream));
  CHK(copy_back(c, out, 0, d, (size_t)want * nch, dev));
  return finish(c, dev);
}

int mmla_resample_sinc(mmla_ctx* c, const float* x, int64_t n, int32_t sr_orig, int32_t sr_new,
                       const double* half_window, int64_t window_len, int32_t num_table, float* y,
                       int64_t n_out, uint32_t flags) {
  if (!c) return MMLA_E_INVALID;
  if (n < 0 || sr_orig < 1 || sr_new < 1 || window_len < 2 || num_table < 1 || !half_window ||
      (n > 0 && (!x || !y)))
    return fail(c, MMLA_E_INVALID, "bad resample args");
  const double ratio = (double)sr_new / (double)sr_orig;
  const int64_t want = (int64_t)((double)n * ratio);      // resampy: int(n * sample_ratio)
  if (n_out != want)
    return fail(c, MMLA_E_INVALID, "resampling %lld samples %d -> %d Hz gives %lld, not %lld",
                (long long)n, sr_orig, sr_new, (long long)want, (long long)n_out);
  if (n_out == 0) return MMLA_OK;
  const double scale = std::min(1.0, ratio);
  const int index_step = (int)(scale * num_table);
  if (index_step < 1) return fail(c, MMLA_E_INVALID, "ratio %g too small for the filter table", ratio);
  HIPCHK(c, hipSetDevice(c->device));
  const bool dev = flags & MMLA_DEVICE_PTR;
  // the filter as resampy prepares it: scaled by the ratio when downsampling, then its forward
  // difference (last entry 0), interleaved (win, delta) for one 16-B load per tap
  std::vector<double> wd(2 * window_len);
  for (int64_t i = 0; i < window_len; ++i) wd[2 * i] = ratio < 1 ? half_window[i] * ratio : half_window[i];
  for (int64_t i = 0; i < window_len; ++i)
    wd[2 * i + 1] = i + 1 < window_len ? wd[2 * i + 2] - wd[2 * i] : 0.0;
  // the time register of the sequential loop: repeated float64 addition of 1 / ratio
  std::vector<double> tr(n_out);
  const double inc = 1.0 / ratio;
  double t_reg = 0.0;
  for (int64_t t = 0; t < n_out; ++t) {
    tr[t] = t_reg;
    t_reg += inc;
  }
  void *ptr = nullptr, *pw = nullptr;
  CHK(ws_get(c, S_RS_TR, (size_t)n_out * sizeof(double), &ptr));
  CHK(ws_get(c, S_RS_WIN, wd.size() * sizeof(double), &pw));
  HIPCHK(c, hipMemcpyAsync(ptr, tr.data(), (size_t)n_out * sizeof(double), hipMemcpyHostToDevice,
                           c->stream));
  HIPCHK(c, hipMemcpyAsync(pw, wd.data(), wd.size() * sizeof(double), hipMemcpyHostToDevice, c->stream));
  const float* dx = x;
  if (!dev) {
    void* p = nullptr;
    CHK(ws_get(c, S_IN, (size_t)n * sizeof(float), &p));
    HIPCHK(c, hipMemcpyAsync(p, x, (size_t)n * sizeof(float), hipMemcpyHostToDevice, c->stream));
    dx = static_cast<const float*>(p);
  }
  SincResampleArgs a{};
  a.x = dx;
  a.n_orig = n;
  a.tr = static_cast<const double*>(ptr);
  a.win = static_cast<const double*>(pw);
  a.nwin = window_len;
  a.num_table = num_table;
  a.index_step = index_step;
  a.scale = scale;
  a.n_out = n_out;
  CHK(out_ptr(c, y, 0, (size_t)n_out, dev, S_OUT0, &a.y));
  LAUNCH(c, MMLA_STAGE_GLUE, 4.0 * (double)(n + n_out), sinc_resample_launch(a, c->stream));
  CHK(copy_back(c, y, 0, a.y, (size_t)n_out, dev));
  // the host vectors above are read by the async uploads: wait before they go out of scope
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return finish(c, dev);
}

int mmla_debug_od_trace(mmla_ctx* c, const float* x, int64_t n, int stage, float* out,
                        int64_t out_floats) {
  if (!c || !x || !out || n < 1 || stage < 0 || stage > 11) return MMLA_E_INVALID;
  if (!c->od_loaded) return fail(c, MMLA_E_NOWEIGHTS, "OD weights not loaded");
  HIPCHK(c, hipSetDevice(c->device));
  void* p = nullptr;
  CHK(ws_get(c, S_IN, n * OD_IMG * sizeof(float), &p));
  HIPCHK(c, hipMemcpyAsync(p, x, n * OD_IMG * sizeof(float), hipMemcpyHostToDevice, c->stream));
  const float* tap = nullptr;
  int64_t tn = 0;
  CHK(run_od_net(c, nullptr, static_cast<float*>(p), n, nullptr, nullptr, OdGate(), stage, &tap,
                 &tn));
  if (tn > out_floats) return fail(c, MMLA_E_SHAPE, "trace stage %d needs %lld floats", stage, (long long)tn);
  HIPCHK(c, hipMemcpyAsync(out, tap, tn * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MMLA_OK;
}

int mmla_debug_ws_slot(mmla_ctx* c, int slot, void** ptr, size_t* bytes) {
  if (!c || !ptr || !bytes || slot < 0) return MMLA_E_INVALID;
  const bool have = slot < (int)c->ws.size() && c->ws[slot];
  *ptr = have ? c->ws[slot] : nullptr;
  *bytes = have ? c->ws_size[slot] : 0;
  return MMLA_OK;
}

int mmla_profile_enable(mmla_ctx* c, int on) {
  if (!c) return MMLA_E_INVALID;
  c->prof_on = on != 0;
  return MMLA_OK;
}

int mmla_profile_read(mmla_ctx* c, double* ms, int64_t* launches, double* work, int reset) {
  if (!c) return MMLA_E_INVALID;
  CHK(prof_collect(c));
  for (int i = 0; i < MMLA_NSTAGES; ++i) {
    if (ms) ms[i] = c->prof_ms[i];
    if (launches) launches[i] = c->prof_n[i];
    if (work) work[i] = c->prof_work[i];
    if (reset) {
      c->prof_ms[i] = 0.0;
      c->prof_n[i] = 0;
      c->prof_work[i] = 0.0;
    }
  }
  return MMLA_OK;
}

}  // extern "C"
