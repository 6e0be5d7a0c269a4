// Implicit-GEMM NHWC convolution on gfx950 f32 MFMA (v_mfma_f32_32x32x2_f32: exact f32 products,
// the reference's Conv2D/Conv1D/Dense run float32 in TF -- SURVEY.md 8a a9, a16).
//
//   C[p][co] = sum_{dy,dx,ci} act(bn(x[n][ho*s+dy-ph][wo*s+dx-pw][ci])) * w[dy][dx][ci][co]
//   y[p][co] = C + bias[co] (+ res[p][co]) (+ maxpool2x2_same(src)[p][co])
//
// Tiling: 256 threads = 4 waves; block tile = 128 output pixels x BN output channels; wave w owns
// pixel rows [32w, 32w+32) and all BN columns (BN/32 accumulators of 32x32).  K is walked tap by
// tap in chunks of 16 input channels, staged global -> registers -> LDS (register prefetch of the
// next chunk overlaps the MFMAs of the current one).  The prologue BatchNorm + ELU/ReLU is applied
// while staging (padding taps stay 0, as Keras pads the activated tensor); the epilogue fuses the
// bias, the identity residual, or the pool-block residual "shortcut + MaxPool2D(2,'same')(t)".
#include "common.h"
#include "conv.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NT = 256;
constexpr int BM = 128;
constexpr int KC = 16;
constexpr int LDA = BM + 4;

template <int PRO>
MMLA_DEV float prologue(float v, float sc, float sh) {
  if constexpr (PRO == PRO_NONE) {
    return v;
  } else {
    v = fmaf(v, sc, sh);
    if constexpr (PRO == PRO_BN_ELU) return v > 0.0f ? v : expm1f(v);
    return fmaxf(v, 0.0f);
  }
}

template <int BN, int PRO, int EPI, bool VEC>
__global__ void __launch_bounds__(NT) conv_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) float As[KC][LDA];
  __shared__ __attribute__((aligned(16))) float Bs[KC][BN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int64_t P = (int64_t)a.n * a.ho * a.wo;
  const int64_t p0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;

  // A staging: two (pixel, channel-quad) slots per thread
  int am[2], akq[2], an[2], ahb[2], awb[2];
  bool aval[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int idx = tid + NT * r;
    akq[r] = idx & 3;
    am[r] = idx >> 2;
    const int64_t p = p0 + am[r];
    aval[r] = p < P;
    const int64_t pp = aval[r] ? p : 0;
    const int hw = a.ho * a.wo;
    an[r] = (int)(pp / hw);
    const int rem = (int)(pp - (int64_t)an[r] * hw);
    const int ho = rem / a.wo, wo = rem - ho * a.wo;
    ahb[r] = ho * a.stride - a.pad_h;
    awb[r] = wo * a.stride - a.pad_w;
  }

  const int nchunk_c = (a.cin + KC - 1) / KC;
  const int nchunks = a.kh * a.kw * nchunk_c;

  float areg[2][4];
  float breg[(KC * BN + NT - 1) / NT];

  auto load_chunk = [&](int c) {
    const int tap = c / nchunk_c;
    const int ci0 = (c - tap * nchunk_c) * KC;
    const int dy = tap / a.kw, dx = tap - dy * a.kw;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int hi = ahb[r] + dy, wi = awb[r] + dx;
      const int ci = ci0 + akq[r] * 4;
      const bool inb = aval[r] && hi >= 0 && hi < a.h && wi >= 0 && wi < a.w;
      const float* src = a.x + (((int64_t)an[r] * a.h + hi) * a.w + wi) * a.cin + ci;
      if constexpr (VEC) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (inb && ci < a.cin) {
          v = *reinterpret_cast<const float4*>(src);
          if constexpr (PRO != PRO_NONE) {
            const float4 sc = *reinterpret_cast<const float4*>(a.scale + ci);
            const float4 sh = *reinterpret_cast<const float4*>(a.shift + ci);
            v.x = prologue<PRO>(v.x, sc.x, sh.x);
            v.y = prologue<PRO>(v.y, sc.y, sh.y);
            v.z = prologue<PRO>(v.z, sc.z, sh.z);
            v.w = prologue<PRO>(v.w, sc.w, sh.w);
          }
        }
        areg[r][0] = v.x;
        areg[r][1] = v.y;
        areg[r][2] = v.z;
        areg[r][3] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = 0.0f;
          if (inb && ci + j < a.cin) {
            v = src[j];
            if constexpr (PRO != PRO_NONE) v = prologue<PRO>(v, a.scale[ci + j], a.shift[ci + j]);
          }
          areg[r][j] = v;
        }
      }
    }
    // B: rows ci0 .. ci0+15 of tap (dy, dx), columns n0 .. n0+BN-1
    const float* wt = a.wt + ((int64_t)tap * a.cin) * a.cout_pad + n0;
#pragma unroll
    for (int r = 0; r < (KC * BN + NT - 1) / NT; ++r) {
      const int idx = tid + NT * r;
      const int k = idx / BN, col = idx - k * BN;
      float v = 0.0f;
      if (idx < KC * BN && ci0 + k < a.cin) v = wt[(int64_t)(ci0 + k) * a.cout_pad + col];
      breg[r] = v;
    }
  };

  auto store_chunk = [&]() {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) As[akq[r] * 4 + j][am[r]] = areg[r][j];
#pragma unroll
    for (int r = 0; r < (KC * BN + NT - 1) / NT; ++r) {
      const int idx = tid + NT * r;
      if (idx < KC * BN) Bs[idx / BN][idx % BN] = breg[r];
    }
  };

  f32x16 acc[BN / 32];
#pragma unroll
  for (int t = 0; t < BN / 32; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.0f;

  load_chunk(0);
  for (int c = 0; c < nchunks; ++c) {
    __syncthreads();
    store_chunk();
    __syncthreads();
    if (c + 1 < nchunks) load_chunk(c + 1);
#pragma unroll
    for (int ks = 0; ks < KC / 2; ++ks) {
      const int k = 2 * ks + (lane >> 5);
      const float av = As[k][wave * 32 + (lane & 31)];
#pragma unroll
      for (int t = 0; t < BN / 32; ++t) {
        const float bv = Bs[k][t * 32 + (lane & 31)];
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[t], 0, 0, 0);
      }
    }
  }

  // epilogue: acc register r of lane holds row (r&3) + 8(r>>2) + 4(lane>>5), column lane&31.
  // All residual loads are issued before the first store (y and res may alias: interleaved, each
  // load would wait behind the previous store)
  float rsd[BN / 32][16];
  if constexpr (EPI == EPI_ADD) {
#pragma unroll
    for (int t = 0; t < BN / 32; ++t) {
      const int co = n0 + t * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t p = p0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        rsd[t][r] = (co < a.cout && p < P) ? a.res[p * a.cout + co] : 0.0f;
      }
    }
  }
#pragma unroll
  for (int t = 0; t < BN / 32; ++t) {
    const int co = n0 + t * 32 + (lane & 31);
    if (co >= a.cout) continue;
    const float b = a.bias[co];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int64_t p = p0 + wave * 32 + row;
      if (p >= P) continue;
      float v = acc[t][r] + b;
      if constexpr (EPI == EPI_ADD) {
        v += rsd[t][r];
      } else if constexpr (EPI == EPI_ADD_POOL) {
        const int hw = a.ho * a.wo;
        const int n = (int)(p / hw);
        const int rem = (int)(p - (int64_t)n * hw);
        const int ho = rem / a.wo, wo = rem - ho * a.wo;
        float m = -INFINITY;
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
          for (int dx = 0; dx < 2; ++dx) {
            const int hh = 2 * ho + dy, ww = 2 * wo + dx;
            if (hh < a.hp && ww < a.wp)
              m = fmaxf(m, a.res[(((int64_t)n * a.hp + hh) * a.wp + ww) * a.cout + co]);
          }
        v += m;
      }
      a.y[p * a.ldy + co] = v;
    }
  }
}

template <int BN, int PRO, int EPI>
hipError_t launch3(const ConvArgs& a, hipStream_t s) {
  const int64_t P = (int64_t)a.n * a.ho * a.wo;
  dim3 grid((unsigned)((P + BM - 1) / BM), (unsigned)(a.cout_pad / BN));
  if (a.cin % 4 == 0)
    hipLaunchKernelGGL((conv_kernel<BN, PRO, EPI, true>), grid, dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL((conv_kernel<BN, PRO, EPI, false>), grid, dim3(NT), 0, s, a);
  return hipGetLastError();
}

template <int BN>
hipError_t launch2(const ConvArgs& a, hipStream_t s) {
#define MMLA_CONV_CASE(P, E) \
  if (a.pro == P && a.epi == E) return launch3<BN, P, E>(a, s);
  MMLA_CONV_CASE(PRO_NONE, EPI_BIAS)
  MMLA_CONV_CASE(PRO_NONE, EPI_ADD)
  MMLA_CONV_CASE(PRO_NONE, EPI_ADD_POOL)
  MMLA_CONV_CASE(PRO_BN_ELU, EPI_BIAS)
  MMLA_CONV_CASE(PRO_BN_ELU, EPI_ADD)
  MMLA_CONV_CASE(PRO_BN_RELU, EPI_BIAS)
  MMLA_CONV_CASE(PRO_BN_RELU, EPI_ADD)
#undef MMLA_CONV_CASE
  return hipErrorInvalidValue;
}

}  // namespace

hipError_t conv_launch(const ConvArgs& a, hipStream_t s) {
  if ((int64_t)a.n * a.ho * a.wo == 0) return hipSuccess;
  if (a.cout_pad % 32 != 0 || a.cout > a.cout_pad) return hipErrorInvalidValue;
  if (a.cout_pad % 128 == 0 && a.cout_pad >= 128) return launch2<128>(a, s);
  if (a.cout_pad % 64 == 0) return launch2<64>(a, s);
  return launch2<32>(a, s);
}
