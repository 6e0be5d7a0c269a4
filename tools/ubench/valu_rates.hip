// VALU issue rates on gfx950 (dev tool, not product): independent chains of one instruction kind,
// 16 waves per CU, timed with HIP events.  Prints wave64-instructions per CU per cycle-equivalent
// at the measured clock-independent rate (instructions / s / CU) and the implied cycles per wave
// instruction at 2.4 GHz and at the --mhz argument.
//   hipcc --offload-arch=gfx950 -O3 -o valu_rates valu_rates.hip && ./valu_rates 2100
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

constexpr int ITERS = 4096;
constexpr int CH = 8;   // independent chains per lane

template <int KIND>
__global__ void __launch_bounds__(256) rate_kernel(float* out, double* outd, float s) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (KIND == 0) {   // v_fma_f64
    double a[CH];
    for (int c = 0; c < CH; ++c) a[c] = t * 1e-9 + c;
    const double m = 0.999999 + s * 1e-12, k = 1e-7;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
      for (int c = 0; c < CH; ++c) a[c] = __builtin_fma(a[c], m, k);
    double r = 0;
    for (int c = 0; c < CH; ++c) r += a[c];
    outd[t] = r;
  } else if constexpr (KIND == 1) {   // v_add_f64
    double a[CH];
    for (int c = 0; c < CH; ++c) a[c] = t * 1e-9 + c;
    const double k = 1e-7 + s * 1e-12;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        a[c] = a[c] + k;
        asm volatile("" : "+v"(a[c]));
      }
    double r = 0;
    for (int c = 0; c < CH; ++c) r += a[c];
    outd[t] = r;
  } else if constexpr (KIND == 2) {   // v_fma_f32
    float a[CH];
    for (int c = 0; c < CH; ++c) a[c] = t * 1e-9f + c;
    const float m = 0.999999f + s * 1e-12f, k = 1e-7f;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        a[c] = __builtin_fmaf(a[c], m, k);
        asm volatile("" : "+v"(a[c]));   // one chain per register: no v_pk_fma_f32 pairing
      }
    float r = 0;
    for (int c = 0; c < CH; ++c) r += a[c];
    out[t] = r;
  } else if constexpr (KIND == 3) {   // v_pk_fma_f32
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a[CH];
    for (int c = 0; c < CH; ++c) a[c] = f2{t * 1e-9f + c, t * 2e-9f + c};
    const f2 m = {0.999999f + s * 1e-12f, 0.999998f}, k = {1e-7f, 2e-7f};
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
      for (int c = 0; c < CH; ++c) a[c] = __builtin_elementwise_fma(a[c], m, k);
    float r = 0;
    for (int c = 0; c < CH; ++c) r += a[c].x + a[c].y;
    out[t] = r;
  } else if constexpr (KIND == 4) {   // v_mul_f64
    double a[CH];
    for (int c = 0; c < CH; ++c) a[c] = t * 1e-9 + c + 1.0;
    const double m = 0.999999 + s * 1e-12;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        a[c] = a[c] * m;
        asm volatile("" : "+v"(a[c]));
      }
    double r = 0;
    for (int c = 0; c < CH; ++c) r += a[c];
    outd[t] = r;
  } else if constexpr (KIND == 6) {   // v_add_u32 (+ v_xor via the chain mix)
    uint32_t a[CH];
    for (int c = 0; c < CH; ++c) a[c] = t * 7 + c;
    const uint32_t k = 0x9e3779b9u + (uint32_t)s;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        a[c] = a[c] + k;
        asm volatile("" : "+v"(a[c]));
      }
    uint32_t r = 0;
    for (int c = 0; c < CH; ++c) r ^= a[c];
    out[t] = (float)r;
  } else if constexpr (KIND == 7) {   // v_perm_b32
    uint32_t a[CH];
    for (int c = 0; c < CH; ++c) a[c] = t * 7 + c;
    const uint32_t k = 0x01234567u + (uint32_t)s;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
      for (int c = 0; c < CH; ++c) a[c] = __builtin_amdgcn_perm(a[c], k, 0x05010400u);
    uint32_t r = 0;
    for (int c = 0; c < CH; ++c) r ^= a[c];
    out[t] = (float)r;
  } else if constexpr (KIND == 8) {   // v_cvt_pk_f16_f32 (f32 pair -> packed f16), chained through a bitcast
    float a[CH];
    for (int c = 0; c < CH; ++c) a[c] = t * 1e-3f + c;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        typedef float fl2 __attribute__((ext_vector_type(2)));
        const h2 h = __builtin_convertvector((fl2{a[c], a[c]}), h2);
        a[c] = __builtin_bit_cast(float, h);
      }
    float r = 0;
    for (int c = 0; c < CH; ++c) r += a[c];
    out[t] = r;
  } else if constexpr (KIND == 9) {   // v_dot4_i32_i8
    int a[CH];
    for (int c = 0; c < CH; ++c) a[c] = t * 7 + c;
    const int k = 0x01020304 + (int)s;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
      for (int c = 0; c < CH; ++c) a[c] = __builtin_amdgcn_sdot4(a[c], k, a[c], false);
    int r = 0;
    for (int c = 0; c < CH; ++c) r ^= a[c];
    out[t] = (float)r;
  } else {   // v_exp_f32 + v_sub_f32
    float a[CH];
    for (int c = 0; c < CH; ++c) a[c] = -(t & 7) * 0.1f - c * 0.01f;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        a[c] = __builtin_amdgcn_exp2f(a[c]) - 1.0f;
        asm volatile("" : "+v"(a[c]));
      }
    float r = 0;
    for (int c = 0; c < CH; ++c) r += a[c];
    out[t] = r;
  }
}

template <int KIND>
double run(const char* name, int cus, float* o, double* od, double mhz, int per_iter) {
  const int blocks = cus * 4;   // 4 x 256 threads = 16 waves per CU
  hipLaunchKernelGGL(rate_kernel<KIND>, dim3(blocks), dim3(256), 0, 0, o, od, 1.0f);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  const int reps = 5;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(rate_kernel<KIND>, dim3(blocks), dim3(256), 0, 0, o, od, 1.0f);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double waves = (double)blocks * 4 * reps;
  const double insts = waves * ITERS * CH * per_iter;        // wave instructions of the kind
  const double per_cu_s = insts / cus / (ms * 1e-3);         // wave-instructions / s / CU
  const double cyc = 4.0 * mhz * 1e6 / per_cu_s;             // cycles per wave-instr per SIMD
  printf("%-14s %8.3f ms  %.3e wave-inst/s/CU  => %.2f cycles per wave64 instruction per SIMD at %.0f MHz\n",
         name, ms / reps, per_cu_s, cyc, mhz);
  return cyc;
}

int main(int argc, char** argv) {
  const double mhz = argc > 1 ? atof(argv[1]) : 2100.0;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  printf("%s, %d CUs, clockRate %d kHz\n", p.gcnArchName, cus, p.clockRate);
  float* o;
  double* od;
  hipMalloc(&o, sizeof(float) * cus * 1024);
  hipMalloc(&od, sizeof(double) * cus * 1024);
  run<2>("v_fma_f32", cus, o, od, mhz, 1);
  run<3>("v_pk_fma_f32", cus, o, od, mhz, 1);
  run<0>("v_fma_f64", cus, o, od, mhz, 1);
  run<1>("v_add_f64", cus, o, od, mhz, 1);
  run<4>("v_mul_f64", cus, o, od, mhz, 1);
  run<5>("v_exp_f32+sub", cus, o, od, mhz, 1);
  run<6>("v_add_u32", cus, o, od, mhz, 1);
  run<7>("v_perm_b32", cus, o, od, mhz, 1);
  run<8>("v_cvt_pk_f16_f32", cus, o, od, mhz, 1);
  run<9>("v_dot4_i32_i8", cus, o, od, mhz, 1);
  hipFree(o);
  hipFree(od);
  return 0;
}
