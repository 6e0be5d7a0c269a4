// dev probe: does a workgroup with a large LDS allocation disturb the LDS of a co-resident
// workgroup of another kernel?  (The OD front-end's power rows were corrupted only while the
// fused res-block kernel, 68-79 KB of LDS per workgroup, ran on another stream.)
//
// big<B>:   256 threads, B bytes of LDS; every round fills its whole LDS with a workgroup-specific
//           pattern, then checks it.
// small<B>: one wave, B bytes of LDS, same pattern test.
// Both kernels run concurrently on two streams; each thread writes its mismatch count with a plain
// vector store.  Build: hipcc -O3 --offload-arch=gfx950 tools/lds_probe.hip -o tools/lds_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__device__ __forceinline__ uint32_t pat(uint32_t tag, uint32_t i, uint32_t it) {
  return tag ^ (i * 2654435761u) ^ (it * 40503u);
}

template <int B, int NT>
__global__ void __launch_bounds__(NT) lds_fill_check(uint32_t* err, int iters, uint32_t kind) {
  __shared__ uint32_t s[B / 4];
  const uint32_t tag = (kind << 28) ^ blockIdx.x;
  uint32_t bad = 0;
  for (int it = 0; it < iters; ++it) {
    for (int i = threadIdx.x; i < B / 4; i += NT) s[i] = pat(tag, i, it);
    __syncthreads();
    for (int i = threadIdx.x; i < B / 4; i += NT) bad += s[i] != pat(tag, i, it);
    __syncthreads();
  }
  err[(size_t)blockIdx.x * NT + threadIdx.x] = bad;
}

template <int BIG>
int run(int big_blocks, int small_blocks) {
  constexpr int SMALL = 18 * 1024;
  uint32_t *eb = nullptr, *es = nullptr;
  CHECK(hipMalloc(&eb, (size_t)big_blocks * 256 * 4));
  CHECK(hipMalloc(&es, (size_t)small_blocks * 64 * 4));
  hipStream_t s1, s2;
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  uint64_t bad_big = 0, bad_small = 0;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL((lds_fill_check<BIG, 256>), dim3(big_blocks), dim3(256), 0, s1, eb, 400, 1u);
    hipLaunchKernelGGL((lds_fill_check<SMALL, 64>), dim3(small_blocks), dim3(64), 0, s2, es, 400, 2u);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    std::vector<uint32_t> hb((size_t)big_blocks * 256), hs((size_t)small_blocks * 64);
    CHECK(hipMemcpy(hb.data(), eb, hb.size() * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(hs.data(), es, hs.size() * 4, hipMemcpyDeviceToHost));
    for (uint32_t v : hb) bad_big += v;
    for (uint32_t v : hs) bad_small += v;
  }
  std::printf("big workgroup LDS %6d B (+ one-wave %d B co-running): mismatches big %llu, small %llu\n",
              BIG, SMALL, (unsigned long long)bad_big, (unsigned long long)bad_small);
  std::fflush(stdout);
  CHECK(hipStreamDestroy(s1));
  CHECK(hipStreamDestroy(s2));
  CHECK(hipFree(eb));
  CHECK(hipFree(es));
  return 0;
}

#ifndef LDS_PROBE_LIB
int main() {
  const int bb = 256 * 2 * 8, sb = 256 * 8 * 8;
  int rc = 0;
  rc |= run<60 * 1024>(bb, sb);
  rc |= run<64 * 1024>(bb, sb);
  rc |= run<65 * 1024>(bb, sb);
  rc |= run<68 * 1024>(bb, sb);
  rc |= run<78 * 1024>(bb, sb);
  return rc;
}
#endif

// ---- shared-library entry for Python co-run tests (tools/corun_diag8.py): launch the big-LDS
// kernel on a caller's stream.  kind: 0 -> 32 KB, 1 -> 60 KB, 2 -> 68 KB, 3 -> 78 KB per workgroup
extern "C" int lds_hog(void* stream, int kind, int blocks, int iters, uint32_t* err) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (kind) {
    case 0: hipLaunchKernelGGL((lds_fill_check<32 * 1024, 256>), dim3(blocks), dim3(256), 0, s, err, iters, 1u); break;
    case 1: hipLaunchKernelGGL((lds_fill_check<60 * 1024, 256>), dim3(blocks), dim3(256), 0, s, err, iters, 1u); break;
    case 2: hipLaunchKernelGGL((lds_fill_check<68 * 1024, 256>), dim3(blocks), dim3(256), 0, s, err, iters, 1u); break;
    default: hipLaunchKernelGGL((lds_fill_check<78 * 1024, 256>), dim3(blocks), dim3(256), 0, s, err, iters, 1u); break;
  }
  return (int)hipGetLastError();
}
