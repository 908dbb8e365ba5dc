// Issue rate of v_mfma_f32_32x32x2f32 chains on gfx950: NACC independent accumulators per wave
// (NACC = 1: every MFMA depends on the previous one through its accumulator, as in the LU trailing
// update's per-wave 32x32 tile), 1 or 2 waves per SIMD (WPS).  Prints cycles per MFMA per SIMD.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/mfma_chain_probe.hip -o tools/mfma_chain_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float floatx16 __attribute__((ext_vector_type(16)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int NACC>
__global__ __launch_bounds__(256) void chain(int iters, float* out, float seed) {
  const int lane = threadIdx.x & 63;
  const float a = seed * (lane + 1), b = seed * (lane + 2);
  floatx16 acc[NACC];
  for (int i = 0; i < NACC; ++i) for (int q = 0; q < 16; ++q) acc[i][q] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 64 / NACC; ++u)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b + u, acc[i], 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) for (int q = 0; q < 16; ++q) s += acc[i][q];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NACC>
void run(int wps, float* out) {
  int dev; CK(hipGetDevice(&dev));
  hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, dev));
  const int cus = pr.multiProcessorCount, iters = 2000;
  const int blocks = cus * wps;  // 256 threads = one wave per SIMD per block
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(chain<NACC>, dim3(blocks), dim3(256), 0, 0, 10, out, 1e-3f);
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(chain<NACC>, dim3(blocks), dim3(256), 0, 0, iters, out, 1e-3f);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  const double mfma_per_simd = (double)wps * iters * 64;
  const double clk = pr.clockRate * 1e3;  // Hz
  printf("NACC=%d waves/SIMD=%d: %.3f ms, %.1f cycles per MFMA per SIMD (clock %.0f MHz), %.1f TF/s\n", NACC, wps, ms,
         ms * 1e-3 * clk / mfma_per_simd, clk / 1e6, (double)blocks * 4 * iters * 64 * 4096.0 / (ms * 1e-3) / 1e12);
}

int main() {
  float* out; CK(hipMalloc(&out, 4096 * 256 * 4));
  for (int rep = 0; rep < 2; ++rep)
    for (int wps : {1, 2}) { run<1>(wps, out); run<2>(wps, out); run<4>(wps, out); }
  return 0;
}
