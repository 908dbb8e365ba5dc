// Variant microbenchmark of the LU trailing-update kernel (lu.hip lu_trail_kernel) at the Stage-II
// bench shape (B = 1024, N = 2000), first block (K0 = 0, 1936 x 1936 trailing matrix):
// hipEvent timing of the kernel and of its memory pipeline alone (DIAG 1: no MFMAs), algorithmic GB/s
// on the A22 read + write.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lubench.hip -o tools/lubench.bin
#include "../i-admm-lstm_amd/csrc/lu.hip"

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill(float* p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 1e-3f * (float)((i * 2654435761u) & 1023) - 0.5f;
}

template <int DIAG>
float run(int B, int N, int K0, float* A, int reps) {
  const int rest = N - K0 - kBlk;
  const int ntc = (rest + kTC - 1) / kTC, nrc = (rest + kTRW - 1) / kTRW;
  CK(hipFuncSetAttribute((const void*)lu_trail_kernel<true, DIAG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTrailLds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((lu_trail_kernel<true, DIAG>), dim3(B * ntc * nrc), dim3(kTrailThreads), kTrailLds, 0, N, K0, ntc, nrc, N, A);
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((lu_trail_kernel<true, DIAG>), dim3(B * ntc * nrc), dim3(kTrailThreads), kTrailLds, 0, N, K0, ntc, nrc, N, A);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024, N = argc > 2 ? atoi(argv[2]) : 2000;
  float* A;
  CK(hipMalloc(&A, (size_t)B * N * N * sizeof(float)));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, A, (int64_t)B * N * N);
  CK(hipDeviceSynchronize());
  for (int K0 : {0, 960}) {
    const double rest = N - K0 - kBlk;
    const double bytes = (double)B * 4.0 * (2 * rest * rest + 2 * rest * kBlk);
    const double flops = (double)B * 2.0 * rest * rest * kBlk;
    const char* names[2] = {"full", "no-mfma"};
    for (int round = 0; round < 2; ++round) {
      float t[2] = {run<0>(B, N, K0, A, 5), run<1>(B, N, K0, A, 5)};
      for (int v = 0; v < 2; ++v)
        printf("K0=%4d %-10s %8.3f ms  %7.0f GB/s alg  %6.1f TF\n", K0, names[v], t[v], bytes / t[v] / 1e6, flops / t[v] / 1e9);
    }
  }
  CK(hipFree(A));
  return 0;
}
