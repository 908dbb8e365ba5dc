// Variant microbenchmark of the fused TRSM + rank-128 trailing update (lu.hip lu_trail128_kernel) at
// the Stage-II bench shape (B = 1024, N = 2000), outer blocks P = 0 and P = 896: hipEvent time of the
// kernel, of its main loop without MFMAs (DIAG 1: the memory / LDS pipeline alone) and without the
// main loop's global traffic (DIAG 2: MFMA + LDS + barriers alone).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lubench128.hip -o tools/lubench128.bin
#include "../i-admm-lstm_amd/csrc/lu.hip"

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill(float* p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 1e-3f * (float)((i * 2654435761u) & 1023) - 0.5f;
}

template <int DIAG>
float run(int B, int N, int P, float* A, float* Linv, int reps) {
  const int ntc = (N - P - kOB + kT2C - 1) / kT2C;
  CK(hipFuncSetAttribute((const void*)lu_trail128_kernel<true, DIAG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kT2Lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((lu_trail128_kernel<true, DIAG>), dim3(B * ntc), dim3(kT2Threads), kT2Lds, 0, N, P, ntc, A, Linv, nullptr);
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((lu_trail128_kernel<true, DIAG>), dim3(B * ntc), dim3(kT2Threads), kT2Lds, 0, N, P, ntc, A, Linv, nullptr);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024, N = argc > 2 ? atoi(argv[2]) : 2000;
  float *A, *Linv;
  CK(hipMalloc(&A, (size_t)B * N * N * sizeof(float)));
  CK(hipMalloc(&Linv, (size_t)B * kLinvFloats * sizeof(float)));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, A, (int64_t)B * N * N);
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, Linv, (int64_t)B * kLinvFloats);
  CK(hipDeviceSynchronize());
  for (int P : {0, 896}) {
    const double rest = N - P - kOB;
    const double bytes = (double)B * 4.0 * (2 * rest * rest + rest * kOB + 2 * kOB * rest);
    const double flops = (double)B * 2.0 * (rest * rest * kOB + kOB * kOB * rest);
    const char* names[3] = {"full", "no-mfma", "no-global"};
    for (int round = 0; round < 2; ++round) {
      float t[3] = {run<0>(B, N, P, A, Linv, 5), run<1>(B, N, P, A, Linv, 5), run<2>(B, N, P, A, Linv, 5)};
      for (int v = 0; v < 3; ++v)
        printf("P=%4d %-12s %8.3f ms  %7.0f GB/s alg  %6.1f TF\n", P, names[v], t[v], bytes / t[v] / 1e6, flops / t[v] / 1e9);
    }
  }
  CK(hipFree(A)); CK(hipFree(Linv));
  return 0;
}
