// Variant microbenchmark of the fused TRSM + rank-128 trailing update at the Stage-II bench shape
// (B = 1024, N = 2000), outer blocks P = 0 and P = 896: hipEvent time of lu_trail128_kernel (r03)
// and of the wave-specialised lu_trail128ws_kernel (r04), each in full, without MFMAs (DIAG 1: the
// memory / LDS pipeline alone) and without the main loop's global traffic (DIAG 2: MFMA + LDS +
// barriers alone); and a bitwise comparison of the two kernels' outputs on the same input.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lubench128.hip -o tools/lubench128.bin
#include "../i-admm-lstm_amd/csrc/lu.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill(float* p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 1e-3f * (float)((i * 2654435761u) & 1023) - 0.5f;
}

template <int WS, int DIAG>
void launch(int B, int N, int P, float* A, float* Linv) {
  const int ntc = (N - P - kOB + kT2C - 1) / kT2C;
  if (WS) hipLaunchKernelGGL((lu_trail128ws_kernel<DIAG>), dim3(B * ntc), dim3(kWSThreads), kT2Lds, 0, N, P, ntc, A, Linv, nullptr);
  else hipLaunchKernelGGL((lu_trail128_kernel<true, DIAG>), dim3(B * ntc), dim3(kT2Threads), kT2Lds, 0, N, P, ntc, A, Linv, nullptr);
}

template <int WS, int DIAG>
float run(int B, int N, int P, float* A, float* Linv, int reps) {
  if (WS) CK(hipFuncSetAttribute((const void*)lu_trail128ws_kernel<DIAG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kT2Lds));
  else CK(hipFuncSetAttribute((const void*)lu_trail128_kernel<true, DIAG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kT2Lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  launch<WS, DIAG>(B, N, P, A, Linv);
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch<WS, DIAG>(B, N, P, A, Linv);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024, N = argc > 2 ? atoi(argv[2]) : 2000;
  float *A, *A2, *Linv;
  const size_t n = (size_t)B * N * N;
  CK(hipMalloc(&A, n * sizeof(float)));
  CK(hipMalloc(&A2, n * sizeof(float)));
  CK(hipMalloc(&Linv, (size_t)B * kLinvFloats * sizeof(float)));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, Linv, (int64_t)B * kLinvFloats);
  // bitwise: one launch of each kernel on the same input
  for (int P : {0, 896, N - kOB - 64}) {
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, A, (int64_t)n);
    CK(hipMemcpy(A2, A, n * sizeof(float), hipMemcpyDeviceToDevice));
    CK(hipFuncSetAttribute((const void*)lu_trail128ws_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kT2Lds));
    CK(hipFuncSetAttribute((const void*)lu_trail128_kernel<true, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kT2Lds));
    launch<0, 0>(B, N, P, A, Linv);
    launch<1, 0>(B, N, P, A2, Linv);
    CK(hipDeviceSynchronize());
    const size_t chk = (size_t)4 * N * N;  // first four instances
    std::vector<unsigned> h1(chk), h2(chk);
    CK(hipMemcpy(h1.data(), A, chk * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), A2, chk * 4, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (size_t i = 0; i < chk; ++i) diff += h1[i] != h2[i];
    std::vector<unsigned> t1(N * N), t2(N * N);  // the last instance (every XCD mapping position)
    CK(hipMemcpy(t1.data(), A + (size_t)(B - 1) * N * N, (size_t)N * N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(t2.data(), A2 + (size_t)(B - 1) * N * N, (size_t)N * N * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < (size_t)N * N; ++i) diff += t1[i] != t2[i];
    printf("P=%4d bitwise r03 vs ws: %zu differing words (instances 0-3 and %d)\n", P, diff, B - 1);
  }
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, A, (int64_t)n);
  CK(hipDeviceSynchronize());
  for (int P : {0, 896}) {
    const double rest = N - P - kOB;
    const double bytes = (double)B * 4.0 * (2 * rest * rest + rest * kOB + 2 * kOB * rest);
    const double flops = (double)B * 2.0 * (rest * rest * kOB + kOB * kOB * rest);
    const char* names[3] = {"full", "no-mfma", "no-global"};
    for (int round = 0; round < 2; ++round) {
      float t[6] = {run<0, 0>(B, N, P, A, Linv, 5), run<0, 1>(B, N, P, A, Linv, 5), run<0, 2>(B, N, P, A, Linv, 5),
                    run<1, 0>(B, N, P, A, Linv, 5), run<1, 1>(B, N, P, A, Linv, 5), run<1, 2>(B, N, P, A, Linv, 5)};
      for (int v = 0; v < 6; ++v)
        printf("P=%4d %-3s %-10s %8.3f ms  %7.0f GB/s alg  %6.1f TF\n", P, v < 3 ? "r03" : "ws", names[v % 3], t[v],
               bytes / t[v] / 1e6, flops / t[v] / 1e9);
    }
  }
  CK(hipFree(A)); CK(hipFree(A2)); CK(hipFree(Linv));
  return 0;
}
