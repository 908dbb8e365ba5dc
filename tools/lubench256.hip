// Timing breakdown of the paired rank-256 update (lu_trail256_kernel, lu.hip) at the Stage-II bench
// shape (B = 1024, N = 2000), pair rows Pp = 0, 512, 1024: hipEvent time per launch, in full and in
// the diagnostic variants -- without the main loop's memory work (MODE 4), without its MFMAs (8: one
// VALU op each instead), without the prologue's MFMAs (16), and with only the main loop's MFMAs
// (4 + 16) -- on identity permutations (every row in place: the gathered addressing is still
// exercised, through the identity tables).  Results of the diagnostic variants are meaningless (and
// no-mem ones are void: the compiler drops the chain whose result is never stored).
// (r05 second form, one 8-wave workgroup per CU: profiles/r05_lubench256.txt, in this file's history.)
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lubench256.hip -o tools/lubench256.bin
#include "../i-admm-lstm_amd/csrc/lu.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

namespace iadmm {
__global__ void fill(float* p, int64_t n, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = scale * (1e-3f * (float)((i * 2654435761u) & 1023) - 0.5f);
}
// identity permutations of the pair's two blocks (rows [Pp, Pp + 128) and [Pp + 128, Pp + 256))
__global__ void ident(int64_t B, int Pp, int* perm0, int* perm1) {
  const int64_t b = blockIdx.x;
  int* pa = perm0 + b * kPermInts;
  int* qb = perm1 + b * kPermInts;
  for (int i = threadIdx.x; i < 2 * kPermMax; i += blockDim.x) {
    pa[i] = pa[2 * kPermMax + i] = Pp + i;
    qb[i] = qb[2 * kPermMax + i] = Pp + kOB + i;
  }
  if (threadIdx.x == 0) { pa[4 * kPermMax] = kOB; qb[4 * kPermMax] = kOB; }
}
}  // namespace iadmm
using namespace iadmm;

template <int MODE>
void launch(int B, int N, int Pp, float* A, const float* L0, const float* L1, const int* pp, const int* p1) {
  const int ntc = (N - Pp - kR2 + kT2C - 1) / kT2C;
  hipLaunchKernelGGL(lu_trail256_kernel<MODE>, dim3(B * ntc), dim3(kD2Threads), kP2Lds, 0, N, Pp, ntc, 0, A, L0, L1, pp, p1);
}

template <int MODE>
float run(int B, int N, int Pp, float* A, const float* L0, const float* L1, const int* pp, const int* p1, int reps) {
  CK(hipFuncSetAttribute((const void*)lu_trail256_kernel<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kP2Lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  launch<MODE>(B, N, Pp, A, L0, L1, pp, p1);
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch<MODE>(B, N, Pp, A, L0, L1, pp, p1);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024, N = argc > 2 ? atoi(argv[2]) : 2000;
  if (N % 4 || N > 2048 || N < 3 * kOB) { printf("need N %% 4 == 0, 384 <= N <= 2048\n"); return 1; }
  const size_t n = (size_t)B * N * N;
  float *A, *A2, *L0, *L1;
  int *pp, *p1;
  CK(hipMalloc(&A, n * sizeof(float)));
  CK(hipMalloc(&A2, n * sizeof(float)));
  CK(hipMalloc(&L0, (size_t)B * kLinvFloats * sizeof(float)));
  CK(hipMalloc(&L1, (size_t)B * kLinvFloats * sizeof(float)));
  CK(hipMalloc(&pp, (size_t)B * kPermInts * sizeof(int)));
  CK(hipMalloc(&p1, (size_t)B * kPermInts * sizeof(int)));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, L0, (int64_t)B * kLinvFloats, 0.05f);
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, L1, (int64_t)B * kLinvFloats, 0.05f);
  for (int Pp : {0, 512, 1024}) {
    hipLaunchKernelGGL(ident, dim3(B), dim3(256), 0, 0, (int64_t)B, Pp, pp, p1);
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, A, (int64_t)n, 1.0f);
    CK(hipDeviceSynchronize());
    const double rest = N - Pp - kR2;
    const double flops = (double)B * 2.0 * (rest * rest * kR2 + kR2 * kR2 * rest);
    const double bytes = (double)B * 4.0 * (2 * rest * rest + rest * kR2 + 2 * kR2 * rest);
    const char* names[5] = {"full", "no-mem", "no-mfma", "no-pro", "loop-mfma"};
    for (int round = 0; round < 2; ++round) {
      float t[5] = {run<0>(B, N, Pp, A, L0, L1, pp, p1, 3), run<4>(B, N, Pp, A, L0, L1, pp, p1, 3),
                    run<8>(B, N, Pp, A, L0, L1, pp, p1, 3), run<16>(B, N, Pp, A, L0, L1, pp, p1, 3),
                    run<4 + 16>(B, N, Pp, A, L0, L1, pp, p1, 3)};
      for (int v = 0; v < 5; ++v)
        printf("Pp=%4d %-10s %8.3f ms  %7.0f GB/s alg  %6.1f TF\n", Pp, names[v], t[v], bytes / t[v] / 1e6, flops / t[v] / 1e9);
      fflush(stdout);
    }
  }
  CK(hipFree(A)); CK(hipFree(A2)); CK(hipFree(L0)); CK(hipFree(L1)); CK(hipFree(pp)); CK(hipFree(p1));
  return 0;
}
