// Where a Stage-II panel launch goes (B = 1024, N = 2000): lu_panel_kernel<M, 16, 256> as the
// factorization launches it at panel starts k0 with M = 1, 2, 4, 6, 8 rows per thread, in full and
// without its column steps (DIAG 1), without panel_finish (the in-block interchanges and the
// 16-row TRSM; DIAG 2), and with neither (the panel's load and store alone; DIAG 3).  hipEvents,
// median of 5 launches each, on the same (refactored in place) matrices.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lupanelbench.hip -o tools/lupanelbench.bin
#include "../i-admm-lstm_amd/csrc/lu.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace iadmm;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill(float* p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (x & 0xffffff) / 16777216.0f - 0.5f;
  }
}

__global__ void count_diff(const unsigned* a, const unsigned* b, int64_t n, unsigned long long* out) {
  unsigned long long c = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) c += a[i] != b[i];
  if (c) atomicAdd(out, c);
}

template <int M, int DIAG>
float run(int B, int N, int k0, float* A, int* piv, int* info) {
  const int K0 = (k0 / 64) * 64, cend = std::min(N, K0 + 64);
  std::vector<float> t;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int r = 0; r < 6; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((lu_panel_kernel<M, 16, 256, DIAG>), dim3(B), dim3(256), 0, 0, N, K0, k0, cend, A, piv, info);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r) t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

template <int M>
void row(int B, int N, int k0, float* A, int* piv, int* info) {
  const float f = run<M, 0>(B, N, k0, A, piv, info), c = run<M, 1>(B, N, k0, A, piv, info);
  const float p = run<M, 2>(B, N, k0, A, piv, info), m = run<M, 3>(B, N, k0, A, piv, info);
  printf("M=%d k0=%4d rows=%4d | full %7.1f us | no columns %7.1f | no finish %7.1f | load+store only %7.1f\n", M, k0,
         N - k0, f * 1e3, c * 1e3, p * 1e3, m * 1e3);
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024, N = 2000;
  float* A;
  int *piv, *info;
  CK(hipMalloc(&A, (size_t)B * N * N * 4));
  CK(hipMalloc(&piv, (size_t)B * N * 4));
  CK(hipMalloc(&info, (size_t)B * 4));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, A, (int64_t)B * N * N);
  CK(hipMemset(info, 0, B * 4));
  CK(hipDeviceSynchronize());
  {  // determinism: the full kernel on two copies of one input, outputs and pivots compared bit for bit
    float* A2;
    int* piv2;
    CK(hipMalloc(&A2, (size_t)B * N * N * 4));
    CK(hipMalloc(&piv2, (size_t)B * N * 4));
    for (int trial = 0; trial < 4; ++trial) {
      const int k0s[5] = {16, 528, 1040, 1552, 1808};
      for (int t = 0; t < 5; ++t) {
        const int k0 = k0s[t], K0 = (k0 / 64) * 64, cend = std::min(N, K0 + 64);
        hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, A, (int64_t)B * N * N);
        CK(hipMemcpy(A2, A, (size_t)B * N * N * 4, hipMemcpyDeviceToDevice));
        CK(hipMemset(piv, 0, (size_t)B * N * 4));
        CK(hipMemset(piv2, 0, (size_t)B * N * 4));
        float* As[2] = {A, A2};
        int* ps[2] = {piv, piv2};
        for (int c = 0; c < 2; ++c) {
          if (t == 0) hipLaunchKernelGGL((lu_panel_kernel<8, 16, 256, 0>), dim3(B), dim3(256), 0, 0, N, K0, k0, cend, As[c], ps[c], info);
          if (t == 1) hipLaunchKernelGGL((lu_panel_kernel<6, 16, 256, 0>), dim3(B), dim3(256), 0, 0, N, K0, k0, cend, As[c], ps[c], info);
          if (t == 2) hipLaunchKernelGGL((lu_panel_kernel<4, 16, 256, 0>), dim3(B), dim3(256), 0, 0, N, K0, k0, cend, As[c], ps[c], info);
          if (t == 3) hipLaunchKernelGGL((lu_panel_kernel<2, 16, 256, 0>), dim3(B), dim3(256), 0, 0, N, K0, k0, cend, As[c], ps[c], info);
          if (t == 4) hipLaunchKernelGGL((lu_panel_kernel<1, 16, 256, 0>), dim3(B), dim3(256), 0, 0, N, K0, k0, cend, As[c], ps[c], info);
        }
        CK(hipDeviceSynchronize());
        unsigned long long* cnt;
        CK(hipMalloc(&cnt, 16));
        CK(hipMemset(cnt, 0, 16));
        hipLaunchKernelGGL(count_diff, dim3(4096), dim3(256), 0, 0, (const unsigned*)A, (const unsigned*)A2, (int64_t)B * N * N, cnt);
        hipLaunchKernelGGL(count_diff, dim3(256), dim3(256), 0, 0, (const unsigned*)piv, (const unsigned*)piv2, (int64_t)B * N, cnt + 1);
        unsigned long long hc[2];
        CK(hipMemcpy(hc, cnt, 16, hipMemcpyDeviceToHost));
        CK(hipFree(cnt));
        const size_t d = hc[0], dp = hc[1];
        printf("determinism trial %d k0=%4d: %zu differing matrix words, %zu differing pivots\n", trial, k0, d, dp);
      }
    }
    CK(hipFree(A2));
    CK(hipFree(piv2));
  }
  for (int rep = 0; rep < 2; ++rep) {
    row<8>(B, N, 16, A, piv, info);
    row<6>(B, N, 528, A, piv, info);
    row<4>(B, N, 1040, A, piv, info);
    row<2>(B, N, 1552, A, piv, info);
    row<1>(B, N, 1808, A, piv, info);
  }
  CK(hipGetLastError());
  return 0;
}
