// Variant microbenchmark of the fused LSTM-cell kernel at the bench shape (M = 1024*2000 rows,
// h = 800): interleaved rounds of every variant in one process (cdna_hip_programming.md §5.4
// rule 24), hipEvent timing, TFLOP/s on the algorithmic 8*M*h^2 + 18*M*h flops.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -mllvm -disable-promote-alloca-to-lds \
//          tools/cellbench.hip -o tools/cellbench.bin
// Variants are instances of the production kernel template (cell_tile.h cell_fwd_kernel<VEC, NW,
// PRIO>); the first is the one lstm.hip launches.  Round-1 study of earlier variants (BK 16 / double
// buffer / fast transcendentals / 16x16x4 MFMA): profiles/r01_cellbench.txt.
#include "../i-admm-lstm_amd/csrc/cell_tile.h"

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <string>
#include <algorithm>
#include <cmath>

using namespace iadmm;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill(float* p, int64_t n, uint32_t seed, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = scale * ((x & 0xffffff) / 16777216.0f * 2.f - 1.f);
  }
}

// Pure-MFMA ceiling at the cell kernel's register shape (8 accumulators, operands in registers,
// same grid and occupancy): how many fp32 MFMA TFLOP/s this device sustains under load.
typedef float floatx4 __attribute__((ext_vector_type(4)));
template <int SHAPE>
__global__ __launch_bounds__(256, 2) void mfma_ceiling(int iters, float* out, float seed) {
  const int lane = threadIdx.x & 63;
  float av = seed * (lane + 1), bv = seed * (lane + 3);
  if constexpr (SHAPE == 32) {
    floatx16 acc[8];
    for (int i = 0; i < 8; ++i) for (int q = 0; q < 16; ++q) acc[i][q] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv + i, acc[i], 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 8; ++i) for (int q = 0; q < 16; ++q) s += acc[i][q];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else if constexpr (SHAPE == 33) {  // 32x32x2 with random full-mantissa operands, 64 pairings
    float ar[8], br[8];
    for (int i = 0; i < 8; ++i) {
      uint32_t x = (uint32_t)(threadIdx.x * 8 + i + blockIdx.x * 4096) * 2654435761u;
      x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
      ar[i] = (x & 0xffffff) / 16777216.0f * 2.f - 1.f;
      x = x * 2654435761u + 12345u; x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
      br[i] = (x & 0xffffff) / 16777216.0f * 2.f - 1.f;
    }
    floatx16 acc[8];
    for (int i = 0; i < 8; ++i) for (int q = 0; q < 16; ++q) acc[i][q] = 0.f;
    for (int it = 0; it < iters; it += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[i], br[(i + u) & 7], acc[i], 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 8; ++i) for (int q = 0; q < 16; ++q) s += acc[i][q];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else {
    floatx4 acc[32];
    for (int i = 0; i < 32; ++i) for (int q = 0; q < 4; ++q) acc[i][q] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 32; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv + i, acc[i], 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 32; ++i) for (int q = 0; q < 4; ++q) s += acc[i][q];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  }
}

struct Variant {
  std::string name;
  void (*launch)(CellArgsT, int64_t, hipStream_t);
};

template <int NW, int PRIO, bool BUF = false>
void launch_v(CellArgsT a, int64_t M, hipStream_t s) {
  const int64_t rows = 64 * NW;
  const int64_t nrt = (M + rows - 1) / rows;
  hipLaunchKernelGGL((cell_fwd_kernel<true, NW, PRIO, BUF>), dim3((unsigned)(nrt * a.njt)), dim3(64 * NW), 0, s, a);
}

template <int DIAG, bool K16 = true>
void launch_dma(CellArgsT a, int64_t M, hipStream_t s) {
  static bool once = [] {
    CK(hipFuncSetAttribute((const void*)cell_fwd_dma_kernel<DIAG, K16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           kDmaLdsBytes));
    return true;
  }();
  (void)once;
  const int64_t nrt = (M + 255) / 256;
  hipLaunchKernelGGL((cell_fwd_dma_kernel<DIAG, K16>), dim3((unsigned)(nrt * a.njt)), dim3(256), kDmaLdsBytes, s, a);
}

int main(int argc, char** argv) {
  const int64_t B = argc > 1 ? atoll(argv[1]) : 1024;
  const int64_t N = 2000, h = 800;
  const int64_t M = B * N;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const int njt = (h + 31) / 32, nkc32 = (h + 31) / 32;
  float *H, *C, *xv, *g, *Upk, *Wx, *Hn, *Cn, *part;
  CK(hipMalloc(&H, M * h * 4)); CK(hipMalloc(&C, M * h * 4)); CK(hipMalloc(&Hn, M * h * 4)); CK(hipMalloc(&Cn, M * h * 4));
  CK(hipMalloc(&xv, M * 4)); CK(hipMalloc(&g, M * 4)); CK(hipMalloc(&part, (int64_t)njt * M * 4 + (int64_t)njt * ((M + 255) / 256) * 64));
  const int64_t nup = (int64_t)njt * nkc32 * 128 * 32, nwx = (int64_t)njt * 32 * 16;
  CK(hipMalloc(&Upk, nup * 4)); CK(hipMalloc(&Wx, nwx * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, H, M * h, 1u, 0.9f);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, C, M * h, 2u, 0.5f);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, xv, M, 3u, 1.0f);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, g, M, 4u, 1.0f);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, Upk, nup, 5u, 0.02f);
  hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, 0, Wx, nwx, 6u, 0.02f);
  CK(hipDeviceSynchronize());
  CellArgsT a{M, (int)h, njt, nkc32, H, C, xv, g, Upk, Wx, Hn, Cn, part, 4};
  if (argc > 3 && std::string(argv[3]) == "phase") {  // raw DIAG-6 stamps -> argv[4] (tools/cellphase.py)
    const int64_t nwg = njt * ((M + 255) / 256);
    launch_dma<0>(a, M, 0);
    launch_dma<6>(a, M, 0);
    CK(hipDeviceSynchronize());
    launch_dma<6>(a, M, 0);
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> st(nwg * 8);
    CK(hipMemcpy(st.data(), reinterpret_cast<char*>(part) + (int64_t)njt * M * 4, nwg * 64, hipMemcpyDeviceToHost));
    FILE* f = fopen(argc > 4 ? argv[4] : "phase.bin", "wb");
    fwrite(st.data(), 8, st.size(), f);
    fclose(f);
    printf("wrote %lld workgroups x 8 words\n", (long long)nwg);
    return 0;
  }
  std::vector<Variant> vs = {
      {"NW4 (production)        ", launch_v<4, 0>},
      {"LDS-DMA ring, generic   ", launch_dma<0, false>},
      {"LDS-DMA ring, K16 (prod)", launch_dma<0>},
      {"DIAG: DMA + stamps      ", launch_dma<4>},
      {"DIAG: stamps, no stores ", launch_dma<5>},
      {"DIAG: DMA, no epilogue  ", launch_dma<1>},
      {"DIAG: DMA, no H/C stores", launch_dma<2>},
      {"DIAG: DMA, no C loads   ", launch_dma<3>},
  };
  const double flop = (8.0 * h * h + 18.0 * h) * M;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<std::vector<float>> t(vs.size());
  for (auto& v : vs) { v.launch(a, M, s); }  // warm-up
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipEventRecord(e0, s));
      vs[i].launch(a, M, s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms);
    }
  }
  CK(hipGetLastError());
  {  // cross-check: every variant must reproduce the production kernel bit for bit
    std::vector<float> h1(1 << 22), h2(1 << 22), p1(1 << 20), p2(1 << 20);
    vs[0].launch(a, M, s);
    CK(hipMemcpyAsync(h1.data(), Hn, h1.size() * 4, hipMemcpyDeviceToHost, s));
    CK(hipMemcpyAsync(p1.data(), part, p1.size() * 4, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    for (size_t i = 1; i < vs.size(); ++i) {
      if (vs[i].name.rfind("DIAG", 0) == 0) continue;
      vs[i].launch(a, M, s);
      CK(hipMemcpyAsync(h2.data(), Hn, h2.size() * 4, hipMemcpyDeviceToHost, s));
      CK(hipMemcpyAsync(p2.data(), part, p2.size() * 4, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      size_t bad = 0;
      for (size_t k = 0; k < h1.size(); ++k) bad += h1[k] != h2[k];
      for (size_t k = 0; k < p1.size(); ++k) bad += p1[k] != p2[k];
      printf("bitwise check %s: %zu mismatches\n", vs[i].name.c_str(), bad);
    }
  }
  printf("M=%lld h=%lld rounds=%d\n", (long long)M, (long long)h, rounds);
  for (int dv : {4, 5}) {  // per-workgroup phase lengths (s_memtime cycles) from the stamped variants
    const int64_t nwg = njt * ((M + 255) / 256);
    if (dv == 4) launch_dma<4>(a, M, s); else launch_dma<5>(a, M, s);
    CK(hipStreamSynchronize(s));
    std::vector<uint64_t> st(nwg * 4);
    CK(hipMemcpy(st.data(), reinterpret_cast<char*>(part) + (int64_t)njt * M * 4, nwg * 32, hipMemcpyDeviceToHost));
    std::vector<double> ml, cw, ep;
    for (int64_t w = 0; w < nwg; ++w) {
      ml.push_back((double)(st[4 * w + 1] - st[4 * w]));
      cw.push_back((double)(st[4 * w + 2] - st[4 * w + 1]));
      ep.push_back((double)(st[4 * w + 3] - st[4 * w + 2]));
    }
    std::sort(ml.begin(), ml.end()); std::sort(cw.begin(), cw.end()); std::sort(ep.begin(), ep.end());
    printf("stamps DIAG %d: main loop median %.0f cyc (p10 %.0f p90 %.0f) | operand wait median %.0f (p90 %.0f) | "
           "epilogue compute+store median %.0f (p10 %.0f p90 %.0f)\n", dv,
           ml[nwg / 2], ml[nwg / 10], ml[9 * nwg / 10], cw[nwg / 2], cw[9 * nwg / 10], ep[nwg / 2], ep[nwg / 10], ep[9 * nwg / 10]);
  }
  {  // MFMA ceiling: 512 blocks x 4 waves, each wave 8 x 32x32x2 (or 32 x 16x16x4) per iteration
    const int iters = 20000, blocks = 512;
    for (int shape : {32, 33, 32, 33}) {
      CK(hipEventRecord(e0, s));
      if (shape == 32) hipLaunchKernelGGL(mfma_ceiling<32>, dim3(blocks), dim3(256), 0, s, iters, part, 1e-3f);
      else hipLaunchKernelGGL(mfma_ceiling<33>, dim3(blocks), dim3(256), 0, s, iters, part, 1e-3f);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double f = (double)blocks * 4 * iters * 8 * 4096.0;  // 8 MFMAs x 4096 flop per wave-iteration
      printf("MFMA ceiling 32x32x2 f32, %s operands: %8.3f ms  %7.1f TFLOP/s\n",
             shape == 32 ? "fixed small" : "random     ", ms, f / (ms * 1e-3) / 1e12);
    }
  }
  for (size_t i = 0; i < vs.size(); ++i) {
    auto v = t[i];
    std::sort(v.begin(), v.end());
    const float med = v[v.size() / 2];
    printf("%s  median %8.3f ms  min %8.3f ms  %7.1f TFLOP/s (median)\n", vs[i].name.c_str(), med, v[0], flop / (med * 1e-3) / 1e12);
  }
  return 0;
}
