// Probe: how much VALU work hides beside v_mfma_f32_32x32x2_f32 on gfx950.
//  mode 1: one wave per SIMD (256-thread workgroup, one per CU): per iteration 8 MFMAs on 8
//          independent accumulators, each followed by NV independent VALU instructions of KIND.
//  mode 2: two waves per SIMD (512-thread workgroup): waves 0-3 MFMA-only, waves 4-7 VALU-only
//          (NV VALU per MFMA-slot of the partner), i.e. the cell kernel's epilogue-beside-partner case.
//  mode 3: two waves per SIMD, both as mode 1 (MFMA + NV VALU per MFMA).
// KIND: 0 v_fma_f32, 1 v_pk_fma_f32, 2 v_exp_f32, 3 s_add_u32, 4 ds_read_b128, 5 LDS-DMA piece
// (buffer_load_dwordx4 ... lds, 1 KiB per wave), 6 v_add_u32.  Output: cycles per MFMA (s_memtime, shader clock).
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_valu_probe.hip -o tools/mfma_valu_probe.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float float2v __attribute__((ext_vector_type(2)));

template <int KIND>
__device__ __forceinline__ void valu(float& a0, float& a1, float& a2, float& a3, float2v& p0, float2v& p1,
                                     float2v& p2, float2v& p3, int i, int& sc,
                                     __amdgpu_buffer_rsrc_t rs, float* lds, unsigned voff) {
  const int s = i & 3;
  if constexpr (KIND == 0) {
    if (s == 0) asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(a0));
    else if (s == 1) asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(a1));
    else if (s == 2) asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(a2));
    else asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(a3));
  } else if constexpr (KIND == 1) {
    if (s == 0) asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(p0));
    else if (s == 1) asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(p1));
    else if (s == 2) asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(p2));
    else asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(p3));
  } else if constexpr (KIND == 3) {
    asm volatile("s_add_u32 %0, %0, 1" : "+s"(sc));
  } else if constexpr (KIND == 5) {
    typedef __attribute__((address_space(3))) void lds_void;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + 256 * (i & 15)), 16, voff + 1024u * (i & 15), 0, 0, 0);
  } else if constexpr (KIND == 6) {
    asm volatile("v_add_u32 %0, %0, 3" : "+v"(sc));
  } else if constexpr (KIND == 4) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    f4v t;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(t) : "v"(0), "i"(16 * (i & 7)));
    asm volatile("s_waitcnt lgkmcnt(8)" :: "v"(t));
  } else {
    if (s == 0) asm volatile("v_exp_f32 %0, %0" : "+v"(a0));
    else if (s == 1) asm volatile("v_exp_f32 %0, %0" : "+v"(a1));
    else if (s == 2) asm volatile("v_exp_f32 %0, %0" : "+v"(a2));
    else asm volatile("v_exp_f32 %0, %0" : "+v"(a3));
  }
}

template <int MODE, int NV, int KIND>
__global__ __launch_bounds__(MODE == 1 ? 256 : 512, 1) void probe(int iters, float* out, uint64_t* cyc, const float* src) {
  extern __shared__ float dyn[];  // sized on the host so one workgroup fills a CU
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool mfma_wave = MODE != 2 || wave < 4;
  float a = 1e-3f * (lane + 1), b = 2e-3f * (lane + 3);
  floatx16 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[j][q] = 0.f;
  float a0 = 0.1f * lane, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  float2v p0 = {a0, a1}, p1 = {a1, a2}, p2 = {a2, a3}, p3 = {a3, a0};
  int sc = __builtin_amdgcn_readfirstlane(iters);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), 0, 1 << 20, 0x00020000);
  const unsigned voff = (unsigned)(lane * 16 + (blockIdx.x & 15) * 16384);
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (!mfma_wave) {  // mode 2, waves 4-7: VALU only
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int v = 0; v < NV; ++v) valu<KIND>(a0, a1, a2, a3, p0, p1, p2, p3, v, sc, rs, dyn, voff);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + tid] = (float)sc + a0 + a1 + a2 + a3 + p0.x + p1.y + p2.x + p3.y;
    if (lane == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
    return;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (MODE != 2) {
#pragma unroll
        for (int v = 0; v < NV; ++v) valu<KIND>(a0, a1, a2, a3, p0, p1, p2, p3, v, sc, rs, dyn, voff);
        if constexpr (KIND == 5) __builtin_amdgcn_s_waitcnt((12 & 15) | ((12 >> 4) << 14) | (7 << 4) | (15 << 8));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  float s = (float)sc + a0 + a1 + a2 + a3 + p0.x + p1.y + p2.x + p3.y;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += acc[j][lane & 15];
  out[blockIdx.x * blockDim.x + tid] = s;
  if (lane == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
  (void)dyn;
}

template <int MODE, int NV, int KIND>
static void run(float* out, uint64_t* cyc, uint64_t* hc, int iters) {
  static float* src = nullptr;
  if (!src) { hipMalloc(&src, 1 << 20); hipMemset(src, 0, 1 << 20); }
  const int nthr = MODE == 1 ? 256 : 512;
  const int lds = 100 * 1024;
  hipFuncSetAttribute((const void*)probe<MODE, NV, KIND>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipMemset(cyc, 0, 256 * 8 * 8);
  hipLaunchKernelGGL((probe<MODE, NV, KIND>), dim3(256), dim3(nthr), lds, 0, iters, out, cyc, src);
  hipLaunchKernelGGL((probe<MODE, NV, KIND>), dim3(256), dim3(nthr), lds, 0, iters, out, cyc, src);
  hipDeviceSynchronize();
  hipMemcpy(hc, cyc, 256 * 8 * 8, hipMemcpyDeviceToHost);
  double m = 0, v = 0;
  int nm = 0, nv = 0;
  for (int b = 0; b < 256; ++b)
    for (int w = 0; w < nthr / 64; ++w) {
      const double c = (double)hc[b * 8 + w] / (iters * 8.0);
      if (MODE != 2 || w < 4) { m += c; ++nm; } else { v += c; ++nv; }
    }
  const char* kn[7] = {"v_fma_f32", "v_pk_fma_f32", "v_exp_f32", "s_add_u32", "ds_read_b128", "lds-dma piece", "v_add_u32"};
  if (MODE == 3)
    printf("mode3 (2 waves/SIMD, both MFMA + %2d x %-12s per MFMA): %7.1f cyc per MFMA slot per wave\n", NV, kn[KIND], m / nm);
  else if (MODE == 1)
    printf("mode1 (1 wave/SIMD, MFMA + %2d x %-12s per MFMA): %7.1f cyc per MFMA slot\n", NV, kn[KIND], m / nm);
  else
    printf("mode2 (2 waves/SIMD: MFMA-only | %2d x %-12s per slot): MFMA wave %7.1f cyc/MFMA, VALU wave %7.1f cyc/slot\n",
           NV, kn[KIND], m / nm, v / nv);
}

int main(int argc, char** argv) {
  float* out;
  uint64_t* cyc;
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&cyc, 256 * 8 * 8);
  static uint64_t hc[256 * 8];
  const int it = 2000;
  if (argc > 1) {  // DMA / integer-VALU study only
    run<1, 0, 0>(out, cyc, hc, it);
    run<1, 1, 5>(out, cyc, hc, it);
    run<1, 2, 5>(out, cyc, hc, it);
    run<1, 4, 5>(out, cyc, hc, it);
    run<1, 4, 6>(out, cyc, hc, it);
    run<1, 8, 6>(out, cyc, hc, it);
    run<3, 1, 5>(out, cyc, hc, it);
    run<3, 2, 5>(out, cyc, hc, it);
    printf("%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
  }
  run<1, 0, 0>(out, cyc, hc, it);
  run<1, 4, 0>(out, cyc, hc, it);
  run<1, 8, 0>(out, cyc, hc, it);
  run<1, 12, 0>(out, cyc, hc, it);
  run<1, 16, 0>(out, cyc, hc, it);
  run<1, 24, 0>(out, cyc, hc, it);
  run<1, 4, 1>(out, cyc, hc, it);
  run<1, 8, 1>(out, cyc, hc, it);
  run<1, 12, 1>(out, cyc, hc, it);
  run<1, 4, 2>(out, cyc, hc, it);
  run<1, 8, 2>(out, cyc, hc, it);
  run<1, 12, 2>(out, cyc, hc, it);
  run<1, 8, 3>(out, cyc, hc, it);
  run<1, 16, 3>(out, cyc, hc, it);
  run<1, 2, 4>(out, cyc, hc, it);
  run<1, 4, 4>(out, cyc, hc, it);
  run<1, 8, 4>(out, cyc, hc, it);
  run<2, 0, 0>(out, cyc, hc, it);
  run<2, 4, 0>(out, cyc, hc, it);
  run<2, 8, 0>(out, cyc, hc, it);
  run<2, 16, 0>(out, cyc, hc, it);
  run<2, 4, 1>(out, cyc, hc, it);
  run<2, 8, 1>(out, cyc, hc, it);
  run<2, 4, 2>(out, cyc, hc, it);
  run<2, 8, 2>(out, cyc, hc, it);
  run<2, 4, 4>(out, cyc, hc, it);
  run<3, 0, 0>(out, cyc, hc, it);
  run<3, 4, 0>(out, cyc, hc, it);
  run<3, 8, 0>(out, cyc, hc, it);
  run<3, 16, 0>(out, cyc, hc, it);
  run<3, 4, 2>(out, cyc, hc, it);
  run<3, 8, 2>(out, cyc, hc, it);
  printf("%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
