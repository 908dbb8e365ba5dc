// Shared device helpers for the gfx950 kernels of libiadmm.so.
// Compiled with -ffp-contract=off: every fused multiply-add below is an explicit fmaf(), so the
// elementwise kernels keep the reference's rounding order (mul, then add) exactly.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/iadmm.h"

#define IADMM_DEV __device__ __forceinline__

namespace iadmm {

constexpr int kWave = 64;  // CDNA wavefront

IADMM_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

IADMM_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// torch.minimum / torch.maximum semantics: NaN propagates.
IADMM_DEV float tmin(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : (a < b ? a : b); }
IADMM_DEV float tmax(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : (a > b ? a : b); }

IADMM_DEV float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

IADMM_DEV float get4(const float4& v, int e) {
  return e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w));
}
IADMM_DEV void set4(float4& v, int e, float s) {
  if (e == 0) v.x = s; else if (e == 1) v.y = s; else if (e == 2) v.z = s; else v.w = s;
}

// Block-wide deterministic sum of one value per thread (fixed shuffle tree + fixed wave order).
// ``red`` is >= nwaves floats of LDS.  Result valid in every thread.
IADMM_DEV float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = red[0];
  for (int w = 1; w < nw; ++w) s += red[w];
  __syncthreads();
  return s;
}

__host__ __device__ inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace iadmm

// Dynamic LDS above 64 KiB (gfx950 has 160 KiB per CU) must be opted into per kernel.
#define IADMM_ALLOW_LDS(kernel, bytes)                                                        \
  do {                                                                                         \
    if ((bytes) > 65536) {                                                                     \
      hipError_t e_ = hipFuncSetAttribute((const void*)(kernel),                               \
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)(bytes)); \
      if (e_ != hipSuccess) return static_cast<int>(e_);                                       \
    }                                                                                          \
  } while (0)

#define IADMM_CHECK_LAUNCH()                          \
  do {                                                \
    hipError_t e_ = hipGetLastError();                \
    if (e_ != hipSuccess) return static_cast<int>(e_); \
  } while (0)
