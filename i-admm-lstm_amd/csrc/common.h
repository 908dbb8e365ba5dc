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

// LSTM-cell transcendentals (branch-free, <= 2 ulp; tools/mathcheck.hip measures them against
// fp64 over the fp32 range the gates see).  sigmoid: accurate expf, hardware reciprocal in place of
// the IEEE division.  tanh: odd minimax polynomial x + x^3 P(x^2) on |x| < 0.625 (approximation
// error 4.5e-9 relative), 1 - 2/(e^{2|x|} + 1) above (no cancellation there: 2/(e+1) <= 0.45).
IADMM_DEV float sigmoid_cell(float x) { return __builtin_amdgcn_rcpf(1.0f + expf(-x)); }
IADMM_DEV float tanh_cell(float x) {
  const float ax = fabsf(x);
  const float s = x * x;
  float p = fmaf(s, -0.0057040372917676625f, 0.020637863933015994f);
  p = fmaf(s, p, -0.05373916009365762f);
  p = fmaf(s, p, 0.13331431844163766f);
  p = fmaf(s, p, -0.3333328129024227f);
  const float small = fmaf(x * s, p, x);
  const float e = __expf(2.0f * ax);
  const float big = 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
  return ax < 0.625f ? small : copysignf(big, x);
}

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
