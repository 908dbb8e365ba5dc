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

// LSTM-cell transcendentals (branch-free, <= 3.1 ulp; tools/mathcheck.hip measures them against
// fp64).  Each has a scalar form and a packed two-lane form (v_pk_*_f32 for everything but the
// v_exp/v_rcp transcendentals) built from the SAME operation sequence, so both give bitwise
// identical results; the cell epilogue runs the packed form, the training recompute the scalar.
//   exp:     e^y = 2^th * 2^tl with th + tl = y log2(e) split exactly by an fma, 2^th on v_exp_f32
//            and 2^tl ~ 1 + tl ln2 (|tl| < 2^-10, so the dropped terms are < 2^-22 relative)
//   sigmoid: 1 / (1 + e^-x) with the hardware reciprocal
//   tanh:    odd minimax polynomial x + x^3 P(x^2) on |x| < 0.625 (approximation error 4.5e-9
//            relative), 1 - 2/(e^{2|x|} + 1) above (no cancellation there: 2/(e+1) <= 0.45)
typedef float float2v __attribute__((ext_vector_type(2)));
constexpr float kL2E = 1.44269502f;           // fp32(log2 e)
constexpr float kL2E_LO = 1.925963033e-08f;   // log2(e) - kL2E
constexpr float kLN2 = 0.693147181f;
constexpr float kTh4 = -0.0057040372917676625f, kTh3 = 0.020637863933015994f, kTh2 = -0.05373916009365762f,
                kTh1 = 0.13331431844163766f, kTh0 = -0.3333328129024227f;

// y is clamped to [-87, 88] first (v_med3): e^y stays finite, so the fma correction never meets
// inf (inf * negative + inf = NaN) and +-inf inputs give sigmoid 0 / 1 like torch; beyond the clamp
// the sigmoid differs from the exact value by < 1e-38.
IADMM_DEV float exp_cell(float y) {
  y = __builtin_amdgcn_fmed3f(y, -87.0f, 88.0f);
  const float th = y * kL2E;
  float tl = fmaf(y, kL2E, -th);
  tl = fmaf(y, kL2E_LO, tl);
  const float e = __builtin_amdgcn_exp2f(th);
  return fmaf(e, tl * kLN2, e);
}
IADMM_DEV float sigmoid_cell(float x) { return __builtin_amdgcn_rcpf(1.0f + exp_cell(-x)); }
IADMM_DEV float tanh_cell(float x) {
  const float s = x * x;
  float p = fmaf(s, kTh4, kTh3);
  p = fmaf(s, p, kTh2);
  p = fmaf(s, p, kTh1);
  p = fmaf(s, p, kTh0);
  const float small = fmaf(x * s, p, x);
  const float ax = fabsf(x);
  const float e = __builtin_amdgcn_exp2f((ax + ax) * kL2E);
  const float big = fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
  return ax < 0.625f ? small : copysignf(big, x);
}

IADMM_DEV float2v fma2(float2v a, float2v b, float2v c) { return __builtin_elementwise_fma(a, b, c); }
IADMM_DEV float2v splat2(float v) { return float2v{v, v}; }
IADMM_DEV float2v exp_cell2(float2v y) {
  y = float2v{__builtin_amdgcn_fmed3f(y.x, -87.0f, 88.0f), __builtin_amdgcn_fmed3f(y.y, -87.0f, 88.0f)};
  const float2v th = y * splat2(kL2E);
  float2v tl = fma2(y, splat2(kL2E), -th);
  tl = fma2(y, splat2(kL2E_LO), tl);
  const float2v e = float2v{__builtin_amdgcn_exp2f(th.x), __builtin_amdgcn_exp2f(th.y)};
  return fma2(e, tl * splat2(kLN2), e);
}
IADMM_DEV float2v rcp2(float2v d) { return float2v{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)}; }
IADMM_DEV float2v sigmoid_cell2(float2v x) { return rcp2(splat2(1.0f) + exp_cell2(-x)); }
IADMM_DEV float2v tanh_cell2(float2v x) {
  const float2v s = x * x;
  float2v p = fma2(s, splat2(kTh4), splat2(kTh3));
  p = fma2(s, p, splat2(kTh2));
  p = fma2(s, p, splat2(kTh1));
  p = fma2(s, p, splat2(kTh0));
  const float2v small = fma2(x * s, p, x);
  const float2v ax = float2v{fabsf(x.x), fabsf(x.y)};
  const float2v t = (ax + ax) * splat2(kL2E);
  const float2v e = float2v{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  const float2v big = fma2(splat2(-2.0f), rcp2(e + splat2(1.0f)), splat2(1.0f));
  return float2v{ax.x < 0.625f ? small.x : copysignf(big.x, x.x), ax.y < 0.625f ? small.y : copysignf(big.y, x.y)};
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
