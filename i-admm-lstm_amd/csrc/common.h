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

// LSTM-cell transcendentals, branch-free (tools/mathcheck.hip measures them against fp64).  Each
// has a scalar form and a packed two-lane form (v_pk_*_f32 for everything but the v_exp/v_rcp
// transcendentals and the clamp) built from the SAME operation sequence, so both give bitwise
// identical results; the cell epilogue runs the packed form, the training recompute the scalar.
//   sigmoid: 1 / (1 + 2^(-x log2 e)) on v_exp_f32 + v_rcp_f32 (relative error ~|x| 2^-24: no
//            cancellation anywhere)
//   tanh:    x P(x^2) / Q(x^2), P of degree 6, Q of degree 3 in x^2, on |x| clamped to 7.9053
//            (where fp32 tanh reaches 1 within 5 ulp); coefficients fitted here for minimal relative
//            error (5e-9 in exact arithmetic, <= ~6 ulp evaluated in fp32): relative accuracy down
//            to 0 (small LSTM states), no exp, no select
// The sigmoid needs no clamp: 2^(+inf) = inf -> rcp = 0, 2^(-inf) = 0 -> rcp(1) = 1, so it
// saturates to 0 / 1 like torch and NaN propagates; tanh saturates through its clamp, and a NaN
// input is passed through explicitly (v_med3 with a NaN operand returns min3 of its operands, i.e.
// the clamp would turn tanh(NaN) into tanh(-7.9) = -1 and hide a divergent solve; torch.tanh
// propagates NaN: one compare + select per element, r03).
// Why so lean: on gfx950 v_mfma_f32_32x32x2_f32 runs on the fp32 VALU datapath, so every VALU
// cycle of the epilogue is a cycle the SIMD's matrix work stalls (tools/mfma_valu_probe.hip,
// profiles/r02_mfma_valu_probe.txt).  The r01 forms (Cody-Waite exp with a v_med3 clamp, tanh as a
// polynomial/exp select with |x| and copysign) spent ~2x the VALU cycles.
typedef float float2v __attribute__((ext_vector_type(2)));
constexpr float kNL2E = -1.44269502f;          // -fp32(log2 e)
constexpr float kTanhClamp = 7.90531110763549805f;
constexpr float kTp1 = 0.1313343644142151f, kTp2 = 0.0031596473418176174f, kTp3 = 1.1755176274164114e-05f,
                kTp4 = -2.281726452224575e-08f, kTp5 = 6.643676581097324e-11f, kTp6 = -1.241359852367438e-13f;
constexpr float kTq1 = 0.4646677076816559f, kTq2 = 0.024715565145015717f, kTq3 = 0.00026282211183570325f;

IADMM_DEV float sigmoid_cell(float x) { return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * kNL2E)); }
IADMM_DEV float tanh_cell(float x0) {
  const float x = __builtin_amdgcn_fmed3f(x0, -kTanhClamp, kTanhClamp);
  const float s = x * x;
  float p = fmaf(s, kTp6, kTp5);
  p = fmaf(s, p, kTp4);
  p = fmaf(s, p, kTp3);
  p = fmaf(s, p, kTp2);
  p = fmaf(s, p, kTp1);
  p = fmaf(s, p, 1.0f);
  float q = fmaf(s, kTq3, kTq2);
  q = fmaf(s, q, kTq1);
  q = fmaf(s, q, 1.0f);
  const float r = (x * p) * __builtin_amdgcn_rcpf(q);
  return x0 != x0 ? x0 : r;
}
// Gate pre-activation: (b + in0 w0 + in1 w1) + acc, i.e. inputs @ W + H @ U + b
// (models/lstm.py:74-77) with the two-term input product on fmas.
IADMM_DEV float cell_pre(float in0, float in1, float acc, float w0, float w1, float b) {
  return fmaf(in1, w1, fmaf(in0, w0, b)) + acc;
}

IADMM_DEV float2v fma2(float2v a, float2v b, float2v c) { return __builtin_elementwise_fma(a, b, c); }
IADMM_DEV float2v splat2(float v) { return float2v{v, v}; }
IADMM_DEV float2v exp2_2(float2v y) { return float2v{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)}; }
IADMM_DEV float2v rcp2(float2v d) { return float2v{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)}; }
IADMM_DEV float2v sigmoid_cell2(float2v x) { return rcp2(splat2(1.0f) + exp2_2(x * splat2(kNL2E))); }
IADMM_DEV float nan_pass(float x0, float r) { return x0 != x0 ? x0 : r; }
IADMM_DEV float2v tanh_cell2(float2v x0) {
  const float2v x = float2v{__builtin_amdgcn_fmed3f(x0.x, -kTanhClamp, kTanhClamp),
                            __builtin_amdgcn_fmed3f(x0.y, -kTanhClamp, kTanhClamp)};
  const float2v s = x * x;
  float2v p = fma2(s, splat2(kTp6), splat2(kTp5));
  p = fma2(s, p, splat2(kTp4));
  p = fma2(s, p, splat2(kTp3));
  p = fma2(s, p, splat2(kTp2));
  p = fma2(s, p, splat2(kTp1));
  p = fma2(s, p, splat2(1.0f));
  float2v q = fma2(s, splat2(kTq3), splat2(kTq2));
  q = fma2(s, q, splat2(kTq1));
  q = fma2(s, q, splat2(1.0f));
  const float2v r = (x * p) * rcp2(q);
  return float2v{nan_pass(x0.x, r.x), nan_pass(x0.y, r.y)};
}
// Four-lane forms (two unit pairs at once): every operation splits into two independent packed
// halves, so dependent packed ops never sit back to back (no s_nop hazard padding) and the
// transcendentals come four at a time.  Same operation sequence: bitwise equal to the scalar forms.
typedef float float4v __attribute__((ext_vector_type(4)));
IADMM_DEV float4v splat4(float v) { return float4v{v, v, v, v}; }
IADMM_DEV float4v fma4(float4v a, float4v b, float4v c) { return __builtin_elementwise_fma(a, b, c); }
IADMM_DEV float4v exp2_4(float4v y) {
  return float4v{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y), __builtin_amdgcn_exp2f(y.z),
                 __builtin_amdgcn_exp2f(y.w)};
}
IADMM_DEV float4v rcp4(float4v d) {
  return float4v{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z),
                 __builtin_amdgcn_rcpf(d.w)};
}
IADMM_DEV float4v sigmoid_cell4(float4v x) { return rcp4(splat4(1.0f) + exp2_4(x * splat4(kNL2E))); }
IADMM_DEV float4v tanh_cell4(float4v x0) {
  const float4v x = float4v{__builtin_amdgcn_fmed3f(x0.x, -kTanhClamp, kTanhClamp),
                            __builtin_amdgcn_fmed3f(x0.y, -kTanhClamp, kTanhClamp),
                            __builtin_amdgcn_fmed3f(x0.z, -kTanhClamp, kTanhClamp),
                            __builtin_amdgcn_fmed3f(x0.w, -kTanhClamp, kTanhClamp)};
  const float4v s = x * x;
  float4v p = fma4(s, splat4(kTp6), splat4(kTp5));
  p = fma4(s, p, splat4(kTp4));
  p = fma4(s, p, splat4(kTp3));
  p = fma4(s, p, splat4(kTp2));
  p = fma4(s, p, splat4(kTp1));
  p = fma4(s, p, splat4(1.0f));
  float4v q = fma4(s, splat4(kTq3), splat4(kTq2));
  q = fma4(s, q, splat4(kTq1));
  q = fma4(s, q, splat4(1.0f));
  const float4v r = (x * p) * rcp4(q);
  return float4v{nan_pass(x0.x, r.x), nan_pass(x0.y, r.y), nan_pass(x0.z, r.z), nan_pass(x0.w, r.w)};
}
IADMM_DEV float4v cell_pre4(float4v in0, float4v in1, float4v acc, float4v w0, float4v w1, float4v b) {
  return fma4(in1, w1, fma4(in0, w0, b)) + acc;
}
IADMM_DEV float2v cell_pre2(float2v in0, float2v in1, float2v acc, float2v w0, float2v w1, float2v b) {
  return fma2(in1, w1, fma2(in0, w0, b)) + acc;
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

#define IADMM_HIP_RC(call)                            \
  do {                                                \
    hipError_t e_ = (call);                           \
    if (e_ != hipSuccess) return static_cast<int>(e_); \
  } while (0)
