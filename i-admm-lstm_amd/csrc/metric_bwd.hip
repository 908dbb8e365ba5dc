// Backward of the reporting metrics (reference utils.py:53-60: obj_fn, ineq_dist, eq_dist), the two
// batched primitives their gradients need beside the forward matvec (iadmm_bmv):
//   iadmm_bmv_t  out[b] = M[b]^T v[b]          d/dx of ineq_dist / eq_dist (G^T w, A^T w) and
//                                              the Q^T (x g / 2) half of d/dx obj_fn
//   iadmm_bger   out[b] (+)= u[b] v[b]^T       d/dG, d/dA, d/dQ (rank-1 per instance)
// Both are HBM-bound streams of the [B, R, C] matrix (read once / written once).
#include "common.h"

namespace iadmm {

constexpr int kBmvtThreads = 256;
constexpr int kBmvtCols = 4 * kBmvtThreads;  // columns per workgroup (4 per thread)

// One workgroup per (instance, 1024-column strip); thread t owns columns 4t..4t+3 of the strip and
// walks the R rows in order (16-B loads, the row loop unrolled so 8 loads are in flight): every
// output is a fixed-order fma chain over r, so results do not depend on B or on the launch.  v[b]
// is staged once in LDS (broadcast reads).
template <bool VEC>
__global__ __launch_bounds__(kBmvtThreads) void bmv_t_kernel(int R, int C, const float* __restrict__ M,
                                                            const float* __restrict__ v, float* __restrict__ out) {
  extern __shared__ float vs[];
  const size_t b = blockIdx.x;
  const float* Mb = M + b * (size_t)R * C;
  for (int r = threadIdx.x; r < R; r += blockDim.x) vs[r] = v[b * (size_t)R + r];
  __syncthreads();
  const int c0 = blockIdx.y * kBmvtCols + 4 * threadIdx.x;
  if (c0 >= C) return;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if constexpr (VEC) {
    const float* p = Mb + c0;
#pragma unroll 8
    for (int r = 0; r < R; ++r) {
      const float4 m = *reinterpret_cast<const float4*>(p + (size_t)r * C);
      const float s = vs[r];
      a0 = fmaf(m.x, s, a0); a1 = fmaf(m.y, s, a1); a2 = fmaf(m.z, s, a2); a3 = fmaf(m.w, s, a3);
    }
    *reinterpret_cast<float4*>(out + b * (size_t)C + c0) = make_float4(a0, a1, a2, a3);
  } else {
    const int nc = min(4, C - c0);
#pragma unroll 4
    for (int r = 0; r < R; ++r) {
      const float* row = Mb + (size_t)r * C + c0;
      const float s = vs[r];
      a0 = fmaf(row[0], s, a0);
      if (nc > 1) a1 = fmaf(row[1], s, a1);
      if (nc > 2) a2 = fmaf(row[2], s, a2);
      if (nc > 3) a3 = fmaf(row[3], s, a3);
    }
    float* o = out + b * (size_t)C + c0;
    o[0] = a0;
    if (nc > 1) o[1] = a1;
    if (nc > 2) o[2] = a2;
    if (nc > 3) o[3] = a3;
  }
}

// out[b, r, c] = (acc ? out[b, r, c] : 0) + u[b, r] * v[b, c]; grid-stride over float4 groups of
// a row (VEC: C % 4 == 0 and 16-B aligned out) or single elements.
template <bool VEC>
__global__ __launch_bounds__(256) void bger_kernel(int64_t B, int R, int C, const float* __restrict__ u,
                                                   const float* __restrict__ v, int acc, float* __restrict__ out) {
  const int W = VEC ? 4 : 1;
  const int64_t per_row = C / W, per_b = (int64_t)R * per_row, tot = B * per_b;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < tot; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = k / per_b;
    const int64_t rem = k - b * per_b;
    const int r = (int)(rem / per_row);
    const int c = (int)(rem - (int64_t)r * per_row) * W;
    const float ur = u[b * R + r];
    float* o = out + (b * R + r) * (int64_t)C + c;
    if constexpr (VEC) {
      const float4 vv = *reinterpret_cast<const float4*>(v + b * C + c);
      float4 y = make_float4(ur * vv.x, ur * vv.y, ur * vv.z, ur * vv.w);
      if (acc) {
        const float4 p = *reinterpret_cast<const float4*>(o);
        y = make_float4(p.x + y.x, p.y + y.y, p.z + y.z, p.w + y.w);
      }
      *reinterpret_cast<float4*>(o) = y;
    } else {
      const float y = ur * v[b * C + c];
      *o = acc ? *o + y : y;
    }
  }
}

}  // namespace iadmm

using namespace iadmm;

extern "C" int iadmm_bmv_t(int64_t B, int64_t R, int64_t C, const float* M, const float* v, float* out,
                           void* stream) {
  if (B <= 0 || R <= 0 || C <= 0 || !M || !v || !out) return IADMM_E_ARG;
  const size_t lds = (size_t)R * sizeof(float);
  if (lds > 160 * 1024 || B > 0x7fffffff || C > 0x7fffffff) return IADMM_E_SIZE;
  const dim3 grid((unsigned)B, (unsigned)((C + kBmvtCols - 1) / kBmvtCols));
  hipStream_t s = (hipStream_t)stream;
  if (C % 4 == 0 && aligned16(M) && aligned16(out)) {
    IADMM_ALLOW_LDS(bmv_t_kernel<true>, lds);
    hipLaunchKernelGGL(bmv_t_kernel<true>, grid, dim3(kBmvtThreads), lds, s, (int)R, (int)C, M, v, out);
  } else {
    IADMM_ALLOW_LDS(bmv_t_kernel<false>, lds);
    hipLaunchKernelGGL(bmv_t_kernel<false>, grid, dim3(kBmvtThreads), lds, s, (int)R, (int)C, M, v, out);
  }
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_bger(int64_t B, int64_t R, int64_t C, const float* u, const float* v, int accumulate,
                          float* out, void* stream) {
  if (B <= 0 || R <= 0 || C <= 0 || !u || !v || !out) return IADMM_E_ARG;
  if (R > 0x7fffffff || C > 0x7fffffff) return IADMM_E_SIZE;
  const bool vec = C % 4 == 0 && aligned16(out) && aligned16(v);
  const int64_t tot = B * R * (vec ? C / 4 : C);
  const int64_t blocks = (tot + 255) / 256;
  const dim3 grid((unsigned)(blocks < 65536 ? blocks : 65536));
  hipStream_t s = (hipStream_t)stream;
  if (vec) hipLaunchKernelGGL(bger_kernel<true>, grid, dim3(256), 0, s, B, (int)R, (int)C, u, v, accumulate, out);
  else hipLaunchKernelGGL(bger_kernel<false>, grid, dim3(256), 0, s, B, (int)R, (int)C, u, v, accumulate, out);
  IADMM_CHECK_LAUNCH();
  return 0;
}
