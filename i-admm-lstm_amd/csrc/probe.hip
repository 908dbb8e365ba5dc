// Box-ceiling probes: the fp32 MFMA rate and the HBM copy rate THIS box
// delivers, measured in-process before the bench's timed steps, so a headline fraction can be
// read against the box as well as against the spec (MI355X boxes differ by a few % in clock and
// HBM).  Not on the solve path.
//
//   probe_mfma_kernel  every wave streams v_mfma_f32_32x32x2_f32 on 8 independent accumulators
//                      from registers (no memory in the loop): 4096 flop per MFMA per wave; two
//                      4-wave workgroups per CU = 2 waves per SIMD, the cell kernel's residency.
//   probe_copy_kernel  float4 copy, one contiguous chunk per workgroup (16-B accesses, 8 in flight per thread).
//   probe_read_kernel  float4 read-only sweep (the residual matvec's access: 16-B loads, one contiguous
//                      chunk per workgroup), UNROLL loads in flight per thread, at a chosen number of
//                      workgroups per CU (r05: the copy alone, 5.3 TB/s, sat below the matvec's own
//                      5.65 TB/s of reads, so it was no ceiling for it; bench.py takes the best shape).
#include <algorithm>

#include "common.h"

namespace iadmm {

typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256, 2) void probe_mfma_kernel(int iters, float* out) {
  const int tid = threadIdx.x, lane = tid & 63;
  const float a = 1e-3f * (float)(lane + 1), b = 2e-3f * (float)(lane + 3);
  floatx16 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[j][q] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) s += acc[j][q];
  out[(size_t)blockIdx.x * blockDim.x + tid] = s;
}

__global__ __launch_bounds__(256) void probe_copy_kernel(int64_t n4, const float4* __restrict__ src,
                                                         float4* __restrict__ dst) {
  // each workgroup streams one contiguous chunk, 8 x 1 KiB per wave in flight (the KKT sweeps'
  // access shape; a grid-stride form touching 8 far-apart windows per thread measured 0.56 of spec)
  const int64_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const int64_t c0 = (int64_t)blockIdx.x * per, c1 = c0 + per < n4 ? c0 + per : n4;
  int64_t i = c0 + threadIdx.x;
  for (; i + 7 * 256 < c1; i += 8 * 256) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[i + u * 256];
#pragma unroll
    for (int u = 0; u < 8; ++u) dst[i + u * 256] = v[u];
  }
  for (; i < c1; i += 256) dst[i] = src[i];
}

template <int UNROLL>
__global__ __launch_bounds__(256) void probe_read_kernel(int64_t n4, const float4* __restrict__ src, float* out) {
  const int64_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const int64_t c0 = (int64_t)blockIdx.x * per, c1 = c0 + per < n4 ? c0 + per : n4;
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v* s4 = reinterpret_cast<const f4v*>(src);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int64_t i = c0 + threadIdx.x;
  for (; i + (UNROLL - 1) * 256 < c1; i += UNROLL * 256) {
    f4v v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(s4 + i + u * 256);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
  }
  for (; i < c1; i += 256) { const float4 v = src[i]; acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w; }
  out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = (acc.x + acc.y) + (acc.z + acc.w);
}

}  // namespace iadmm

using namespace iadmm;

extern "C" int64_t iadmm_probe_mfma_flop(int64_t blocks, int64_t iters) {
  return blocks * 4 * iters * 8 * 4096;  // waves x MFMAs per wave x 32*32*2*2
}

extern "C" int iadmm_probe_mfma(int64_t blocks, int64_t iters, float* out, void* stream) {
  if (blocks <= 0 || iters <= 0 || iters > 0x7fffffff || blocks > 0x7fffffff || !out) return IADMM_E_ARG;
  hipLaunchKernelGGL(probe_mfma_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (int)iters, out);
  return (int)hipGetLastError();
}

extern "C" int iadmm_probe_copy(int64_t bytes, const void* src, void* dst, void* stream) {
  if (bytes <= 0 || !src || !dst) return IADMM_E_ARG;
  if ((bytes & 15) || (reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 15))
    return IADMM_E_ALIGN;
  const int64_t n4 = bytes / 16;
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t blocks = std::min<int64_t>((n4 + 255) / 256, (int64_t)cus * 8);
  hipLaunchKernelGGL(probe_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n4,
                     static_cast<const float4*>(src), static_cast<float4*>(dst));
  return (int)hipGetLastError();
}

extern "C" int iadmm_probe_read(int64_t bytes, const void* src, float* out, int64_t wg_per_cu, int64_t unroll,
                                void* stream) {
  if (bytes <= 0 || !src || !out || wg_per_cu <= 0 || wg_per_cu > 32 || (unroll != 8 && unroll != 16))
    return IADMM_E_ARG;
  if ((bytes & 15) || (reinterpret_cast<uintptr_t>(src) & 15)) return IADMM_E_ALIGN;
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t n4 = bytes / 16, blocks = (int64_t)cus * wg_per_cu;
  if (unroll == 8)
    hipLaunchKernelGGL(probe_read_kernel<8>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n4,
                       static_cast<const float4*>(src), out);
  else
    hipLaunchKernelGGL(probe_read_kernel<16>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n4,
                       static_cast<const float4*>(src), out);
  return (int)hipGetLastError();
}
