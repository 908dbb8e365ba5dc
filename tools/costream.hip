// Co-residency probe (tools/costream.py): a one-wave, register-lean streaming reader that can sit
// beside the cell kernel's two workgroups on a CU (they leave 48 VGPRs per SIMD and 12 KiB of LDS
// free).  Each workgroup sums a contiguous chunk of `chunk` floats with 16-B loads, INFL of them
// in flight per lane, and writes one float.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int INFL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(40))) void stream_read_kernel(
    const float4* __restrict__ p, int64_t chunk4, float* out) {
  const float4* c = p + (int64_t)blockIdx.x * chunk4;
  const int lane = threadIdx.x;
  float acc = 0.f;
  for (int64_t i = lane; i < chunk4; i += 64 * INFL) {
    float4 v[INFL];
#pragma unroll
    for (int u = 0; u < INFL; ++u) v[u] = (i + 64 * u < chunk4) ? c[i + 64 * u] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < INFL; ++u) acc += (v[u].x + v[u].y) + (v[u].z + v[u].w);
  }
  if (acc == 12345.678f) out[blockIdx.x] = acc;  // keep the loads alive, write nothing in practice
}

extern "C" int costream_read(const float* p, int64_t nfloats, int64_t chunk, int infl, float* out, void* stream) {
  const int64_t nwg = nfloats / chunk;
  hipStream_t s = (hipStream_t)stream;
  if (infl == 2)
    hipLaunchKernelGGL(stream_read_kernel<2>, dim3((unsigned)nwg), dim3(64), 0, s, (const float4*)p, chunk / 4, out);
  else if (infl == 4)
    hipLaunchKernelGGL(stream_read_kernel<4>, dim3((unsigned)nwg), dim3(64), 0, s, (const float4*)p, chunk / 4, out);
  else
    hipLaunchKernelGGL(stream_read_kernel<6>, dim3((unsigned)nwg), dim3(64), 0, s, (const float4*)p, chunk / 4, out);
  return (int)hipGetLastError();
}
