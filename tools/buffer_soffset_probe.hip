// Is a buffer store's SGPR offset (soffset) part of the descriptor's range check on gfx950?
// Descriptor over the first 256 B of a 4 KiB zeroed buffer; lane 0 stores 1.0 with voffset 0 and
// soffset 512 (in range without soffset, out of range with it); lane 1 voffset 512, soffset 0
// (out of range either way).  Prints what landed at bytes 512 and 516.
// Build: hipcc -O3 --offload-arch=gfx950 tools/buffer_soffset_probe.hip -o tools/buffer_soffset_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(float* p, int so) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, 0, 256, 0x00020000);
  const int lane = threadIdx.x;
  if (lane == 0) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(1.0f), r, 0u, so, 0);
  if (lane == 1) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(2.0f), r, 516u, 0, 0);
  if (lane == 2) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(3.0f), r, 8u, 0, 0);
}
int main() {
  float* d; hipMalloc(&d, 4096); hipMemset(d, 0, 4096);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 512);
  float h[1024]; hipMemcpy(h, d, 4096, hipMemcpyDeviceToHost);
  printf("byte 8 (in range): %g | byte 512 (voffset 0 + soffset 512): %g | byte 516 (voffset 516): %g\n", h[2], h[128], h[129]);
  printf("soffset %s the range check\n", h[128] == 0.f ? "IS part of" : "is NOT part of");
  return 0;
}
