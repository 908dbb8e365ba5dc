// Does v_mfma_f32_32x32x2_f32 round each product before accumulating (unlike an FMA)?  acc =
// -(1 + 2^-22) + (1 + 2^-23)^2: an exact (fused) product leaves 2^-46, a rounded product 0.  Also the
// same with the product in the second k slot, and the VALU fmaf for comparison.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_fma_check.hip -o tools/mfma_fma_check.bin
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ void k(float* out, float a, float c) {
  const int lane = threadIdx.x;
  floatx16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = c;
  const int kslot = lane >> 5;
  floatx16 r0 = __builtin_amdgcn_mfma_f32_32x32x2f32(kslot == 0 ? a : 0.f, kslot == 0 ? a : 0.f, acc, 0, 0, 0);
  floatx16 r1 = __builtin_amdgcn_mfma_f32_32x32x2f32(kslot == 1 ? a : 0.f, kslot == 1 ? a : 0.f, acc, 0, 0, 0);
  // two products that cancel exactly: a*a - a*a + c with both in one instruction
  floatx16 r2 = __builtin_amdgcn_mfma_f32_32x32x2f32(kslot == 0 ? a : -a, a, acc, 0, 0, 0);
  if (lane == 0) {
    out[0] = r0[0];
    out[1] = r1[0];
    out[2] = r2[0];
    out[3] = fmaf(a, a, c);
    out[4] = __fadd_rn(__fmul_rn(a, a), c);
  }
}

int main() {
  float* d;
  hipMalloc(&d, 64);
  const float a = 1.0f + 0x1p-23f, c = -(1.0f + 0x1p-22f);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, a, c);
  float h[5];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  printf("mfma k0: %a  mfma k1: %a  mfma a*a-a*a+c: %a  fmaf: %a  mul+add: %a  (exact 0x1p-46)\n", h[0], h[1], h[2],
         h[3], h[4]);
  return 0;
}
