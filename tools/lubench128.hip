// Variant microbenchmark of the fused TRSM + rank-128 trailing update at the Stage-II bench shape
// (B = 1024, N = 2000), outer blocks P = 0 and P = 896: hipEvent time of lu_trail128_kernel (the
// product kernel, lu.hip) and of the wave-specialised lu_trail128ws_kernel below (r04, rejected:
// bitwise equal but 6 % slower; the memory waves' VALU starves beside the MFMA stream), each in full, without MFMAs (DIAG 1: the
// memory / LDS pipeline alone) and without the main loop's global traffic (DIAG 2: MFMA + LDS +
// barriers alone); and a bitwise comparison of the two kernels' outputs on the same input.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lubench128.hip -o tools/lubench128.bin
#include "../i-admm-lstm_amd/csrc/lu.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace iadmm {
// ---- the r04 wave-specialised variant (rejected, DESIGN.md §5b: profiles/r04f_lubench128_ws.txt) ----
// Wave-specialised form of lu_trail128_kernel (r04), same arithmetic bit for bit.  The r03 kernel
// ran every wave through "loads, MFMAs, barrier, output": the memory and MFMA phases of one 8-wave
// workgroup (the only one on its CU: 143 KB of LDS) overlapped only partly, ~14.6 k cycles per
// 64-row step against 8.2 k of MFMA issue per SIMD.  Here waves 0-3 (one per SIMD) only compute
// and waves 4-7 only move data, with one barrier per step:
//   MFMA wave w, interval t:    columns [32w, 32w + 32) of step t, both 32-row halves (two
//                               accumulators, U12 operand in registers as before, -L21 from
//                               Ls[t & 1]), the product -> Cb[t & 1];
//   memory waves, interval t:   issue the loads of A22 (t) and L21 (t + 2); the output of step t - 1
//                               (A22 (t - 1), loaded during interval t - 1, minus Cb[(t - 1) & 1]);
//                               L21 (t + 1), loaded during interval t - 1, -> Ls[(t + 1) & 1];
//   barrier.
// The MFMA waves issue no global access and no VALU beyond their fragment reads; everything the
// memory waves wait for was issued one interval (one step of MFMAs) earlier.  Per tile the MFMA
// chain, the product and out = A22 - product are those of lu_trail128_kernel, so the factors are
// bitwise the same.  (VEC path only: N % 4 == 0 and 16-B aligned rows.)
// DIAG (tools/lubench128.hip only): 1 = no MFMAs, 2 = no global A22 / L21 traffic in the main loop.
constexpr int kWSThreads = 768;  // 4 MFMA waves + 8 memory waves (two per SIMD)
constexpr int kWSMaxN = 32767;   // the LDS-DMA buffer spans one instance: N * N * 4 < 2^32
template <int DIAG = 0>
__global__ __launch_bounds__(kWSThreads, 1) void lu_trail128ws_kernel(int N, int P, int ntc, float* A,
                                                                      const float* Linv, const int* perm) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ls0 = sm;
  float* Cb0 = sm + 2 * kT2S * kT2K;
  float* Ut = Ls0;
  float* Li = Cb0;
  int* bsrc = reinterpret_cast<int*>(Cb0 + 2 * kT2S * kT2CS);
  int* tdst = bsrc + kPermMax;
  int* tsrc = tdst + kPermMax;
  int* ddst = tsrc + kPermMax;
  int* dsrc = ddst + kPermMax;
  unsigned* dbits = reinterpret_cast<unsigned*>(dsrc + kPermMax);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, local = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int logical = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  const size_t b = (size_t)(logical / ntc);
  const int tc = logical % ntc;
  float* Ab = A + b * (size_t)N * N;
  const int c0 = P + kOB, cb = c0 + tc * kT2C;
  const int nsteps = (N - c0 + kT2S - 1) / kT2S;
  const int tid = threadIdx.x, lane = tid & 63, il = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int NT = kT2Threads;

  // ---- the permutation (as lu_trail128_kernel)
  const int ndisp = perm ? perm[b * kPermInts + 4 * kPermMax] - kOB : 0;
  {
    const int* pb = perm + b * kPermInts;
    if (tid < kOB) bsrc[tid] = perm ? pb[2 * kPermMax + tid] : P + tid;
    if (tid < ndisp) { tdst[tid] = pb[kOB + tid]; tsrc[tid] = pb[2 * kPermMax + kOB + tid]; }
    for (int w = tid; w < 2 * nsteps + 2; w += kWSThreads) dbits[w] = 0u;
  }
  __syncthreads();
  if (tid < ndisp) {
    const int d = tdst[tid];
    int rank = 0;
    for (int j = 0; j < ndisp; ++j) rank += tdst[j] < d;
    ddst[rank] = d;
    dsrc[rank] = tsrc[tid];
    atomicOr(&dbits[(d - c0) >> 5], 1u << ((d - c0) & 31));
  }
  auto src_row = [&](int row, int ro, unsigned long long m) __attribute__((always_inline)) -> int {
    if (!((m >> ro) & 1ull)) return row;
    int lo = 0, hi = ndisp - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (ddst[mid] < row) lo = mid + 1; else hi = mid;
    }
    return dsrc[lo];
  };

  // ---- prologue: U12 = L11^-1 A12 on this strip (waves 0-7, as lu_trail128_kernel)
  constexpr int CPR = kT2C / 4, LPR = kOB / 4;
  const bool pro = tid < NT;
#pragma unroll
  for (int q = 0; q < kOB * kT2C / 4 / NT; ++q) {
    if (!pro) break;
    const int e = tid + NT * q, k = e / CPR, cl = (e % CPR) * 4, col = cb + cl;
    const float4 x = *reinterpret_cast<const float4*>(Ab + (size_t)bsrc[k] * N + min(col, N - 4));
    const float4 u = col < N ? x : make_float4(0.f, 0.f, 0.f, 0.f);
    Ut[(cl + 0) * kT2K + k] = u.x; Ut[(cl + 1) * kT2K + k] = u.y;
    Ut[(cl + 2) * kT2K + k] = u.z; Ut[(cl + 3) * kT2K + k] = u.w;
  }
  const float* Lb = Linv + b * (size_t)kLinvFloats;
#pragma unroll
  for (int q = 0; q < kOB * kOB / 4 / NT; ++q) {
    if (!pro) break;
    const int e = tid + NT * q, i = e / (kOB / 4), kk = (e % (kOB / 4)) * 4;
    *reinterpret_cast<float4*>(Li + i * kT2K + kk) = *reinterpret_cast<const float4*>(Lb + (size_t)i * kOB + kk);
  }
  __syncthreads();
  floatx16 pu0, pu1;
  if (pro) {
    const int ti = wave >> 1, tj0 = 2 * (wave & 1);
    floatx16 u0, u1;
#pragma unroll
    for (int v = 0; v < 16; ++v) { u0[v] = 0.f; u1[v] = 0.f; }
#pragma unroll 4
    for (int sg = 0; sg < kOB / 8; ++sg) {
      const float4 fa = *reinterpret_cast<const float4*>(Li + (ti * 32 + il) * kT2K + (kOB / 2) * h + 4 * sg);
      const float4 f0 = *reinterpret_cast<const float4*>(Ut + (tj0 * 32 + il) * kT2K + (kOB / 2) * h + 4 * sg);
      const float4 f1 = *reinterpret_cast<const float4*>(Ut + (tj0 * 32 + 32 + il) * kT2K + (kOB / 2) * h + 4 * sg);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        u0 = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(fa, s4), get4(f0, s4), u0, 0, 0, 0);
        u1 = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(fa, s4), get4(f1, s4), u1, 0, 0, 0);
      }
    }
    pu0 = u0;
    pu1 = u1;
  }
  __syncthreads();  // A12^T and L11^-1 consumed
  if (pro) {
    const int ti = wave >> 1, tj0 = 2 * (wave & 1);
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int i = ti * 32 + 8 * (v >> 2) + 4 * h + (v & 3);
      Ut[(tj0 * 32 + il) * kT2K + i] = pu0[v];
      Ut[(tj0 * 32 + 32 + il) * kT2K + i] = pu1[v];
    }
  }
  __syncthreads();
  const bool mfma_wave = wave < 4;
  const int wc = (wave & 3) * 32;
  float4 ub[kOB / 8];  // MFMA waves: U12[64h + 4sg + 0..3][wc + il] for every step
  if (mfma_wave) {
#pragma unroll
    for (int sg = 0; sg < kOB / 8; ++sg)
      ub[sg] = *reinterpret_cast<const float4*>(Ut + (wc + il) * kT2K + (kOB / 2) * h + 4 * sg);
  }
  __syncthreads();  // Ut consumed: Ls from here on

  // ---- memory waves: 512 threads, 4 float4 of A22 per thread and step; L21 goes HBM/L2 -> LDS by
  // LDS-DMA (buffer_load_dwordx4 ... lds, no registers): Ls rows are 128 floats, unpadded, their
  // 16-B chunks XOR-swizzled by (row & 15) on the source address (the DMA image is lane-linear), so
  // the MFMA waves' fragment ds_read_b128 is conflict-free.  The buffer is based at the instance
  // (offsets < 2^32: N <= kWSMaxN), rows >= N read as zero through its range check.
  constexpr int MT = kWSThreads - 256;
  constexpr int MQ = kT2S * kT2C / 4 / MT;
  constexpr int kLS = kOB;                       // LDS row stride of the DMA'd -L21 tiles
  constexpr int LPW = kT2S / 2 / (MT / 64);      // DMA instructions (two rows each) per memory wave
  const int mt = tid - 256, mw = (tid >> 6) - 4;
  const __amdgpu_buffer_rsrc_t lrs =
      __builtin_amdgcn_make_buffer_rsrc(Ab, 0, (int)((unsigned)N * (unsigned)N * 4u), 0x00020000);
  unsigned loff[LPW];
#pragma unroll
  for (int i = 0; i < LPW; ++i) {
    const int rl = 2 * (mw * LPW + i) + (lane >> 5), c = (lane & 31) ^ (rl & 15);
    loff[i] = (unsigned)rl * (unsigned)N * 4u + (unsigned)(P + 4 * c) * 4u;
  }
  auto issueL = [&](int step) __attribute__((always_inline)) {
    float* Ls = Ls0 + (step & 1) * (kT2S * kLS);
    const unsigned so = (unsigned)(c0 + step * kT2S) * (unsigned)N * 4u;
#pragma unroll
    for (int i = 0; i < LPW; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(lrs, (lds_void*)(Ls + 2 * (mw * LPW + i) * kLS), 16, loff[i], so, 0, 0);
  };
  auto loadC = [&](int step, float4 (&c)[MQ]) __attribute__((always_inline)) {
    const unsigned long long m = *reinterpret_cast<const unsigned long long*>(dbits + 2 * step);
    // the source rows first (the binary search is a divergent loop), then every load at once
    int src[MQ];
#pragma unroll
    for (int q = 0; q < MQ; ++q) {
      const int e = mt + MT * q, ro = e / CPR, row = c0 + step * kT2S + ro;
      src[q] = min(src_row(row, ro, m), N - 1);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < MQ; ++q) {
      const int e = mt + MT * q, col = cb + (e % CPR) * 4;
      c[q] = *reinterpret_cast<const float4*>(Ab + (size_t)src[q] * N + min(col, N - 4));
    }
  };
  auto storeOut = [&](int step, float4 (&c)[MQ]) __attribute__((always_inline)) {
    const float* Cb = Cb0 + (step & 1) * (kT2S * kT2CS);
#pragma unroll
    for (int q = 0; q < MQ; ++q) {
      const int e = mt + MT * q, row = c0 + step * kT2S + e / CPR, col = cb + (e % CPR) * 4;
      const float4 pr = *reinterpret_cast<const float4*>(Cb + (e / CPR) * kT2CS + (e % CPR) * 4);
      c[q].x -= pr.x; c[q].y -= pr.y; c[q].z -= pr.z; c[q].w -= pr.w;
      if (row < N && col < N) *reinterpret_cast<float4*>(Ab + (size_t)row * N + col) = c[q];
    }
  };
  // ---- MFMA waves: product of step t -> Cb[t & 1]
  const int sw = il & 15;
  auto product = [&](int step) __attribute__((always_inline)) {
    const float* Ls = Ls0 + (step & 1) * (kT2S * kLS);
    float* Cb = Cb0 + (step & 1) * (kT2S * kT2CS);
    floatx16 a0, a1;
#pragma unroll
    for (int v = 0; v < 16; ++v) { a0[v] = 0.f; a1[v] = 0.f; }
    if constexpr (DIAG != 1) {
      // logical 16-B chunk 16h + sg of rows il and 32 + il sits at chunk 16h + (sg ^ (il & 15));
      // fragments double-buffered by hand (one MFMA wave per SIMD: nothing else fills a stall)
      const float* l0 = Ls + il * kLS + (kOB / 2) * h;
      const float* l1 = l0 + 32 * kLS;
      float4 f0 = *reinterpret_cast<const float4*>(l0 + 4 * sw), f1 = *reinterpret_cast<const float4*>(l1 + 4 * sw);
#pragma unroll
      for (int sg = 0; sg < kOB / 8; ++sg) {
        float4 g0 = f0, g1 = f1;
        if (sg + 1 < kOB / 8) {
          g0 = *reinterpret_cast<const float4*>(l0 + 4 * ((sg + 1) ^ sw));
          g1 = *reinterpret_cast<const float4*>(l1 + 4 * ((sg + 1) ^ sw));
        }
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(f0, s4), get4(ub[sg], s4), a0, 0, 0, 0);
          a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(f1, s4), get4(ub[sg], s4), a1, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        f0 = g0;
        f1 = g1;
      }
    }
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int r = 8 * (v >> 2) + 4 * h + (v & 3);
      Cb[r * kT2CS + wc + il] = a0[v];
      Cb[(32 + r) * kT2CS + wc + il] = a1[v];
    }
  };

  if (mfma_wave) {
    __syncthreads();  // Ls[0] = L21 (0)
    for (int step = 0; step < nsteps; ++step) {
      product(step);
      __syncthreads();
    }
    __syncthreads();  // the memory waves' drain interval
  } else {
    // interval t: L21 (t + 1) -> Ls[(t + 1) & 1] (DMA, issued first); the loads of A22 (t); the
    // output of step t - 1 (A22 loaded in interval t - 1); wait for the DMA; barrier.
    // Unrolled by two so the A22 register sets are static.
    float4 ca[MQ], cbk[MQ];
    if (DIAG != 2) issueL(0);
    vm_wait<0>();
    __syncthreads();
    auto interval = [&](int step, float4 (&cur)[MQ], float4 (&prv)[MQ], bool out) __attribute__((always_inline)) {
      if (DIAG != 2) {
        issueL(step + 1);
        loadC(step, cur);
        if (out) storeOut(step - 1, prv);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (out) vm_wait<2 * MQ>();  // (the DMA, then MQ loads and MQ stores)
      else vm_wait<MQ>();
      __syncthreads();
    };
    interval(0, ca, cbk, false);
    int step = 1;
    for (; step + 1 < nsteps; step += 2) {
      interval(step, cbk, ca, true);
      interval(step + 1, ca, cbk, true);
    }
    if (step < nsteps) {
      interval(step, cbk, ca, true);
      ++step;
      if (DIAG != 2) storeOut(step - 1, cbk);
    } else {
      if (DIAG != 2) storeOut(step - 1, ca);
    }
    __syncthreads();  // (pairs with the MFMA waves' drain barrier)
  }
  __syncthreads();  // every gathered load of a block row has completed: U12 to the block rows
  if (mfma_wave && cb + wc + il < N) {
#pragma unroll
    for (int sg = 0; sg < kOB / 8; ++sg) {
      const int i = (kOB / 2) * h + 4 * sg;
      float* dst = Ab + (size_t)(P + i) * N + cb + wc + il;
      dst[0] = ub[sg].x;
      dst[(size_t)N] = ub[sg].y;
      dst[2 * (size_t)N] = ub[sg].z;
      dst[3 * (size_t)N] = ub[sg].w;
    }
  }
}

}  // namespace iadmm
using namespace iadmm;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill(float* p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 1e-3f * (float)((i * 2654435761u) & 1023) - 0.5f;
}

template <int WS, int DIAG>
void launch(int B, int N, int P, float* A, float* Linv) {
  const int ntc = (N - P - kOB + kT2C - 1) / kT2C;
  if (WS) hipLaunchKernelGGL((lu_trail128ws_kernel<DIAG>), dim3(B * ntc), dim3(kWSThreads), kT2Lds, 0, N, P, ntc, A, Linv, nullptr);
  else hipLaunchKernelGGL((lu_trail128_kernel<true, DIAG>), dim3(B * ntc), dim3(kT2Threads), kT2Lds, 0, N, P, ntc, A, Linv, nullptr);
}

template <int WS, int DIAG>
float run(int B, int N, int P, float* A, float* Linv, int reps) {
  if (WS) CK(hipFuncSetAttribute((const void*)lu_trail128ws_kernel<DIAG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kT2Lds));
  else CK(hipFuncSetAttribute((const void*)lu_trail128_kernel<true, DIAG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kT2Lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  launch<WS, DIAG>(B, N, P, A, Linv);
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch<WS, DIAG>(B, N, P, A, Linv);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024, N = argc > 2 ? atoi(argv[2]) : 2000;
  float *A, *A2, *Linv;
  const size_t n = (size_t)B * N * N;
  CK(hipMalloc(&A, n * sizeof(float)));
  CK(hipMalloc(&A2, n * sizeof(float)));
  CK(hipMalloc(&Linv, (size_t)B * kLinvFloats * sizeof(float)));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, Linv, (int64_t)B * kLinvFloats);
  // bitwise: one launch of each kernel on the same input
  for (int P : {0, 896, N - kOB - 64}) {
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, A, (int64_t)n);
    CK(hipMemcpy(A2, A, n * sizeof(float), hipMemcpyDeviceToDevice));
    CK(hipFuncSetAttribute((const void*)lu_trail128ws_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kT2Lds));
    CK(hipFuncSetAttribute((const void*)lu_trail128_kernel<true, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kT2Lds));
    launch<0, 0>(B, N, P, A, Linv);
    launch<1, 0>(B, N, P, A2, Linv);
    CK(hipDeviceSynchronize());
    const size_t chk = (size_t)4 * N * N;  // first four instances
    std::vector<unsigned> h1(chk), h2(chk);
    CK(hipMemcpy(h1.data(), A, chk * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), A2, chk * 4, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (size_t i = 0; i < chk; ++i) diff += h1[i] != h2[i];
    std::vector<unsigned> t1(N * N), t2(N * N);  // the last instance (every XCD mapping position)
    CK(hipMemcpy(t1.data(), A + (size_t)(B - 1) * N * N, (size_t)N * N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(t2.data(), A2 + (size_t)(B - 1) * N * N, (size_t)N * N * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < (size_t)N * N; ++i) diff += t1[i] != t2[i];
    printf("P=%4d bitwise r03 vs ws: %zu differing words (instances 0-3 and %d)\n", P, diff, B - 1);
  }
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, A, (int64_t)n);
  CK(hipDeviceSynchronize());
  for (int P : {0, 896}) {
    const double rest = N - P - kOB;
    const double bytes = (double)B * 4.0 * (2 * rest * rest + rest * kOB + 2 * kOB * rest);
    const double flops = (double)B * 2.0 * (rest * rest * kOB + kOB * kOB * rest);
    const char* names[3] = {"full", "no-mfma", "no-global"};
    for (int round = 0; round < 2; ++round) {
      float t[6] = {run<0, 0>(B, N, P, A, Linv, 5), run<0, 1>(B, N, P, A, Linv, 5), run<0, 2>(B, N, P, A, Linv, 5),
                    run<1, 0>(B, N, P, A, Linv, 5), run<1, 1>(B, N, P, A, Linv, 5), run<1, 2>(B, N, P, A, Linv, 5)};
      for (int v = 0; v < 6; ++v)
        printf("P=%4d %-3s %-10s %8.3f ms  %7.0f GB/s alg  %6.1f TF\n", P, v < 3 ? "r03" : "ws", names[v % 3], t[v],
               bytes / t[v] / 1e6, flops / t[v] / 1e9);
    }
  }
  CK(hipFree(A)); CK(hipFree(A2)); CK(hipFree(Linv));
  return 0;
}
