// Variant microbenchmark of the fused TRSM + rank-128 trailing update at the Stage-II bench shape
// (B = 1024, N = 2000), outer blocks P = 0 and P = 896: hipEvent time of the r03 kernel (below: one
// 8-wave workgroup per CU, 64-row steps) and of lu_trail128_kernel (lu.hip; r04: two 4-wave
// workgroups per CU, 32-row steps), each in full, without MFMAs (DIAG 1: the memory / LDS pipeline
// alone) and without the main loop's global traffic (DIAG 2: MFMA + LDS + barriers alone); and a
// bitwise comparison of the two kernels' outputs on the same input.  (perm = nullptr: the gathered
// interchanges are exercised by the Stage-II tests, not here.)
// Earlier variants: the r04 wave-specialised kernel (4 MFMA + 8 memory waves; bitwise equal, 6 %
// slower, profiles/r04_lubench128_ws_rejected.txt) is in this file's history.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lubench128.hip -o tools/lubench128.bin
#include "../i-admm-lstm_amd/csrc/lu.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace iadmm {
// ---- the r03 trailing-update kernel (one 8-wave workgroup per CU, 64-row steps, binary-search
// gather): the baseline of this benchmark, replaced in lu.hip by the paired form in r04 ----
constexpr int kR3S = 64;
constexpr int kR3Threads = 512;
constexpr int kR3BitWords = 2 * ((kLuMaxN + kR3S - 1) / kR3S) + 2;
constexpr size_t kR3Lds = (2 * (size_t)kR3S * kT2K + 2 * (size_t)kR3S * kT2CS) * sizeof(float) +
                          (size_t)(5 * kPermMax + kR3BitWords) * sizeof(int);
// Fused row interchanges, U12 = L11^-1 A12 and A22 -= L21 U12 (rank 128) for the columns right of
// [P, P + 128).  One workgroup (8 waves, one per CU) per (instance, 128-column strip), all trailing
// rows.  The block's 128 interchanges (composed by lu_block_perm_kernel: block row P + i takes row
// pcur[i], each displaced row below the block takes an original block row) get no pass of their
// own over these columns: the loads gather through the permutation, and the block rows -- the only
// sources of displaced rows -- are overwritten (with U12) after the last step's loads.
// (perm == nullptr: no interchanges, tools/lubench128.hip.)
//   prologue: the gathered A12 (128 x 128, transposed) and L11^-1 into LDS, U12 on MFMA (each wave
//             two 32 x 32 tiles), transposed into LDS, then each wave's MFMA operand of it -- column
//             wc + il, k in [64h, 64h + 64): 64 registers -- kept in registers for the whole loop;
//   main loop: 64-row steps; wave (wr, wc) owns 32 x 32 of a step (v_mfma_f32_32x32x2f32, 64 per
//             step, -L21 from LDS, U12 from registers).  -L21 and the product tile are
//             double-buffered in LDS, so a step needs ONE barrier: per wave, step t = issue the
//             loads of A22 (t + 1) and L21 (t + 2); the MFMAs; product -> Cb[t & 1]; L21 (t + 1)
//             -> Ls[(t + 1) & 1]; barrier; out = A22 - product for step t (row-contiguous 16-B
//             global stores, the A22 values already in the registers of the storing thread).  Waves
//             leave the barrier together but no longer wait for each other's output phase, which
//             runs beside other waves' MFMAs.
// Strips of one instance are consecutive logical ids on one XCD (its L2 serves the L21 re-reads).
// DIAG (tools/lubench128.hip only): 1 = no MFMAs in the main loop, 2 = no global A22 / L21 traffic in it.
template <bool VEC, int DIAG = 0>
__global__ __launch_bounds__(kR3Threads, 1) void lu_trail128_r03_kernel(int N, int P, int ntc, float* A,
                                                                    const float* Linv, const int* perm) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ls0 = sm;                      // 2 x [kR3S rows][kT2K]: -L21 of a step
  float* Cb0 = sm + 2 * kR3S * kT2K;    // 2 x [kR3S rows][kT2CS]: product of a step
  float* Ut = Ls0;                      // prologue: A12^T, then U12^T [kT2C cols][kT2K], over Ls
  float* Li = Cb0;                      // prologue: L11^-1 [128 rows][kT2K], over Cb
  int* bsrc = reinterpret_cast<int*>(Cb0 + 2 * kR3S * kT2CS);  // [128] source row of block row P + i
  int* tdst = bsrc + kPermMax;          // [128] displaced rows and
  int* tsrc = tdst + kPermMax;          // [128] their sources, as given;
  int* ddst = tsrc + kPermMax;          // [128] the same sorted by row
  int* dsrc = ddst + kPermMax;          // [128]
  unsigned* dbits = reinterpret_cast<unsigned*>(dsrc + kPermMax);  // 2 words per step: displaced rows
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, local = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int logical = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  const size_t b = (size_t)(logical / ntc);
  const int tc = logical % ntc;
  float* Ab = A + b * (size_t)N * N;
  const int c0 = P + kOB, cb = c0 + tc * kT2C;
  const int nsteps = (N - c0 + kR3S - 1) / kR3S;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, il = lane & 31, h = lane >> 5;
  constexpr int NT = kR3Threads;

  typedef typename std::conditional<VEC, float4, float>::type VT;
  constexpr int W = VEC ? 4 : 1;
  constexpr int kCQ = kR3S * kT2C / W / NT;   // A22 accesses per thread per step
  constexpr int kLQ = kR3S * kOB / W / NT;    // -L21 accesses per thread per step
  constexpr int kPQ = kOB * kT2C / W / NT;    // A12 / L11^-1 accesses per thread (prologue)
  constexpr int CPR = kT2C / W, LPR = kOB / W;
  // main-loop loads: unconditional, from a clamped (valid) address.  Rows >= N / columns >= N only
  // feed products that are never stored, so they need no zero fill -- and a load with no select
  // stays out of a branch, which keeps the compiler's vmcnt waits exact (a conditional load costs a
  // full vmcnt(0) drain at every later use).
  auto ldu = [&](int row, int col) -> VT {
    const float* p = Ab + (size_t)row * N + col;
    if constexpr (VEC) return *reinterpret_cast<const float4*>(p);
    else return *p;
  };
  auto ld = [&](int row, int col, bool ok) -> VT {
    const float* p = Ab + (size_t)row * N + col;
    if constexpr (VEC) {
      const float4 x = *reinterpret_cast<const float4*>(p);
      return ok ? x : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      const float x = *p;
      return ok ? x : 0.f;
    }
  };
  auto st_lds = [&](float* d, const VT& v) {
    if constexpr (VEC) *reinterpret_cast<float4*>(d) = v;
    else *d = v;
  };

  // ---- the permutation (displaced rows are >= c0 and distinct; <= 128 of them)
  const int ndisp = perm ? perm[b * kPermInts + 4 * kPermMax] - kOB : 0;
  {
    const int* pb = perm + b * kPermInts;
    if (tid < kOB) bsrc[tid] = perm ? pb[2 * kPermMax + tid] : P + tid;
    if (tid < ndisp) { tdst[tid] = pb[kOB + tid]; tsrc[tid] = pb[2 * kPermMax + kOB + tid]; }
    for (int w = tid; w < 2 * nsteps + 2; w += NT) dbits[w] = 0u;  // (+ the one-past-the-end step)
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
  // (published by the barrier after the prologue's LDS fills below)
  // source row of trailing row `row` (ro = row - the step's first row; m = that step's bitmap)
  auto src_row = [&](int row, int ro, unsigned long long m) -> int {
    if (!((m >> ro) & 1ull)) return row;
    int lo = 0, hi = ndisp - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (ddst[mid] < row) lo = mid + 1; else hi = mid;
    }
    return dsrc[lo];
  };

  // ---- prologue: U12 = L11^-1 A12 on this strip
#pragma unroll
  for (int q = 0; q < kPQ; ++q) {  // A12 -> Ut (transposed)
    const int e = tid + NT * q, k = e / CPR, cl = (e % CPR) * W, col = cb + cl;
    const VT u = ld(bsrc[k], min(col, N - W), col < N);
    if constexpr (VEC) {
      Ut[(cl + 0) * kT2K + k] = u.x; Ut[(cl + 1) * kT2K + k] = u.y;
      Ut[(cl + 2) * kT2K + k] = u.z; Ut[(cl + 3) * kT2K + k] = u.w;
    } else {
      Ut[cl * kT2K + k] = u;
    }
  }
  const float* Lb = Linv + b * (size_t)kLinvFloats;
#pragma unroll
  for (int q = 0; q < kOB * kOB / 4 / NT; ++q) {  // L11^-1 -> Li (rows, 16-B pieces)
    const int e = tid + NT * q, i = e / (kOB / 4), kk = (e % (kOB / 4)) * 4;
    *reinterpret_cast<float4*>(Li + i * kT2K + kk) = *reinterpret_cast<const float4*>(Lb + (size_t)i * kOB + kk);
  }
  __syncthreads();
  {
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
    __syncthreads();  // A12^T and L11^-1 consumed
    // accumulator v <-> row ti*32 + 8(v/4) + 4h + v%4 of U12, column tj*32 + il of the strip
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int i = ti * 32 + 8 * (v >> 2) + 4 * h + (v & 3);
      Ut[(tj0 * 32 + il) * kT2K + i] = u0[v];
      Ut[(tj0 * 32 + 32 + il) * kT2K + i] = u1[v];
    }
  }
  __syncthreads();
  const int wr = (wave >> 2) * 32, wc = (wave & 3) * 32;
  float4 ub[kOB / 8];  // U12[64h + 4sg + 0..3][wc + il]: this wave's MFMA operand for every step
#pragma unroll
  for (int sg = 0; sg < kOB / 8; ++sg)
    ub[sg] = *reinterpret_cast<const float4*>(Ut + (wc + il) * kT2K + (kOB / 2) * h + 4 * sg);
  __syncthreads();  // Ut consumed: Ls from here on

  // ---- main loop
  auto loadC = [&](int step, VT (&c)[kCQ]) {
    const unsigned long long m = *reinterpret_cast<const unsigned long long*>(dbits + 2 * step);
#pragma unroll
    for (int q = 0; q < kCQ; ++q) {
      const int e = tid + NT * q, ro = e / CPR, row = c0 + step * kR3S + ro, col = cb + (e % CPR) * W;
      c[q] = ldu(min(src_row(row, ro, m), N - 1), min(col, N - W));
    }
  };
  auto loadL = [&](int step, VT (&l)[kLQ]) {
#pragma unroll
    for (int q = 0; q < kLQ; ++q) {
      const int e = tid + NT * q, row = c0 + step * kR3S + e / LPR;
      l[q] = ldu(min(row, N - 1), P + (e % LPR) * W);
    }
  };
  auto writeL = [&](float* Ls, const VT (&l)[kLQ]) {
#pragma unroll
    for (int q = 0; q < kLQ; ++q) {
      const int e = tid + NT * q;
      st_lds(Ls + (e / LPR) * kT2K + (e % LPR) * W, l[q]);
    }
  };
  // (the result overwrites c in place and is stored from there: a store's data registers stay busy
  // until the store completes, and c is not reloaded until the next step but one)
  auto storeOut = [&](int step, const float* Cb, VT (&c)[kCQ]) {
#pragma unroll
    for (int q = 0; q < kCQ; ++q) {
      const int e = tid + NT * q, row = c0 + step * kR3S + e / CPR, col = cb + (e % CPR) * W;
      const float* src = Cb + (e / CPR) * kT2CS + (e % CPR) * W;
      if constexpr (VEC) {
        const float4 pr = *reinterpret_cast<const float4*>(src);
        c[q].x -= pr.x; c[q].y -= pr.y; c[q].z -= pr.z; c[q].w -= pr.w;
      } else {
        c[q] -= *src;
      }
      if (row < N && col < N) {
        if constexpr (VEC) *reinterpret_cast<float4*>(Ab + (size_t)row * N + col) = c[q];
        else Ab[(size_t)row * N + col] = c[q];
      }
    }
  };

  // step t (cc = A22 (t), loaded during step t - 1; lw = L21 (t + 1), loaded during step t - 1)
  auto body = [&](int step, VT (&cc)[kCQ], VT (&cn)[kCQ], const VT (&lw)[kLQ], VT (&lnext)[kLQ]) {
    const float* Ls = Ls0 + (step & 1) * (kR3S * kT2K);
    float* Cb = Cb0 + (step & 1) * (kR3S * kT2CS);
    if (DIAG != 2) {  // (past the last step: clamped rows, never used)
      loadC(step + 1, cn);
      loadL(step + 2, lnext);
    }
    floatx16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.f;
    if constexpr (DIAG != 1) {
#pragma unroll
      for (int sg = 0; sg < kOB / 8; ++sg) {
        const float4 fa = *reinterpret_cast<const float4*>(Ls + (wr + il) * kT2K + (kOB / 2) * h + 4 * sg);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(fa, s4), get4(ub[sg], s4), acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int v = 0; v < 16; ++v) Cb[(wr + 8 * (v >> 2) + 4 * h + (v & 3)) * kT2CS + wc + il] = acc[v];
    writeL(Ls0 + ((step + 1) & 1) * (kR3S * kT2K), lw);
    __syncthreads();  // Cb[t & 1] = product (t), Ls[(t + 1) & 1] = L21 (t + 1); Ls[t & 1] consumed
    if (DIAG != 2) storeOut(step, Cb, cc);
  };

  if constexpr (VEC) {
    VT c0r[kCQ], c1r[kCQ], la[kLQ], lb[kLQ];
    loadC(0, c0r);
    loadL(0, la);
    loadL(1, lb);
    writeL(Ls0, la);
    __syncthreads();
    // pairs of steps, the odd last one after the loop: no conditional body inside the loop, whose
    // merge would make the compiler copy the register sets (waiting on their loads to do so)
    int step = 0;
    for (; step + 1 < nsteps; step += 2) {
      body(step, c0r, c1r, lb, la);
      body(step + 1, c1r, c0r, la, lb);
    }
    if (step < nsteps) body(step, c0r, c1r, lb, la);
  } else {
    // scalar path (N % 4 != 0: 16 single-float accesses per thread and array): one register set
    // each, the next step's loads issued after the output (the double sets spill here)
    VT c[kCQ], l[kLQ];
    loadC(0, c);
    loadL(0, l);
    writeL(Ls0, l);
    loadL(1, l);
    __syncthreads();
    for (int step = 0; step < nsteps; ++step) {
      const float* Ls = Ls0 + (step & 1) * (kR3S * kT2K);
      float* Cb = Cb0 + (step & 1) * (kR3S * kT2CS);
      floatx16 acc;
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[v] = 0.f;
      if constexpr (DIAG != 1) {
#pragma unroll
        for (int sg = 0; sg < kOB / 8; ++sg) {
          const float4 fa = *reinterpret_cast<const float4*>(Ls + (wr + il) * kT2K + (kOB / 2) * h + 4 * sg);
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(fa, s4), get4(ub[sg], s4), acc, 0, 0, 0);
        }
      }
#pragma unroll
      for (int v = 0; v < 16; ++v) Cb[(wr + 8 * (v >> 2) + 4 * h + (v & 3)) * kT2CS + wc + il] = acc[v];
      writeL(Ls0 + ((step + 1) & 1) * (kR3S * kT2K), l);
      __syncthreads();
      if (DIAG != 2) {
        storeOut(step, Cb, c);
        loadC(step + 1, c);
        loadL(step + 2, l);
      }
    }
  }
  __syncthreads();  // every gathered load of a block row has completed: U12 to the block rows
  if (cb + wc + il < N) {
#pragma unroll
    for (int sg = 0; sg < kOB / 8; ++sg) {  // (static register index: the two waves with the same
      if ((sg >= kOB / 16) != (wave >= 4)) continue;  //  columns split the rows)
      const int i = (kOB / 2) * h + 4 * sg;
      float* dst = Ab + (size_t)(P + i) * N + cb + wc + il;
      dst[0] = ub[sg].x;
      dst[(size_t)N] = ub[sg].y;
      dst[2 * (size_t)N] = ub[sg].z;
      dst[3 * (size_t)N] = ub[sg].w;
    }
  }
}


// ---- r04 variant "direct": the product never goes through LDS ----
// Two 4-wave workgroups per CU as lu_trail128_kernel, but 64-row steps and each wave owns columns
// [32w, 32w + 32) of BOTH 32-row tiles of a step (two accumulators, 128 MFMAs per step and barrier);
// A22 is loaded and stored in the accumulator layout (lane (il, h), element v: row 8(v/4) + 4h +
// v%4 of the tile, column il: every dword instruction moves two whole 128-B row segments), so
// out = A22 - product is formed in the registers of the wave that computed the product: no Cb
// tile, no product round trip, no barrier between the MFMAs and the output.  L21 double-buffered
// in LDS (the only barrier per step).  Source rows of each step's 64 rows (the gathered
// interchanges) are tabulated once per step by 64 threads.  Same chains (k order), same products,
// same subtraction: bitwise the factors of lu_trail128_kernel.  VEC only, N <= 32767 (32-bit
// buffer offsets over one instance).
constexpr int kDRS = 64;
constexpr int kDBitWords = (kLuMaxN + 31) / 32 + 2;
constexpr int kDMainFloats = 2 * kDRS * kT2K;
constexpr int kDProFloats = 2 * kOB * kT2PK;
constexpr int kDAreaFloats = kDMainFloats > kDProFloats ? kDMainFloats : kDProFloats;
constexpr size_t kDLds = (size_t)kDAreaFloats * 4 + (4 * kPermMax + 2 * kDRS + kDBitWords) * 4 + ((kDBitWords + 3) & ~3);
static_assert(2 * kDLds <= 160 * 1024, "two workgroups per CU");

template <int DIAG = 0>
__global__ __launch_bounds__(256, 2) void lu_trail128d_kernel(int N, int P, int ntc, float* A, const float* Linv,
                                                             const int* perm) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ls0 = sm;
  float* Lh = sm;
  float* Uh = sm + kOB * kT2PK;
  float* Ut = sm;
  int* bsrc = reinterpret_cast<int*>(sm + kDAreaFloats);
  int* tdst = bsrc + kPermMax;
  int* tsrc = tdst + kPermMax;
  int* dsrc = tsrc + kPermMax;
  int* srow0 = dsrc + kPermMax;                                     // 2 x [64]: source rows of a step
  unsigned* dbits = reinterpret_cast<unsigned*>(srow0 + 2 * kDRS);    // 1 word per 32 rows
  unsigned char* dpre = reinterpret_cast<unsigned char*>(dbits + kDBitWords);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, local = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int logical = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  const size_t b = (size_t)(logical / ntc);
  const int tc = logical % ntc;
  float* Ab = A + b * (size_t)N * N;
  const int c0 = P + kOB, cb = c0 + tc * kT2C;
  const int nsteps = (N - c0 + kDRS - 1) / kDRS;
  const int nwords = (N - c0 + 31) / 32;
  const int tid = threadIdx.x, lane = tid & 63, il = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int NT = 256;

  const int ndisp = perm ? perm[b * kPermInts + 4 * kPermMax] - kOB : 0;
  {
    const int* pb = perm + b * kPermInts;
    if (tid < kOB) bsrc[tid] = perm ? pb[2 * kPermMax + tid] : P + tid;
    if (tid < ndisp) { tdst[tid] = pb[kOB + tid]; tsrc[tid] = pb[2 * kPermMax + kOB + tid]; }
    for (int w = tid; w < nwords + 4; w += NT) { dbits[w] = 0u; dpre[w] = 0; }
  }
  __syncthreads();
  int drank = 0, dd = 0;
  if (tid < ndisp) {
    dd = tdst[tid] - c0;
    for (int j = 0; j < ndisp; ++j) drank += tdst[j] - c0 < dd;
    dsrc[drank] = tsrc[tid];
    atomicOr(&dbits[dd >> 5], 1u << (dd & 31));
  }
  __syncthreads();
  if (tid < ndisp && __builtin_popcount(dbits[dd >> 5] & ((1u << (dd & 31)) - 1u)) == 0)
    dpre[dd >> 5] = (unsigned char)drank;
  // source row (clamped) of trailing row c0 + ro
  auto src_of = [&](int ro) -> int {
    const int w = ro >> 5, bit = ro & 31;
    const unsigned m = dbits[w];
    const int s = dsrc[(dpre[w] + __builtin_popcount(m & ((1u << bit) - 1u))) & (kPermMax - 1)];
    return min(((m >> bit) & 1u) ? s : c0 + ro, N - 1);
  };

  // ---- prologue (as lu_trail128_kernel)
  const float* Lb = Linv + b * (size_t)kLinvFloats;
  floatx16 u[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int v = 0; v < 16; ++v) u[j][v] = 0.f;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (pass) __syncthreads();
    float4 av[8], lv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + NT * q, kk = e / 32, col = cb + (e % 32) * 4;
      const int k = kk < 32 ? 32 * pass + kk : 64 + 32 * pass + kk - 32;
      const float4 x = *reinterpret_cast<const float4*>(Ab + (size_t)bsrc[k] * N + min(col, N - 4));
      av[q] = col < N ? x : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + NT * q, i = e / 16, kk = (e % 16) * 4;
      const int k = kk < 32 ? 32 * pass + kk : 64 + 32 * pass + kk - 32;
      lv[q] = *reinterpret_cast<const float4*>(Lb + (size_t)i * kOB + k);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + NT * q, kk = e / 32, cl = (e % 32) * 4;
      Uh[(cl + 0) * kT2PK + kk] = av[q].x; Uh[(cl + 1) * kT2PK + kk] = av[q].y;
      Uh[(cl + 2) * kT2PK + kk] = av[q].z; Uh[(cl + 3) * kT2PK + kk] = av[q].w;
      *reinterpret_cast<float4*>(Lh + (e / 16) * kT2PK + (e % 16) * 4) = lv[q];
    }
    __syncthreads();
#pragma unroll 2
    for (int sg = 0; sg < 8; ++sg) {
      const float4 fa = *reinterpret_cast<const float4*>(Lh + (wave * 32 + il) * kT2PK + 32 * h + 4 * sg);
      float4 fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const float4*>(Uh + (j * 32 + il) * kT2PK + 32 * h + 4 * sg);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int j = 0; j < 4; ++j) u[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(fa, s4), get4(fb[j], s4), u[j], 0, 0, 0);
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int v = 0; v < 16; ++v) Ut[(j * 32 + il) * kT2K + wave * 32 + 8 * (v >> 2) + 4 * h + (v & 3)] = u[j][v];
  __syncthreads();
  const int wc = wave * 32;
  float4 ub[kOB / 8];
#pragma unroll
  for (int sg = 0; sg < kOB / 8; ++sg)
    ub[sg] = *reinterpret_cast<const float4*>(Ut + (wc + il) * kT2K + (kOB / 2) * h + 4 * sg);
  __syncthreads();  // Ut consumed

  // ---- main loop
  const int col = cb + wc + il;
  const bool cok = col < N;
  const unsigned colb = (unsigned)min(col, N - 1) * 4u;
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(Ab, 0, (int)((unsigned)N * (unsigned)N * 4u), 0x00020000);
  // A22 tile t (rows c0 + 64t + 32rt + 8(v/4) + 4h + v%4): per (rt, v) one dword load of this lane
  auto loadC = [&](int step, const int* srow, float (&c)[32]) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int4 r4 = *reinterpret_cast<const int4*>(srow + rt * 32 + 8 * g + 4 * h);
        const int rr[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          c[rt * 16 + 4 * g + e] = __uint_as_float(
              __builtin_amdgcn_raw_buffer_load_b32(rin, (unsigned)rr[e] * (unsigned)N * 4u + colb, 0, 0));
      }
  };
  // (L21 staging: eight named registers -- an array passed to a lambda stayed a scratch alloca here)
  float4 l0, l1, l2, l3, l4, l5, l6, l7;
#define IADMM_LDL(step)                                                                               \
  do {                                                                                                \
    const int rb_ = c0 + (step) * kDRS + tid / 32, cl_ = P + (tid % 32) * 4;                          \
    l0 = *reinterpret_cast<const float4*>(Ab + (size_t)min(rb_ + 0, N - 1) * N + cl_);                \
    l1 = *reinterpret_cast<const float4*>(Ab + (size_t)min(rb_ + 8, N - 1) * N + cl_);                \
    l2 = *reinterpret_cast<const float4*>(Ab + (size_t)min(rb_ + 16, N - 1) * N + cl_);               \
    l3 = *reinterpret_cast<const float4*>(Ab + (size_t)min(rb_ + 24, N - 1) * N + cl_);               \
    l4 = *reinterpret_cast<const float4*>(Ab + (size_t)min(rb_ + 32, N - 1) * N + cl_);               \
    l5 = *reinterpret_cast<const float4*>(Ab + (size_t)min(rb_ + 40, N - 1) * N + cl_);               \
    l6 = *reinterpret_cast<const float4*>(Ab + (size_t)min(rb_ + 48, N - 1) * N + cl_);               \
    l7 = *reinterpret_cast<const float4*>(Ab + (size_t)min(rb_ + 56, N - 1) * N + cl_);               \
  } while (0)
#define IADMM_WRL(Ls)                                                                                 \
  do {                                                                                                \
    float* d_ = (Ls) + (tid / 32) * kT2K + (tid % 32) * 4;                                            \
    *reinterpret_cast<float4*>(d_) = l0; *reinterpret_cast<float4*>(d_ + 8 * kT2K) = l1;              \
    *reinterpret_cast<float4*>(d_ + 16 * kT2K) = l2; *reinterpret_cast<float4*>(d_ + 24 * kT2K) = l3; \
    *reinterpret_cast<float4*>(d_ + 32 * kT2K) = l4; *reinterpret_cast<float4*>(d_ + 40 * kT2K) = l5; \
    *reinterpret_cast<float4*>(d_ + 48 * kT2K) = l6; *reinterpret_cast<float4*>(d_ + 56 * kT2K) = l7; \
  } while (0)
  auto fill_srow = [&](int step, int* dst) {
    if (tid < kDRS) dst[tid] = src_of(min(step * kDRS + tid, N - c0 - 1));
  };
  auto storeOut = [&](int step, float (&c)[32], const floatx16 (&acc)[2]) {
    const int r0 = c0 + step * kDRS;
    const int nval = min(kDRS, N - r0);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(Ab + (size_t)r0 * N, 0, nval * N * 4, 0x00020000);
    const unsigned vb = cok ? ((unsigned)(4 * h) * (unsigned)N * 4u + (unsigned)col * 4u) : 0x80000000u;
    if (nval == kDRS) {  // (full steps: the SGPR row offset; gfx950 does count soffset in the range check --
                         //  profiles/r04_buffer_soffset_probe.txt -- but this bench keeps the r03 guard)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const float o = c[rt * 16 + v] - acc[rt][v];
          const int so = (rt * 32 + 8 * (v >> 2) + (v & 3)) * N * 4;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), ro, vb, so, 0);
        }
    } else {  // the last, partial step: the whole offset in the VGPR, so rows past N are dropped
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const float o = c[rt * 16 + v] - acc[rt][v];
          const unsigned so = (unsigned)((rt * 32 + 8 * (v >> 2) + (v & 3)) * N * 4);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), ro, cok ? vb + so : 0x80000000u, 0, 0);
        }
    }
  };
  auto chain = [&](const float* Ls, floatx16 (&acc)[2]) {
    const floatx16 zero = {};
    const float* l0 = Ls + il * kT2K + (kOB / 2) * h;
    const float* l1 = l0 + 32 * kT2K;
    float4 fa[kOB / 8][2];
    __builtin_amdgcn_sched_barrier(0);
    fa[0][0] = *reinterpret_cast<const float4*>(l0);
    fa[0][1] = *reinterpret_cast<const float4*>(l1);
#pragma unroll
    for (int sg = 0; sg < kOB / 8; ++sg) {
      if (sg + 1 < kOB / 8) {
        fa[sg + 1][0] = *reinterpret_cast<const float4*>(l0 + 4 * (sg + 1));
        fa[sg + 1][1] = *reinterpret_cast<const float4*>(l1 + 4 * (sg + 1));
      }
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
          acc[rt] = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(fa[sg][rt], s4), get4(ub[sg], s4),
                                                         (sg == 0 && s4 == 0) ? zero : acc[rt], 0, 0, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
    for (int sg = 0; sg < kOB / 8 - 1; ++sg) {
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  // step t: chain t (L21 from Ls[t & 1]); out = A22 (t) - product; the loads of A22 (t + 1) into
  // the same registers (a store reads its data registers at issue); L21 (t + 1), loaded during step
  // t - 1, -> Ls[(t + 1) & 1]; the loads of L21 (t + 2); the source rows of step t + 2; barrier.
  // One register set per array: everything loaded in step t is consumed in step t + 1.
  float cc[32];
  fill_srow(0, srow0);
  fill_srow(1, srow0 + kDRS);
  __syncthreads();
  loadC(0, srow0, cc);
  IADMM_LDL(0);
  IADMM_WRL(Ls0);
  IADMM_LDL(1);
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    floatx16 acc[2] = {};
    if constexpr (DIAG != 1) chain(Ls0 + (step & 1) * (kDRS * kT2K), acc);
    if (DIAG != 2) {
      storeOut(step, cc, acc);
      loadC(step + 1, srow0 + ((step + 1) & 1) * kDRS, cc);
    }
    IADMM_WRL(Ls0 + ((step + 1) & 1) * (kDRS * kT2K));
    if (DIAG != 2) IADMM_LDL(step + 2);
    fill_srow(step + 2, srow0 + (step & 1) * kDRS);
    __syncthreads();
  }
  __syncthreads();
  if (cok) {
#pragma unroll
    for (int sg = 0; sg < kOB / 8; ++sg) {
      const int i = (kOB / 2) * h + 4 * sg;
      float* dst = Ab + (size_t)(P + i) * N + col;
      dst[0] = ub[sg].x;
      dst[(size_t)N] = ub[sg].y;
      dst[2 * (size_t)N] = ub[sg].z;
      dst[3 * (size_t)N] = ub[sg].w;
    }
  }
#undef IADMM_LDL
#undef IADMM_WRL
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
  if (WS == 2) hipLaunchKernelGGL((lu_trail128d_kernel<DIAG>), dim3(B * ntc), dim3(256), kDLds, 0, N, P, ntc, A, Linv, nullptr);
  else if (WS) hipLaunchKernelGGL((lu_trail128_kernel<true, DIAG>), dim3(B * ntc), dim3(kT2Threads), kT2Lds, 0, N, P, ntc, 0, A, Linv, nullptr);
  else hipLaunchKernelGGL((lu_trail128_r03_kernel<true, DIAG>), dim3(B * ntc), dim3(kR3Threads), kR3Lds, 0, N, P, ntc, A, Linv, nullptr);
}

template <int WS, int DIAG>
float run(int B, int N, int P, float* A, float* Linv, int reps) {
  if (WS == 2) CK(hipFuncSetAttribute((const void*)lu_trail128d_kernel<DIAG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDLds));
  else if (WS) CK(hipFuncSetAttribute((const void*)lu_trail128_kernel<true, DIAG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kT2Lds));
  else CK(hipFuncSetAttribute((const void*)lu_trail128_r03_kernel<true, DIAG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kR3Lds));
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
  // bitwise: one launch of each kernel on the same input (r03 vs paired, paired vs direct)
  CK(hipFuncSetAttribute((const void*)lu_trail128_kernel<true, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kT2Lds));
  CK(hipFuncSetAttribute((const void*)lu_trail128_r03_kernel<true, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kR3Lds));
  CK(hipFuncSetAttribute((const void*)lu_trail128d_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDLds));
  for (int P : {0, 896, N - kOB - 64, N - kOB - 40}) {
    for (int pair = 0; pair < 2; ++pair) {
      hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, A, (int64_t)n);
      CK(hipMemcpy(A2, A, n * sizeof(float), hipMemcpyDeviceToDevice));
      if (pair == 0) { launch<0, 0>(B, N, P, A, Linv); launch<1, 0>(B, N, P, A2, Linv); }
      else { launch<1, 0>(B, N, P, A, Linv); launch<2, 0>(B, N, P, A2, Linv); }
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
      printf("P=%4d bitwise %s: %zu differing words (instances 0-3 and %d)\n", P, pair ? "paired vs direct" : "r03 vs paired",
             diff, B - 1);
    }
  }
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, A, (int64_t)n);
  CK(hipDeviceSynchronize());
  for (int P : {0, 896}) {
    const double rest = N - P - kOB;
    const double bytes = (double)B * 4.0 * (2 * rest * rest + rest * kOB + 2 * kOB * rest);
    const double flops = (double)B * 2.0 * (rest * rest * kOB + kOB * kOB * rest);
    const char* names[3] = {"full", "no-mfma", "no-global"};
    const char* kn[3] = {"r03", "pair", "dir"};
    for (int round = 0; round < 2; ++round) {
      float t[9] = {run<0, 0>(B, N, P, A, Linv, 5), run<0, 1>(B, N, P, A, Linv, 5), run<0, 2>(B, N, P, A, Linv, 5),
                    run<1, 0>(B, N, P, A, Linv, 5), run<1, 1>(B, N, P, A, Linv, 5), run<1, 2>(B, N, P, A, Linv, 5),
                    run<2, 0>(B, N, P, A, Linv, 5), run<2, 1>(B, N, P, A, Linv, 5), run<2, 2>(B, N, P, A, Linv, 5)};
      for (int v = 0; v < 9; ++v)
        printf("P=%4d %-4s %-10s %8.3f ms  %7.0f GB/s alg  %6.1f TF\n", P, kn[v / 3], names[v % 3], t[v],
               bytes / t[v] / 1e6, flops / t[v] / 1e9);
    }
  }
  CK(hipFree(A)); CK(hipFree(A2)); CK(hipFree(Linv));
  return 0;
}
