// The K-loop of the fused LSTM-cell GEMM, shared by the forward kernel (lstm.hip) and the
// recompute in the training backward (train.hip).  See lstm.hip for the tiling.
#pragma once
#include "common.h"

namespace iadmm {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kJT = 32;          // hidden units per workgroup
constexpr int kRows = 256;       // data rows per workgroup
constexpr int kBK = 32;          // K chunk
constexpr int kLD = kBK + 4;     // padded LDS row (floats)
constexpr int kWxF = 16;         // packed per-unit fields: Wi0 Wi1 bi Wf0 Wf1 bf Wo0 Wo1 bo Wu0 Wu1 bu Wh

struct CellArgsT {
  int64_t M;
  int h, njt, nkc32;
  const float *H, *C, *xv, *g, *Upk, *Wx;
  float *Hn, *Cn, *part;
};

// XCD-aware bijective remap: blocks b, b+8, ... share an XCD; give each XCD a contiguous run of
// logical tiles with the hidden tile fastest, so an H panel is reused from that XCD's L2.
IADMM_DEV void cell_tile_of_block(int njt, int& jt, int& rt) {
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, local = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int logical = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + local;
  jt = logical % njt;
  rt = logical / njt;
}

// acc[g][r] (4 gates x 2 row blocks of 32x32) = U_g[:, jt*32 .. +32]^T . H[rbase + wave*64 + r*32 ..]^T
// NW waves per workgroup (64*NW data rows).  PRIO: 0 none; 1 s_setprio(1) around each MFMA
// cluster; 2 (NW = 8) static priority 1 for waves 4-7 (cdna_hip_programming.md T5).
template <bool VEC, int NW = 4, int PRIO = 0>
IADMM_DEV void cell_mainloop(const float* __restrict__ H, int64_t M, int h, int nkc,
                             const float* __restrict__ Ubase, int64_t rbase, float* sA, float* sB,
                             floatx16 (&acc)[4][2], int tid, int wave, int jl, int hf) {
  constexpr int NT = 64 * NW;
  constexpr int A4 = 128 * kBK / 4 / NT;  // weight float4 per thread: 4 (NW 4) or 2 (NW 8)
  static_assert(A4 == 4 || A4 == 2, "NW must be 4 or 8");
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[g][r][q] = 0.f;
  if constexpr (PRIO == 2) {
    if (__builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);
  }

  // Staging registers as named scalars (an array here was turned into an LDS/scratch alloca
  // by the compiler, which then waited for each global load right after issuing it).
  float4 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3, rb4, rb5, rb6, rb7;
  auto ldB = [&](int kc, int i) -> float4 {
    const int idx = tid + NT * i, row = idx >> 3, c4 = idx & 7;
    const int64_t R = rbase + row;
    const int k = kc * kBK + c4 * 4;
    if constexpr (VEC) {
      return (R < M && k < h) ? *reinterpret_cast<const float4*>(H + R * h + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      float4 t;
#pragma unroll
      for (int e = 0; e < 4; ++e) set4(t, e, (R < M && k + e < h) ? H[R * h + k + e] : 0.f);
      return t;
    }
  };
  auto gload = [&](int kc) {
    const float4* Ac = reinterpret_cast<const float4*>(Ubase + (int64_t)kc * 128 * kBK);
    ra0 = Ac[tid];
    ra1 = Ac[tid + NT];
    if constexpr (A4 == 4) {
      ra2 = Ac[tid + 2 * NT];
      ra3 = Ac[tid + 3 * NT];
    }
    rb0 = ldB(kc, 0); rb1 = ldB(kc, 1); rb2 = ldB(kc, 2); rb3 = ldB(kc, 3);
    rb4 = ldB(kc, 4); rb5 = ldB(kc, 5); rb6 = ldB(kc, 6); rb7 = ldB(kc, 7);
  };
  auto st = [&](float* sm, int i, const float4& v) {
    const int idx = tid + NT * i, row = idx >> 3, c4 = idx & 7;
    *reinterpret_cast<float4*>(&sm[row * kLD + c4 * 4]) = v;
  };

  gload(0);
  for (int kc = 0; kc < nkc; ++kc) {
    __syncthreads();
    st(sA, 0, ra0); st(sA, 1, ra1);
    if constexpr (A4 == 4) { st(sA, 2, ra2); st(sA, 3, ra3); }
    st(sB, 0, rb0); st(sB, 1, rb1); st(sB, 2, rb2); st(sB, 3, rb3);
    st(sB, 4, rb4); st(sB, 5, rb5); st(sB, 6, rb6); st(sB, 7, rb7);
    __syncthreads();
    if (kc + 1 < nkc) gload(kc + 1);
    if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int G = 0; G < kBK / 8; ++G) {
      float4 af[4], bf[2];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        af[g] = *reinterpret_cast<const float4*>(&sA[(g * 32 + jl) * kLD + 8 * G + 4 * hf]);
#pragma unroll
      for (int r = 0; r < 2; ++r)
        bf[r] = *reinterpret_cast<const float4*>(&sB[(wave * 64 + r * 32 + jl) * kLD + 8 * G + 4 * hf]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int r = 0; r < 2; ++r)
            acc[g][r] = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(af[g], s), get4(bf[r], s),
                                                             acc[g][r], 0, 0, 0);
    }
    if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
  }
  if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);
}

// The forward cell kernel (production instance: NW = 4, PRIO = 0, lstm.hip): fp32-MFMA gate GEMM
// (cell_mainloop) + the fused cell epilogue.  Workgroup = 32 hidden units x 64*NW rows.
template <bool VEC, int NW = 4, int PRIO = 0>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void cell_fwd_kernel(CellArgsT a) {
  constexpr int ROWS = 64 * NW;
  __shared__ __attribute__((aligned(16))) float sA[128 * kLD];
  __shared__ __attribute__((aligned(16))) float sB[ROWS * kLD];
  __shared__ __attribute__((aligned(16))) float sW[kWxF * kJT];

  int jt, rt;
  cell_tile_of_block(a.njt, jt, rt);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int jl = lane & 31, hf = lane >> 5;
  const int h = a.h;
  const int64_t M = a.M;
  const int64_t rbase = (int64_t)rt * ROWS;

  for (int i = tid; i < kWxF * kJT; i += 64 * NW) {
    const int f = i / kJT, jj = i % kJT;
    sW[i] = a.Wx[(int64_t)(jt * kJT + jj) * kWxF + f];
  }

  floatx16 acc[4][2];
  cell_mainloop<VEC, NW, PRIO>(a.H, M, h, a.nkc32, a.Upk + (int64_t)jt * a.nkc32 * 128 * kBK, rbase, sA, sB,
                               acc, tid, wave, jl, hf);

  // ---- epilogue: gates, cell update, projection partial (all in registers)
  // accumulator element q of lane (jl,hf): hidden jj = (q&3) + 8*(q>>2) + 4*hf, data row jl.
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int64_t R = rbase + wave * 64 + r * 32 + jl;
    const bool rok = R < M;
    const float in0 = rok ? a.xv[R] : 0.f;
    const float in1 = rok ? a.g[R] : 0.f;
    float gsum = 0.f;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int jj0 = 8 * qq + 4 * hf;
      const int j0 = jt * kJT + jj0;
      float4 cold;
      if constexpr (VEC) {
        cold = (rok && j0 < h) ? *reinterpret_cast<const float4*>(a.C + R * h + j0)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) set4(cold, e, (rok && j0 + e < h) ? a.C[R * h + j0 + e] : 0.f);
      }
      float4 wv[13];
#pragma unroll
      for (int f = 0; f < 13; ++f) wv[f] = *reinterpret_cast<const float4*>(&sW[f * kJT + jj0]);
      float4 cnew, hnew;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int q = qq * 4 + e;
        float pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float xw = in0 * get4(wv[3 * g], e) + in1 * get4(wv[3 * g + 1], e);
          pre[g] = (xw + acc[g][r][q]) + get4(wv[3 * g + 2], e);
        }
        const float ig = sigmoidf_(pre[0]), fg = sigmoidf_(pre[1]), og = sigmoidf_(pre[2]);
        const float ug = tanhf(pre[3]);
        const float c2 = ig * ug + fg * get4(cold, e);
        const float h2 = og * tanhf(c2);
        set4(cnew, e, c2);
        set4(hnew, e, h2);
        gsum = fmaf(h2, get4(wv[12], e), gsum);
      }
      if (rok) {
        if constexpr (VEC) {
          if (j0 < h) {
            *reinterpret_cast<float4*>(a.Cn + R * h + j0) = cnew;
            *reinterpret_cast<float4*>(a.Hn + R * h + j0) = hnew;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (j0 + e < h) {
              a.Cn[R * h + j0 + e] = get4(cnew, e);
              a.Hn[R * h + j0 + e] = get4(hnew, e);
            }
          }
        }
      }
    }
    gsum += __shfl_xor(gsum, 32, 64);
    if (hf == 0 && rok) a.part[(int64_t)jt * M + R] = gsum;
  }
}

}  // namespace iadmm
