// Parameterised fused LSTM-cell kernel (forward), shared by the production entry point
// (lstm.hip) and the variant microbenchmark (tools/cellbench.hip).
//
//   NW    waves per workgroup; the workgroup covers 32 hidden units x 64*NW data rows
//   BK    K-chunk staged through LDS (16 or 32)
//   DBUF  two LDS buffers and one barrier per chunk (else one buffer, two barriers)
//   FAST  epilogue transcendentals from v_exp_f32/v_rcp_f32 (else libm expf/tanhf)
//   EPI   0: full cell epilogue; 1: bench-only minimal epilogue (keeps the accumulators alive)
// Upk is packed in 32-deep K chunks ([jt][kc32][128][32]); BK = 16 reads half-chunks.
#pragma once
#include "cell_tile.h"

namespace iadmm {

IADMM_DEV float fast_sigmoid(float x) { return __frcp_rn(1.0f + __expf(-x)); }
IADMM_DEV float fast_tanh(float x) {
  // tanh(x) = 1 - 2 / (exp(2x) + 1); saturates correctly at +-inf
  return 1.0f - 2.0f * __frcp_rn(__expf(2.0f * x) + 1.0f);
}

template <int NW, int BK, bool DBUF, bool FAST, int EPI, bool VEC>
__global__ __launch_bounds__(64 * NW, (NW == 4 ? 2 : 1)) void cell_fwd_kernel(CellArgsT a) {
  constexpr int NT = 64 * NW;
  constexpr int ROWS = 64 * NW;
  constexpr int LD = BK + 4;
  constexpr int NBUF = DBUF ? 2 : 1;
  constexpr int A4 = 128 * BK / 4 / NT;    // float4 per thread for the weight chunk
  constexpr int B4 = ROWS * BK / 4 / NT;   // float4 per thread for the H chunk
  constexpr int C4 = BK / 4;               // float4 per row
  __shared__ __attribute__((aligned(16))) float sA[NBUF][128 * LD];
  __shared__ __attribute__((aligned(16))) float sB[NBUF][ROWS * LD];
  __shared__ __attribute__((aligned(16))) float sW[kWxF * kJT];

  int jt, rt;
  cell_tile_of_block(a.njt, jt, rt);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, jl = lane & 31, hf = lane >> 5;
  const int h = a.h;
  const int64_t M = a.M;
  const int64_t rbase = (int64_t)rt * ROWS;
  const int nkc = (h + BK - 1) / BK;
  const float* Ubase = a.Upk + (int64_t)jt * a.nkc32 * 128 * kBK;

  for (int i = tid; i < kWxF * kJT; i += NT) {
    const int f = i / kJT, jj = i % kJT;
    sW[i] = a.Wx[(int64_t)(jt * kJT + jj) * kWxF + f];
  }

  floatx16 acc[4][2];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[g][r][q] = 0.f;

  float4 ra[A4], rb[B4];
  auto gload = [&](int kc) {
    const int k0 = kc * BK;
    const float* Ac = Ubase + (int64_t)(k0 / kBK) * 128 * kBK + (k0 % kBK);
#pragma unroll
    for (int i = 0; i < A4; ++i) {
      const int idx = tid + NT * i, row = idx / C4, c4 = idx % C4;
      ra[i] = *reinterpret_cast<const float4*>(Ac + row * kBK + c4 * 4);
    }
#pragma unroll
    for (int i = 0; i < B4; ++i) {
      const int idx = tid + NT * i, row = idx / C4, c4 = idx % C4;
      const int64_t R = rbase + row;
      const int k = k0 + c4 * 4;
      if constexpr (VEC) {
        rb[i] = (R < M && k < h) ? *reinterpret_cast<const float4*>(a.H + R * h + k)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        float4 t;
#pragma unroll
        for (int e = 0; e < 4; ++e) set4(t, e, (R < M && k + e < h) ? a.H[R * h + k + e] : 0.f);
        rb[i] = t;
      }
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A4; ++i) {
      const int idx = tid + NT * i, row = idx / C4, c4 = idx % C4;
      *reinterpret_cast<float4*>(&sA[buf][row * LD + c4 * 4]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B4; ++i) {
      const int idx = tid + NT * i, row = idx / C4, c4 = idx % C4;
      *reinterpret_cast<float4*>(&sB[buf][row * LD + c4 * 4]) = rb[i];
    }
  };
  auto compute = [&](int buf) {
#pragma unroll
    for (int G = 0; G < BK / 8; ++G) {
      float4 af[4], bf[2];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        af[g] = *reinterpret_cast<const float4*>(&sA[buf][(g * 32 + jl) * LD + 8 * G + 4 * hf]);
#pragma unroll
      for (int r = 0; r < 2; ++r)
        bf[r] = *reinterpret_cast<const float4*>(&sB[buf][(wave * 64 + r * 32 + jl) * LD + 8 * G + 4 * hf]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int r = 0; r < 2; ++r)
            acc[g][r] = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(af[g], s), get4(bf[r], s), acc[g][r], 0, 0, 0);
    }
  };

  if constexpr (DBUF) {
    gload(0);
    lstore(0);
    if (nkc > 1) gload(1);
    __syncthreads();
    for (int kc = 0; kc < nkc; ++kc) {
      const int buf = kc & 1;
      compute(buf);
      if (kc + 1 < nkc) lstore(buf ^ 1);
      if (kc + 2 < nkc) gload(kc + 2);
      __syncthreads();
    }
  } else {
    gload(0);
    for (int kc = 0; kc < nkc; ++kc) {
      __syncthreads();
      lstore(0);
      __syncthreads();
      if (kc + 1 < nkc) gload(kc + 1);
      compute(0);
    }
  }

  if constexpr (EPI == 1) {  // bench only: consume the accumulators cheaply
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int q = 0; q < 16; ++q) s += acc[g][r][q];
    const int64_t R = rbase + wave * 64 + jl;
    if (R < M && hf == 0) a.part[(int64_t)jt * M + R] = s;
    return;
  }

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
        float ig, fg, og, ug, tc;
        if constexpr (FAST) {
          ig = fast_sigmoid(pre[0]); fg = fast_sigmoid(pre[1]); og = fast_sigmoid(pre[2]);
          ug = fast_tanh(pre[3]);
        } else {
          ig = sigmoidf_(pre[0]); fg = sigmoidf_(pre[1]); og = sigmoidf_(pre[2]);
          ug = tanhf(pre[3]);
        }
        const float c2 = ig * ug + fg * get4(cold, e);
        if constexpr (FAST) tc = fast_tanh(c2); else tc = tanhf(c2);
        const float h2 = og * tc;
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

namespace iadmm {

typedef float floatx4_t __attribute__((ext_vector_type(4)));

// Same cell kernel on v_mfma_f32_16x16x4_f32 (A: lane l holds A[l&15][k=l>>4]; B: B[k=l>>4][l&15];
// C/D: row (hidden) = 4*(l>>4) + reg, col (data row) = l&15).  Wave tile: 4 gates x 32 hidden
// (2 blocks of 16) x 64 rows (4 blocks of 16) = 32 accumulators of 4 registers.  K-permuted so
// each fragment fetch is one ds_read_b128: lane group kq = l>>4 supplies k = 16G + 4kq + s.
template <bool FAST, int EPI>
__global__ __launch_bounds__(256, 2) void cell_fwd16_kernel(CellArgsT a) {
  constexpr int NT = 256, ROWS = 256, BK = 32, LD = BK + 4;
  __shared__ __attribute__((aligned(16))) float sA[128 * LD];
  __shared__ __attribute__((aligned(16))) float sB[ROWS * LD];
  __shared__ __attribute__((aligned(16))) float sW[kWxF * kJT];
  int jt, rt;
  cell_tile_of_block(a.njt, jt, rt);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, il = lane & 15, kq = lane >> 4;
  const int h = a.h;
  const int64_t M = a.M;
  const int64_t rbase = (int64_t)rt * ROWS;
  const int nkc = (h + BK - 1) / BK;
  const float* Ubase = a.Upk + (int64_t)jt * a.nkc32 * 128 * kBK;
  for (int i = tid; i < kWxF * kJT; i += NT) {
    const int f = i / kJT, jj = i % kJT;
    sW[i] = a.Wx[(int64_t)(jt * kJT + jj) * kWxF + f];
  }
  floatx4_t acc[4][2][4];  // [gate][hidden block][row block]
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[g][hb][rb][q] = 0.f;
  float4 ra[4], rb4[8];
  auto gload = [&](int kc) {
    const float4* Ac = reinterpret_cast<const float4*>(Ubase + (int64_t)kc * 128 * kBK);
#pragma unroll
    for (int i = 0; i < 4; ++i) ra[i] = Ac[tid + NT * i];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = tid + NT * i, row = idx >> 3, c4 = idx & 7;
      const int64_t R = rbase + row;
      const int k = kc * BK + c4 * 4;
      rb4[i] = (R < M && k < h) ? *reinterpret_cast<const float4*>(a.H + R * h + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  gload(0);
  for (int kc = 0; kc < nkc; ++kc) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + NT * i, row = idx >> 3, c4 = idx & 7;
      *reinterpret_cast<float4*>(&sA[row * LD + c4 * 4]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = tid + NT * i, row = idx >> 3, c4 = idx & 7;
      *reinterpret_cast<float4*>(&sB[row * LD + c4 * 4]) = rb4[i];
    }
    __syncthreads();
    if (kc + 1 < nkc) gload(kc + 1);
#pragma unroll
    for (int G = 0; G < BK / 16; ++G) {
      float4 bf[4];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
        bf[rb] = *reinterpret_cast<const float4*>(&sB[(wave * 64 + rb * 16 + il) * LD + 16 * G + 4 * kq]);
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        float4 af[4];
#pragma unroll
        for (int g = 0; g < 4; ++g)
          af[g] = *reinterpret_cast<const float4*>(&sA[(g * 32 + hb * 16 + il) * LD + 16 * G + 4 * kq]);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int rb = 0; rb < 4; ++rb)
              acc[g][hb][rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(get4(af[g], s), get4(bf[rb], s),
                                                                     acc[g][hb][rb], 0, 0, 0);
      }
    }
  }
  if constexpr (EPI == 1) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int hb = 0; hb < 2; ++hb)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
          for (int q = 0; q < 4; ++q) s += acc[g][hb][rb][q];
    const int64_t R = rbase + wave * 64 + lane;
    if (R < M) a.part[(int64_t)jt * M + R] = s;
    return;
  }
  // epilogue: lane owns data rows il + 16 rb (rb = 0..3) and hidden units 16 hb + 4 kq + q
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const int64_t R = rbase + wave * 64 + rb * 16 + il;
    const bool rok = R < M;
    const float in0 = rok ? a.xv[R] : 0.f;
    const float in1 = rok ? a.g[R] : 0.f;
    float gsum = 0.f;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      const int jj0 = 16 * hb + 4 * kq;
      const int j0 = jt * kJT + jj0;
      const float4 cold = (rok && j0 < h) ? *reinterpret_cast<const float4*>(a.C + R * h + j0)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 wv[13];
#pragma unroll
      for (int f = 0; f < 13; ++f) wv[f] = *reinterpret_cast<const float4*>(&sW[f * kJT + jj0]);
      float4 cnew, hnew;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float xw = in0 * get4(wv[3 * g], e) + in1 * get4(wv[3 * g + 1], e);
          pre[g] = (xw + acc[g][hb][rb][e]) + get4(wv[3 * g + 2], e);
        }
        float ig, fg, og, ug, tc;
        if constexpr (FAST) {
          ig = fast_sigmoid(pre[0]); fg = fast_sigmoid(pre[1]); og = fast_sigmoid(pre[2]); ug = fast_tanh(pre[3]);
        } else {
          ig = sigmoidf_(pre[0]); fg = sigmoidf_(pre[1]); og = sigmoidf_(pre[2]); ug = tanhf(pre[3]);
        }
        const float c2 = ig * ug + fg * get4(cold, e);
        if constexpr (FAST) tc = fast_tanh(c2); else tc = tanhf(c2);
        const float h2 = og * tc;
        set4(cnew, e, c2);
        set4(hnew, e, h2);
        gsum = fmaf(h2, get4(wv[12], e), gsum);
      }
      if (rok && j0 < h) {
        *reinterpret_cast<float4*>(a.Cn + R * h + j0) = cnew;
        *reinterpret_cast<float4*>(a.Hn + R * h + j0) = hnew;
      }
    }
    // combine the 4 lane groups (kq) that hold the other hidden units of row R
    gsum += __shfl_xor(gsum, 16, 64);
    gsum += __shfl_xor(gsum, 32, 64);
    if (kq == 0 && rok) a.part[(int64_t)jt * M + R] = gsum;
  }
}

}  // namespace iadmm
