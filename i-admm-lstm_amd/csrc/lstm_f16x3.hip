// Optional split-precision LSTM cell ("f16x3"): the gate GEMM of lstm.hip on the gfx950 fp16
// matrix cores, with fp32-level accuracy from a 3-term split.  NOT the default path (the default
// and the headline bench are the fp32-MFMA kernel); selected with precision="f16x3".
//
// Every fp32 operand x is stored as two fp16 planes, x = hi + lo with hi = fp16(x) and
// lo = fp16(x - hi) (|x - hi| <= 2^-11 |x|, so hi + lo carries 22 significant bits), and
//   U . H  ~=  U_hi H_hi + U_hi H_lo + U_lo H_hi          (fp32 accumulation in the MFMA)
// dropping U_lo H_lo (<= 2^-22 relative per product).  The weights are scaled by an exact power of
// two 2^s (max |U| 2^s in [0.5, 1)) before the split so their lo parts stay out of the fp16
// subnormal range; the accumulator is multiplied by 2^-s (exact) in the epilogue.  H lies in
// (-1, 1); an element below 2^-2 has a subnormal lo part, i.e. absolute error <= 2^-25, below the
// fp32 rounding of the values it is summed with.  Measured against the fp32 kernel and the CPU
// oracle in tests/test_f16x3_gpu.py.
//
// Per 32-deep K chunk a wave issues 48 v_mfma_f32_32x32x16_f16 (2 K halves x 4 gates x 2 row
// blocks x 3 terms, 32 cycles each) where the fp32 kernel issues 128 v_mfma_f32_32x32x2_f32
// (64 cycles each): 5.3x less matrix-core time for the same tile.  Tile, XCD remap and the fused
// epilogue are those of the fp32 kernel (cell_tile.h); the epilogue writes the next iteration's
// split planes of H' (and the fp32 H' only when asked, e.g. on the last iteration).
#include "cell_tile.h"

namespace iadmm {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
constexpr int kLD16 = 40;  // halfs per LDS row: 32 + 8 pad (80 B: conflict-free ds_read_b128)

// wscale[0] = 2^s, wscale[1] = 2^-s with max|U| 2^s in [0.5, 1) (1, 1 for all-zero weights).
// One workgroup, fixed-order reduction (deterministic).
__global__ __launch_bounds__(1024) void wscale_kernel(int64_t n, const float* U0, const float* U1,
                                                      const float* U2, const float* U3, float* wscale) {
  __shared__ float red[16];
  float m = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 1024)
    m = fmaxf(m, fmaxf(fmaxf(fabsf(U0[i]), fabsf(U1[i])), fmaxf(fabsf(U2[i]), fabsf(U3[i]))));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float mm = red[0];
    for (int w = 1; w < 16; ++w) mm = fmaxf(mm, red[w]);
    int e = 0;
    if (mm > 0.f && mm < INFINITY) frexpf(mm, &e);  // mm = f 2^e, f in [0.5, 1)
    wscale[0] = ldexpf(1.f, -e);
    wscale[1] = ldexpf(1.f, e);
  }
}

// Upk16[((jt*nkc + kc)*2 + plane)*4096 + (g*32 + jj)*32 + kk] = split(2^s U_g[kc*32+kk][jt*32+jj])
__global__ void pack_f16x3_kernel(int h, int njt, int nkc, const float* U0, const float* U1, const float* U2,
                                  const float* U3, const float* wscale, _Float16* Upk16) {
  const float sc = wscale[0];
  const int64_t tot = (int64_t)njt * nkc * 128 * kBK;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < tot; i += (int64_t)gridDim.x * blockDim.x) {
    const int kk = (int)(i % kBK);
    int64_t t = i / kBK;
    const int row = (int)(t % 128);
    t /= 128;
    const int kc = (int)(t % nkc);
    const int jt = (int)(t / nkc);
    const int g = row >> 5, jj = row & 31;
    const int k = kc * kBK + kk, j = jt * kJT + jj;
    const float* U = g == 0 ? U0 : (g == 1 ? U1 : (g == 2 ? U2 : U3));
    const float v = (k < h && j < h) ? U[(int64_t)k * h + j] * sc : 0.f;
    const _Float16 hi = (_Float16)v;
    const _Float16 lo = (_Float16)(v - (float)hi);
    const int64_t base = ((int64_t)(jt * nkc + kc) * 2) * 4096 + row * 32 + kk;
    Upk16[base] = hi;
    Upk16[base + 4096] = lo;
  }
}

// Y16[0..n) = fp16(x), Y16[n..2n) = fp16(x - fp16(x))
__global__ void split_f16_kernel(int64_t n, const float* X, _Float16* Y16) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = X[i];
    const _Float16 hi = (_Float16)v;
    Y16[i] = hi;
    Y16[n + i] = (_Float16)(v - (float)hi);
  }
}

struct CellF16x3Args {
  int64_t M;
  int h, njt, nkc;
  const _Float16* H16;     // [2][M][h] split planes of H
  const float *C, *xv, *g;
  const _Float16* Upk16;
  const float *Wx, *wscale;
  float* Hn;               // fp32 H' (nullable)
  _Float16* Hn16;          // [2][M][h] split planes of H'
  float *Cn, *part;
};

template <int PRIO>
__global__ __launch_bounds__(256, 2) void cell_f16x3_kernel(CellF16x3Args a) {
  __shared__ __attribute__((aligned(16))) _Float16 sA[2 * 128 * kLD16];
  __shared__ __attribute__((aligned(16))) _Float16 sB[2 * kRows * kLD16];
  __shared__ __attribute__((aligned(16))) float sW[kWxF * kJT];

  int jt, rt;
  cell_tile_of_block(a.njt, jt, rt);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int jl = lane & 31, hf = lane >> 5;
  const int h = a.h, nkc = a.nkc;
  const int64_t M = a.M, MH = a.M * (int64_t)a.h;
  const int64_t rbase = (int64_t)rt * kRows;

  cell_fill_wpairs(a.Wx, jt, sW, tid, 256);  // pair-major, for the packed epilogue

  floatx16 acc[4][2];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[g][r][q] = 0.f;

  // staging: weights 2 planes x 128 rows x 32 halfs = 1024 x 16 B (4 per thread); H 2 planes x
  // 256 rows x 32 halfs = 2048 x 16 B (8 per thread).  Named registers (no alloca).
  const float4* Ubase = reinterpret_cast<const float4*>(a.Upk16 + (int64_t)jt * nkc * 2 * 4096);
  float4 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3, rb4, rb5, rb6, rb7;
  auto ldB = [&](int kc, int i) -> float4 {
    const int idx = tid + 256 * i, plane = idx >> 10, q = idx & 1023, row = q >> 2, c8 = q & 3;
    const int64_t R = rbase + row;
    const int k = kc * kBK + c8 * 8;
    return (R < M && k < h) ? *reinterpret_cast<const float4*>(a.H16 + plane * MH + R * h + k)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto gload = [&](int kc) {
    const float4* Ac = Ubase + (int64_t)kc * 1024;
    ra0 = Ac[tid]; ra1 = Ac[tid + 256]; ra2 = Ac[tid + 512]; ra3 = Ac[tid + 768];
    rb0 = ldB(kc, 0); rb1 = ldB(kc, 1); rb2 = ldB(kc, 2); rb3 = ldB(kc, 3);
    rb4 = ldB(kc, 4); rb5 = ldB(kc, 5); rb6 = ldB(kc, 6); rb7 = ldB(kc, 7);
  };
  auto stA = [&](int i, const float4& v) {
    const int idx = tid + 256 * i, plane = idx >> 9, q = idx & 511, row = q >> 2, c8 = q & 3;
    *reinterpret_cast<float4*>(&sA[(plane * 128 + row) * kLD16 + c8 * 8]) = v;
  };
  auto stB = [&](int i, const float4& v) {
    const int idx = tid + 256 * i, plane = idx >> 10, q = idx & 1023, row = q >> 2, c8 = q & 3;
    *reinterpret_cast<float4*>(&sB[(plane * kRows + row) * kLD16 + c8 * 8]) = v;
  };

  gload(0);
  for (int kc = 0; kc < nkc; ++kc) {
    __syncthreads();
    stA(0, ra0); stA(1, ra1); stA(2, ra2); stA(3, ra3);
    stB(0, rb0); stB(1, rb1); stB(2, rb2); stB(3, rb3);
    stB(4, rb4); stB(5, rb5); stB(6, rb6); stB(7, rb7);
    __syncthreads();
    if (kc + 1 < nkc) gload(kc + 1);
    if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(1);
    // K permutation: lane (jl, hf) feeds MFMA k-slot 8 hf + j with chunk column 16 hf + 8 s + j
    // for both operands (a bijection of the 32 columns; the sum over k is unchanged).
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ko = 16 * hf + 8 * s;
      half8 ah[4], al[4], bh[2], bl[2];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        ah[g] = *reinterpret_cast<const half8*>(&sA[(g * 32 + jl) * kLD16 + ko]);
        al[g] = *reinterpret_cast<const half8*>(&sA[(128 + g * 32 + jl) * kLD16 + ko]);
      }
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        bh[r] = *reinterpret_cast<const half8*>(&sB[(wave * 64 + r * 32 + jl) * kLD16 + ko]);
        bl[r] = *reinterpret_cast<const half8*>(&sB[(kRows + wave * 64 + r * 32 + jl) * kLD16 + ko]);
      }
      // small cross terms first, then hi*hi (8 independent accumulators between dependent MFMAs)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[g][r] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[g], bh[r], acc[g][r], 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[g][r] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[g], bl[r], acc[g][r], 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[g][r] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[g], bh[r], acc[g][r], 0, 0, 0);
    }
    if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
  }

  // ---- epilogue: the fp32 kernel's packed cell math (cell_epi_compute) on the 2^-s-rescaled
  // accumulators, + the split planes of H'
  const float inv = a.wscale[1];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int64_t R = rbase + wave * 64 + r * 32 + jl;
    const bool rok = R < M;
    const float2v in0 = splat2(rok ? a.xv[R] : 0.f), in1 = splat2(rok ? a.g[R] : 0.f);
    float2v gs = splat2(0.f);
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      __builtin_amdgcn_sched_barrier(0);
      const int jj0 = 8 * qq + 4 * hf;
      const int j0 = jt * kJT + jj0;
      const bool ok4 = rok && j0 < h;  // h % 8 == 0: the 4 units are all in range or all out
      const float4 t4 = *reinterpret_cast<const float4*>(a.C + (ok4 ? R * h + j0 : 0));
      const float4 cold = ok4 ? t4 : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 cnew, hnew;
      half4 hhi, hlo;
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const float4* wp = reinterpret_cast<const float4*>(sW + ((jj0 >> 1) + pp) * 32);
        float4 w4[7];
#pragma unroll
        for (int i = 0; i < 7; ++i) w4[i] = wp[i];
        auto fld = [&](int f) -> float2v {
          const float4& t = w4[f >> 1];
          return (f & 1) ? float2v{t.z, t.w} : float2v{t.x, t.y};
        };
        const int q = qq * 4 + 2 * pp;
        float2v pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          pre[g] = cell_pre2(in0, in1, float2v{acc[g][r][q], acc[g][r][q + 1]} * splat2(inv), fld(3 * g),
                             fld(3 * g + 1), fld(3 * g + 2));
        }
        const float2v ig = sigmoid_cell2(pre[0]), fg = sigmoid_cell2(pre[1]), og = sigmoid_cell2(pre[2]);
        const float2v ug = tanh_cell2(pre[3]);
        const float2v cv = pp ? float2v{cold.z, cold.w} : float2v{cold.x, cold.y};
        const float2v c2 = ig * ug + fg * cv;
        const float2v h2 = og * tanh_cell2(c2);
        gs = fma2(h2, fld(12), gs);
        const _Float16 hi0 = (_Float16)h2.x, hi1 = (_Float16)h2.y;
        const _Float16 lo0 = (_Float16)(h2.x - (float)hi0), lo1 = (_Float16)(h2.y - (float)hi1);
        if (pp == 0) {
          cnew.x = c2.x; cnew.y = c2.y; hnew.x = h2.x; hnew.y = h2.y;
          hhi[0] = hi0; hhi[1] = hi1; hlo[0] = lo0; hlo[1] = lo1;
        } else {
          cnew.z = c2.x; cnew.w = c2.y; hnew.z = h2.x; hnew.w = h2.y;
          hhi[2] = hi0; hhi[3] = hi1; hlo[2] = lo0; hlo[3] = lo1;
        }
      }
      if (ok4) {
        *reinterpret_cast<float4*>(a.Cn + R * h + j0) = cnew;
        if (a.Hn) *reinterpret_cast<float4*>(a.Hn + R * h + j0) = hnew;
        *reinterpret_cast<half4*>(a.Hn16 + R * h + j0) = hhi;
        *reinterpret_cast<half4*>(a.Hn16 + MH + R * h + j0) = hlo;
      }
    }
    float gsum = gs.x + gs.y;
    gsum += __shfl_xor(gsum, 32, 64);
    if (hf == 0 && rok) a.part[(int64_t)jt * M + R] = gsum;
  }
}

inline int64_t cdiv16(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace iadmm

using namespace iadmm;

extern "C" int64_t iadmm_lstm_packed16_halfs(int64_t h) { return cdiv16(h, kJT) * cdiv16(h, kBK) * 2 * 128 * kBK; }

extern "C" int iadmm_lstm_pack_f16x3(int64_t h, const float* U_i, const float* U_f, const float* U_o,
                                     const float* U_u, void* Upk16, float* wscale, void* stream) {
  if (h <= 0 || h > (1 << 16) || !U_i || !U_f || !U_o || !U_u || !Upk16 || !wscale) return IADMM_E_ARG;
  if (!aligned16(Upk16)) return IADMM_E_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(wscale_kernel, dim3(1), dim3(1024), 0, s, h * h, U_i, U_f, U_o, U_u, wscale);
  IADMM_CHECK_LAUNCH();
  const int njt = (int)cdiv16(h, kJT), nkc = (int)cdiv16(h, kBK);
  hipLaunchKernelGGL(pack_f16x3_kernel, dim3(2048), dim3(256), 0, s, (int)h, njt, nkc, U_i, U_f, U_o, U_u,
                     wscale, static_cast<_Float16*>(Upk16));
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_split_f16(int64_t n, const float* X, void* Y16, void* stream) {
  if (n <= 0 || !X || !Y16) return IADMM_E_ARG;
  const int64_t blocks = cdiv16(n, 256);
  hipLaunchKernelGGL(split_f16_kernel, dim3((unsigned)(blocks < 16384 ? blocks : 16384)), dim3(256), 0,
                     (hipStream_t)stream, n, X, static_cast<_Float16*>(Y16));
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_lstm_cell_fwd_f16x3(int64_t M, int64_t h, const void* H16, const float* C, const float* xv,
                                         const float* g, const void* Upk16, const float* Wx, const float* wscale,
                                         float* Hn, void* Hn16, float* Cn, float* part, void* stream) {
  if (M <= 0 || h <= 0 || !H16 || !C || !xv || !g || !Upk16 || !Wx || !wscale || !Hn16 || !Cn || !part)
    return IADMM_E_ARG;
  if (Hn16 == H16) return IADMM_E_ARG;  // other workgroups still read H rows
  if (h % 8) return IADMM_E_SIZE;       // 16-B groups of 8 halfs along h
  if (!aligned16(H16) || !aligned16(Hn16) || !aligned16(Upk16) || !aligned16(C) || !aligned16(Cn) ||
      (Hn && !aligned16(Hn)))
    return IADMM_E_ALIGN;
  const int64_t nrt = cdiv16(M, kRows), njt = cdiv16(h, kJT);
  if (nrt * njt > 0x7fffffffLL || h > (1 << 16)) return IADMM_E_SIZE;
  CellF16x3Args a{M, (int)h, (int)njt, (int)cdiv16(h, kBK), static_cast<const _Float16*>(H16), C, xv, g,
                  static_cast<const _Float16*>(Upk16), Wx, wscale, Hn, static_cast<_Float16*>(Hn16), Cn, part};
  hipLaunchKernelGGL(cell_f16x3_kernel<0>, dim3((unsigned)(nrt * njt)), dim3(256), 0, (hipStream_t)stream, a);
  IADMM_CHECK_LAUNCH();
  return 0;
}
