// Generic fp32-MFMA GEMMs for the training backward of the LSTM cell (models/lstm.py:74-80).
//
//   gemm_nt : out[M, Ni] (+)= X[M, K] . W[Ni, K]^T      (dH = dP . U_cat^T, K = 4h)
//   gemm_tn : out[Ni, No]  = X[M, Ni]^T . Y[M, No]      (dU_cat = H^T . dP, split over M)
//
// gemm_nt uses the forward cell kernel's tiling (workgroup = 128 outputs x 256 rows, wave = 128
// outputs x 64 rows = 8 accumulators of v_mfma_f32_32x32x2_f32) and, for K % 4 == 0 with aligned
// operands, its LDS-DMA main loop (cell_tile.h mainloop_dma); otherwise K is staged 32-deep
// through padded LDS by registers.  gemm_tn contracts over the long row dimension:
// a workgroup owns a 128 x 128 output tile and a contiguous slice of rows, stages [32 rows x 128]
// of both operands in LDS (both are row-major along the output dims, so one fragment element per
// lane is a conflict-free ds_read_b32) and writes an fp32 partial slab; iadmm_slab_reduce sums the
// slabs in a fixed order (deterministic, no atomics).
#include "cell_tile.h"

namespace iadmm {

constexpr int kGBK = 32;
constexpr int kGLD = kGBK + 4;

template <bool ACC, bool VEC>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(int64_t M, int Ni, int K, const float* X,
                                                         const float* W, float* out) {
  __shared__ __attribute__((aligned(16))) float sA[128 * kGLD];
  __shared__ __attribute__((aligned(16))) float sB[256 * kGLD];
  const int nit = (Ni + 127) / 128;
  const int it = blockIdx.x % nit;
  const int64_t rt = blockIdx.x / nit;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, jl = lane & 31, hf = lane >> 5;
  const int i0 = it * 128;
  const int64_t r0 = rt * 256;
  floatx16 acc[4][2];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[g][r][q] = 0.f;
  const int nkc = (K + kGBK - 1) / kGBK;
  float4 ra[4], rb[8];
  auto ld4 = [&](const float* base, int64_t row, int64_t nrow, int k) -> float4 {
    if constexpr (VEC) {
      return (row < nrow && k < K) ? *reinterpret_cast<const float4*>(base + row * K + k)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      float4 t;
#pragma unroll
      for (int e = 0; e < 4; ++e) set4(t, e, (row < nrow && k + e < K) ? base[row * K + k + e] : 0.f);
      return t;
    }
  };
  auto gload = [&](int kc) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + 256 * q, row = idx >> 3, c4 = idx & 7;
      ra[q] = ld4(W, i0 + row, Ni, kc * kGBK + c4 * 4);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int idx = tid + 256 * q, row = idx >> 3, c4 = idx & 7;
      rb[q] = ld4(X, r0 + row, M, kc * kGBK + c4 * 4);
    }
  };
  gload(0);
  for (int kc = 0; kc < nkc; ++kc) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + 256 * q, row = idx >> 3, c4 = idx & 7;
      *reinterpret_cast<float4*>(&sA[row * kGLD + c4 * 4]) = ra[q];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int idx = tid + 256 * q, row = idx >> 3, c4 = idx & 7;
      *reinterpret_cast<float4*>(&sB[row * kGLD + c4 * 4]) = rb[q];
    }
    __syncthreads();
    if (kc + 1 < nkc) gload(kc + 1);
#pragma unroll
    for (int G = 0; G < kGBK / 8; ++G) {
      float4 af[4], bf[2];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        af[g] = *reinterpret_cast<const float4*>(&sA[(g * 32 + jl) * kGLD + 8 * G + 4 * hf]);
#pragma unroll
      for (int r = 0; r < 2; ++r)
        bf[r] = *reinterpret_cast<const float4*>(&sB[(wave * 64 + r * 32 + jl) * kGLD + 8 * G + 4 * hf]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int r = 0; r < 2; ++r)
            acc[g][r] = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(af[g], s), get4(bf[r], s), acc[g][r], 0, 0, 0);
    }
  }
  // epilogue: accumulator q of lane (jl,hf) = out[row jl][i0 + g*32 + (q&3) + 8(q>>2) + 4hf]
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int64_t R = r0 + wave * 64 + r * 32 + jl;
    if (R >= M) continue;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int ib = i0 + g * 32 + 8 * qq + 4 * hf;
        float* o = out + R * Ni + ib;
        if (VEC && ib + 3 < Ni) {
          float4 v = make_float4(acc[g][r][4 * qq], acc[g][r][4 * qq + 1], acc[g][r][4 * qq + 2], acc[g][r][4 * qq + 3]);
          if (ACC) {
            const float4 p = *reinterpret_cast<const float4*>(o);
            v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w;
          }
          *reinterpret_cast<float4*>(o) = v;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (ib + e < Ni) o[e] = ACC ? o[e] + acc[g][r][4 * qq + e] : acc[g][r][4 * qq + e];
        }
      }
  }
}

// gemm_nt on the LDS-DMA main loop of the cell kernel (cell_tile.h mainloop_dma): K % 4 == 0,
// Ni % 4 == 0 and 16-B aligned operands.  Output tiles of NA*32 rows of W (NA = 4 or 5, whichever
// pads Ni less: 800 = 5 x 160 wastes nothing where 128-row tiles compute 12 % padding) x 256 rows
// of X.  Workgroups remapped XCD-aware like the cell kernel so the output tiles of one 256-row X
// panel run back to back on one XCD (panel reused from its L2).
// A_PACKED: W given as iadmm_gemm_pack_a's [nit][ceil(K/32)][NA*32][32] tiles (each DMA piece one
// contiguous KiB) instead of row-major [Ni][K] (16 rows x 64 B per piece).
// K16 (A_PACKED, K % 16 == 0): the VALU-free main loop (cell_tile.h mainloop_dma_k16), bitwise the
// same products and order.
// The body: rows [r0, r0 + 256) x outputs [i0, i0 + TI) over the K range [k0, k0 + Klen) of the
// Kfull-wide operands (k0 a multiple of 32; the whole K unless split), stored to out (+ its values
// when ACC).
template <bool ACC, bool A_PACKED, int NA, bool K16>
IADMM_DEV void gemm_nt_dma_tile(int64_t M, int Ni, int Kfull, int k0, int Klen, const float* X, const float* W,
                                float* out) {
  extern __shared__ __attribute__((aligned(16))) float ring[];
  constexpr int TI = NA * 32;
  const int nit = (Ni + TI - 1) / TI;
  int it, rti;
  cell_tile_of_block(nit, it, rti);
  const int64_t rt = rti;
  const int tid = threadIdx.x, lane = tid & 63, jl = lane & 31, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i0 = it * TI;
  const int64_t r0 = rt * 256;
  floatx16 acc[NA][2];
  if constexpr (A_PACKED && K16) {
    const int64_t nkc32 = (Kfull + kBK - 1) / kBK;
    mainloop_dma_k16<NA>(W + ((int64_t)it * nkc32 + k0 / kBK) * TI * kBK, X + r0 * Kfull + k0, M - r0, Kfull, Klen,
                         ring, acc, tid, wave, jl, hf, [] {});
  } else if constexpr (A_PACKED) {
    const int64_t nkc32 = (Kfull + kBK - 1) / kBK;
    mainloop_dma<true, NA>(W + (int64_t)it * nkc32 * TI * kBK, TI, kBK, X + r0 * Kfull, M - r0, Kfull, Kfull, ring,
                           acc, tid, wave, jl, hf, [] {});
  } else {
    mainloop_dma<false, NA>(W + (int64_t)i0 * Kfull, Ni - i0, Kfull, X + r0 * Kfull, M - r0, Kfull, Kfull, ring,
                            acc, tid, wave, jl, hf, [] {});
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int64_t R = r0 + wave * 64 + r * 32 + jl;
    if (R >= M) continue;
#pragma unroll
    for (int g = 0; g < NA; ++g)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int ib = i0 + g * 32 + 8 * qq + 4 * hf;
        float* o = out + R * Ni + ib;
        if (ib < Ni) {  // Ni % 4 == 0: the 4 outputs are all in range or all out
          float4 v = make_float4(acc[g][r][4 * qq], acc[g][r][4 * qq + 1], acc[g][r][4 * qq + 2], acc[g][r][4 * qq + 3]);
          if (ACC) {
            const float4 p = *reinterpret_cast<const float4*>(o);
            v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w;
          }
          *reinterpret_cast<float4*>(o) = v;
        }
      }
  }
}

template <bool ACC, bool A_PACKED, int NA, bool K16 = false>
__global__ __launch_bounds__(256, 2) void gemm_nt_dma_kernel(int64_t M, int Ni, int K, const float* X,
                                                             const float* W, float* out) {
  gemm_nt_dma_tile<ACC, A_PACKED, NA, K16>(M, Ni, K, 0, K, X, W, out);
}

// K split (r06, small M: the recipe's batch 2 has M = 4000 rows = 80 output tiles, a third of the
// CUs): split blockIdx.y takes the K range [kpart * y, min(K, kpart * (y + 1))) (kpart % 32 == 0)
// and writes its partial product to slab[y][M][Ni]; iadmm_slab_reduce sums the slabs in split
// order.  Packed W, K % 16 == 0 (the VALU-free loop).
template <int NA>
__global__ __launch_bounds__(256, 2) void gemm_nt_dma_split_kernel(int64_t M, int Ni, int K, int kpart,
                                                                   const float* X, const float* W, float* slab) {
  const int k0 = kpart * (int)blockIdx.y;
  const int klen = min(kpart, K - k0);
  gemm_nt_dma_tile<false, true, NA, true>(M, Ni, K, k0, klen, X, W, slab + (int64_t)blockIdx.y * M * Ni);
}

// Output-tile height of the DMA gemm_nt: 160 rows when that pads Ni less than 128 rows would.
inline int gemm_nt_tile(int64_t Ni) {
  const int64_t w128 = (Ni + 127) / 128 * 128 - Ni, w160 = (Ni + 159) / 160 * 160 - Ni;
  return w160 < w128 ? 160 : 128;
}

template <bool ACC, bool A_PACKED, int NA, bool K16>
int launch_gemm_nt_dma_t(dim3 grid, int64_t M, int64_t Ni, int64_t K, const float* X, const float* W, float* out,
                         hipStream_t s) {
  constexpr int lds = dma_ring_floats<NA>() * 4;
  IADMM_ALLOW_LDS((gemm_nt_dma_kernel<ACC, A_PACKED, NA, K16>), lds);
  hipLaunchKernelGGL((gemm_nt_dma_kernel<ACC, A_PACKED, NA, K16>), grid, dim3(256), lds, s, M, (int)Ni, (int)K, X, W,
                     out);
  IADMM_CHECK_LAUNCH();
  return 0;
}

template <bool ACC, bool A_PACKED>
int launch_gemm_nt_dma(int64_t M, int64_t Ni, int64_t K, const float* X, const float* W, float* out, hipStream_t s) {
  const int ti = gemm_nt_tile(Ni);
  const int64_t nit = (Ni + ti - 1) / ti, nrt = (M + 255) / 256;
  if (nit * nrt > 0x7fffffffLL) return IADMM_E_SIZE;
  const dim3 grid((unsigned)(nit * nrt));
  const bool k16 = A_PACKED && K % kBKd == 0;
  if (ti == 160)
    return k16 ? launch_gemm_nt_dma_t<ACC, A_PACKED, 5, A_PACKED>(grid, M, Ni, K, X, W, out, s)
               : launch_gemm_nt_dma_t<ACC, A_PACKED, 5, false>(grid, M, Ni, K, X, W, out, s);
  return k16 ? launch_gemm_nt_dma_t<ACC, A_PACKED, 4, A_PACKED>(grid, M, Ni, K, X, W, out, s)
             : launch_gemm_nt_dma_t<ACC, A_PACKED, 4, false>(grid, M, Ni, K, X, W, out, s);
}

// Wpk[((it * nkc32 + kc) * TI + row) * 32 + kk] = W[it*TI + row][kc*32 + kk]  (0 outside)
__global__ void gemm_pack_a_kernel(int Ni, int K, int TI, int nit, int nkc32, const float* W, float* Wpk) {
  const int64_t tot = (int64_t)nit * nkc32 * TI * kBK;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < tot; i += (int64_t)gridDim.x * blockDim.x) {
    const int kk = (int)(i % kBK);
    int64_t t = i / kBK;
    const int row = (int)(t % TI);
    t /= TI;
    const int kc = (int)(t % nkc32);
    const int it = (int)(t / nkc32);
    const int r = it * TI + row, k = kc * kBK + kk;
    Wpk[i] = (r < Ni && k < K) ? W[(int64_t)r * K + k] : 0.f;
  }
}

// Partial slab of X[rows, Ni]^T . Y[rows, No] for the row slice of blockIdx.z.
__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(int64_t M, int Ni, int No, int64_t rows_per_split,
                                                         const float* X, const float* Y, float* slab) {
  __shared__ __attribute__((aligned(16))) float sX[kGBK][128 + 4];
  __shared__ __attribute__((aligned(16))) float sY[kGBK][128 + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, jl = lane & 31, hf = lane >> 5;
  const int i0 = blockIdx.x * 128, o0 = blockIdx.y * 128;
  const int64_t rbeg = (int64_t)blockIdx.z * rows_per_split;
  const int64_t rend = min(M, rbeg + rows_per_split);
  const int wi = (wave >> 1) * 64, wo = (wave & 1) * 64;  // wave tile 64 (i) x 64 (o)
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[a][c][q] = 0.f;
  const bool vx = (Ni % 4 == 0) && aligned16(X), vy = (No % 4 == 0) && aligned16(Y);
  // Loads are not register-prefetched: at 102 VGPRs four workgroups share a CU and hide each
  // other's load latency (a prefetching variant needed 139 VGPRs, ran 3 per CU and was 30 %
  // slower; tools/gemmbench.py).
  for (int64_t rc = rbeg; rc < rend; rc += kGBK) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // 32 rows x 32 float4 per operand, 4 per thread
      const int idx = tid + 256 * q, rr = idx >> 5, c4 = (idx & 31) * 4;
      const int64_t r = rc + rr;
      const bool ok = r < rend;
      float4 tx, ty;
      if (vx && i0 + c4 + 3 < Ni) tx = ok ? *reinterpret_cast<const float4*>(X + r * Ni + i0 + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
      else for (int e = 0; e < 4; ++e) set4(tx, e, (ok && i0 + c4 + e < Ni) ? X[r * Ni + i0 + c4 + e] : 0.f);
      if (vy && o0 + c4 + 3 < No) ty = ok ? *reinterpret_cast<const float4*>(Y + r * No + o0 + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
      else for (int e = 0; e < 4; ++e) set4(ty, e, (ok && o0 + c4 + e < No) ? Y[r * No + o0 + c4 + e] : 0.f);
      *reinterpret_cast<float4*>(&sX[rr][c4]) = tx;
      *reinterpret_cast<float4*>(&sY[rr][c4]) = ty;
    }
    __syncthreads();
#pragma unroll 4
    for (int ks = 0; ks < kGBK / 2; ++ks) {
      const int kk = 2 * ks + hf;
      float av[2], bv[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) av[a] = sX[kk][wi + a * 32 + jl];
#pragma unroll
      for (int c = 0; c < 2; ++c) bv[c] = sY[kk][wo + c * 32 + jl];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c)
          acc[a][c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[c], acc[a][c], 0, 0, 0);
    }
  }
  float* S = slab + (int64_t)blockIdx.z * Ni * No;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = i0 + wi + a * 32 + (q & 3) + 8 * (q >> 2) + 4 * hf;
        const int o = o0 + wo + c * 32 + jl;
        if (i < Ni && o < No) S[(int64_t)i * No + o] = acc[a][c][q];
      }
}

// gemm_tn on an LDS-DMA ring (the cell kernel's pipeline with the contraction over rows):
// workgroup = NA*32 (i) x 256 (o) outputs of one row split (NA = 4 or 5 as for gemm_nt: 160-wide
// i tiles cover Ni = 800 exactly), wave = NA*32 (i) x 64 (o) = NA x 2 accumulators of
// v_mfma_f32_32x32x2_f32.  Per 16-row chunk the workgroup DMAs the X panel (16 rows x NA*32
// columns, lane-linear KiB pieces) and 16 Y pieces (1 row x 256 columns each) into a 3-stage ring,
// row-major as in HBM; fragments are ds_read_b32 of 32 consecutive columns of one row per
// half-wave (conflict-free without a swizzle).  Rows past the split and columns past Ni / No read
// as zero (buffer range / out-of-range offsets).  One barrier per chunk; the chunk kc+2 DMA is
// issued after it, into the stage chunk kc-1 used.  Requires Ni % 4 == No % 4 == 0 and 16-B
// aligned X, Y.
template <int NA>
constexpr int tn_ring_floats() {
  return 3 * (16 * NA * 32 + 16 * 256) + ((NA * 2) % 4 ? 256 : 0);  // + the dummy-piece KiB
}

// The main loop issues no VALU work (gfx950: the fp32 MFMA shares the VALU datapath, every VALU
// instruction beside it is matrix time lost; tools/mfma_valu_probe.hip):
//   * each DMA piece keeps a loop-invariant per-lane voffset; the chunk's rows come in through a
//     per-chunk descriptor (base at the chunk's first row, range ending at the split's last row:
//     SALU only), so rows past the split read zero with no per-lane check;
//   * the chunk loop is unrolled by the 3 ring stages, so every fragment read is a loop-invariant
//     lane address + an immediate (stage 2 from its own lane bases: the ring is 78 KiB and the
//     ds_read offset field reaches 64 KiB).
// Same products in the same order as the r01 loop: bitwise the same slab.
template <int NA>
IADMM_DEV void gemm_tn_dma_body(int64_t M, int Ni, int No, int64_t rows_per_split, const float* X, const float* Y,
                                float* slab, float* ring) {
  constexpr int TI = NA * 32, SX = 16 * TI, SY = 16 * 256, ST = SX + SY, NPX = NA * 2, XPW = (NPX + 3) / 4;
  const int tid = threadIdx.x, lane = tid & 63, jl = lane & 31, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i0 = blockIdx.x * TI, o0 = blockIdx.y * 256;
  const int64_t rbeg = (int64_t)blockIdx.z * rows_per_split;
  const int64_t rend = min(M, rbeg + rows_per_split);
  const int nrows = (int)(rend - rbeg);
  const int nk = (nrows + 15) / 16;
  floatx16 acc[NA][2];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[a][c][q] = 0.f;
  // X piece p (wave p % 4) = stage floats [256p, 256p + 256): lane -> float 256p + 4*lane, i.e.
  // row / column of the [16][TI] image; a wave with no piece left issues an out-of-range dummy
  // into the KiB after the ring.  Y piece q = stage row q, columns o0 + 4*lane .. +4.  Offsets are
  // relative to the chunk's first row.
  unsigned xoff[XPW], yoff[4];
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int p = wave + 4 * i, idx = 256 * p + 4 * lane;
    const int row = idx / TI, col = i0 + idx % TI;
    xoff[i] = (p < NPX && col < Ni) ? (unsigned)(row * Ni + col) * 4u : 0x80000000u;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wave * 4 + i, col = o0 + lane * 4;
    yoff[i] = (col < No) ? (unsigned)(row * No + col) * 4u : 0x80000000u;
  }
  auto issue = [&](int kc, auto S) {
    constexpr int st = decltype(S)::value;
    const int64_t r0 = rbeg + (int64_t)kc * 16;
    const int left = nrows - kc * 16;  // >= 1: chunks are issued only below nk
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(X + r0 * Ni), 0,
                                                                          left * Ni * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Y + r0 * No), 0,
                                                                          left * No * 4, 0x00020000);
    float* sx = ring + st * ST;
    float* sy = sx + SX;
#pragma unroll
    for (int i = 0; i < XPW; ++i) {
      const int p = wave + 4 * i;
      float* dst = (NPX % 4 == 0 || p < NPX) ? sx + p * 256 : ring + 3 * ST;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void*)dst, 16, xoff[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yrs, (lds_void*)(sy + (wave * 4 + i) * 256), 16, yoff[i], 0, 0, 0);
  };
  // fragment lane addresses (LDS bytes, ring base folded in): row kk = 2 ks + hf of the stage,
  // X columns a*32 + jl, Y columns wave*64 + c*32 + jl; [1] = the same + stage 2's base.  One
  // register per column block, laundered once per chunk: reads sharing a base register would be
  // paired into ds_read2_b32, whose 8-bit offsets need a v_add per pair.
  typedef __attribute__((address_space(3))) float lds_float;
  typedef __attribute__((address_space(3))) const float lds_cfloat;
  const unsigned rb = (unsigned)(uintptr_t)(lds_float*)ring;
  unsigned xb[2][NA], yb[2][2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
#pragma unroll
    for (int a = 0; a < NA; ++a) xb[g][a] = rb + (unsigned)(g * 2 * ST + hf * TI + a * 32 + jl) * 4u;
#pragma unroll
    for (int c = 0; c < 2; ++c) yb[g][c] = rb + (unsigned)(g * 2 * ST + SX + hf * 256 + wave * 64 + c * 32 + jl) * 4u;
  }
  auto launder = [&] {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
#pragma unroll
      for (int a = 0; a < NA; ++a) asm volatile("" : "+v"(xb[g][a]));
      asm volatile("" : "+v"(yb[g][0]), "+v"(yb[g][1]));
    }
  };
  auto ld = [](unsigned addr) -> float { return *(lds_cfloat*)(uintptr_t)addr; };
  auto frag = [&](auto S, int ks, float (&av)[NA], float (&bv)[2]) {
    constexpr int st = decltype(S)::value;
    constexpr int g = st == 2;
    constexpr unsigned so = st == 2 ? 0u : st * ST * 4u;
#pragma unroll
    for (int a = 0; a < NA; ++a) av[a] = ld(xb[g][a] + so + (unsigned)(2 * ks * TI) * 4u);
#pragma unroll
    for (int c = 0; c < 2; ++c) bv[c] = ld(yb[g][c] + so + (unsigned)(2 * ks * 256) * 4u);
  };
  // A wave whose 64 output columns all lie past No (the last o tile when No % 256 != 0, e.g. the
  // half-empty 13th tile of No = 4h = 3200) skips its MFMAs: its SIMD's matrix pipe goes to the
  // co-resident workgroup instead of multiplying zeros.
  const bool wact = o0 + wave * 64 < No;
  auto mma = [&](const float (&av)[NA], const float (&bv)[2]) {
    if (!wact) return;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c)
        acc[a][c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[c], acc[a][c], 0, 0, 0);
  };
  float av0[NA], bv0[2], av1[NA], bv1[2];
  // One barrier per chunk, after its first half: each wave has waited for its own pieces of chunk
  // kc+1 (chunk kc+2 not yet issued), so after the barrier chunk kc+1 is readable and the stage of
  // chunk kc-1 is free for chunk kc+2.  The first fragments of chunk kc+1 are read during the
  // second half of chunk kc, so no chunk starts on an LDS-latency stall.
  auto step = [&](int kc, auto S) {
    constexpr int st = decltype(S)::value;
    launder();
#pragma unroll
    for (int ks = 0; ks < 4; ks += 2) {
      frag(S, ks + 1, av1, bv1);
      mma(av0, bv0);
      frag(S, ks + 2, av0, bv0);
      mma(av1, bv1);
    }
    __builtin_amdgcn_sched_barrier(0);
    const bool more = kc + 1 < nk;
    if (more) {
      vm_wait<0>();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (kc + 2 < nk) issue(kc + 2, Stage<(st + 2) % 3>{});
    }
#pragma unroll
    for (int ks = 4; ks < 8; ks += 2) {
      frag(S, ks + 1, av1, bv1);
      mma(av0, bv0);
      if (ks + 2 < 8) frag(S, ks + 2, av0, bv0);
      else if (more) frag(Stage<(st + 1) % 3>{}, 0, av0, bv0);
      mma(av1, bv1);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  issue(0, Stage<0>{});
  if (nk > 1) issue(1, Stage<1>{});
  if (nk > 1) vm_wait<XPW + 4>(); else vm_wait<0>();
  __builtin_amdgcn_s_barrier();
  frag(Stage<0>{}, 0, av0, bv0);
  int kc = 0;
  for (; kc + 3 <= nk; kc += 3) {  // one exit: the chunk index stays scalar
    step(kc, Stage<0>{});
    step(kc + 1, Stage<1>{});
    step(kc + 2, Stage<2>{});
  }
  if (kc < nk) step(kc, Stage<0>{});
  if (kc + 1 < nk) step(kc + 1, Stage<1>{});
  float* S = slab + (int64_t)blockIdx.z * Ni * No;
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = i0 + a * 32 + (q & 3) + 8 * (q >> 2) + 4 * hf;
        const int o = o0 + wave * 64 + c * 32 + jl;
        if (i < Ni && o < No) S[(int64_t)i * No + o] = acc[a][c][q];
      }
}

// (two plain kernels: a __global__ template instantiated from the extern "C" launcher got no host
// stub from this hipcc)
__global__ __launch_bounds__(256, 2) void gemm_tn_dma4_kernel(int64_t M, int Ni, int No, int64_t rps, const float* X,
                                                              const float* Y, float* slab) {
  extern __shared__ __attribute__((aligned(16))) float ring[];
  gemm_tn_dma_body<4>(M, Ni, No, rps, X, Y, slab, ring);
}
__global__ __launch_bounds__(256, 2) void gemm_tn_dma5_kernel(int64_t M, int Ni, int No, int64_t rps, const float* X,
                                                              const float* Y, float* slab) {
  extern __shared__ __attribute__((aligned(16))) float ring[];
  gemm_tn_dma_body<5>(M, Ni, No, rps, X, Y, slab, ring);
}

// Skinny X^T Y (Ni <= 4, e.g. the [xv, g, 1]^T dP bias/input-weight gradient): a streaming
// kernel that reads Y once (HBM-bound; the 128x128 MFMA tile would do 32-128x redundant work).
// slab[s][i][c] = sum over rows of split s of X[r][i] * Y[r][c]; thread = 4 adjacent columns.
template <int NI, bool VEC>
__global__ __launch_bounds__(256) void gemm_tn_skinny_kernel(int64_t M, int No, int64_t rps, const float* X,
                                                             const float* Y, float* slab) {
  const int64_t sp = blockIdx.y;
  const int c = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (c >= No) return;  // no barrier in this kernel
  const int64_t r0 = sp * rps, r1 = (r0 + rps < M) ? r0 + rps : M;
  float acc[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[i][e] = 0.f;
#pragma unroll 4
  for (int64_t r = r0; r < r1; ++r) {
    float4 y;
    if constexpr (VEC) {
      y = *reinterpret_cast<const float4*>(Y + r * No + c);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) set4(y, e, c + e < No ? Y[r * No + c + e] : 0.f);
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const float xi = X[r * NI + i];
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[i][e] = fmaf(xi, get4(y, e), acc[i][e]);
    }
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    float* o = slab + (sp * NI + i) * (int64_t)No + c;
    if constexpr (VEC) {
      *reinterpret_cast<float4*>(o) = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c + e < No) o[e] = acc[i][e];
    }
  }
}

template <int NI>
void launch_skinny(int64_t M, int No, int64_t rps, int64_t ns, const float* X, const float* Y, float* slab,
                   hipStream_t s) {
  const dim3 grid((unsigned)((No + 1023) / 1024), (unsigned)ns);
  if (No % 4 == 0 && aligned16(Y) && aligned16(slab))
    hipLaunchKernelGGL((gemm_tn_skinny_kernel<NI, true>), grid, dim3(256), 0, s, M, No, rps, X, Y, slab);
  else
    hipLaunchKernelGGL((gemm_tn_skinny_kernel<NI, false>), grid, dim3(256), 0, s, M, No, rps, X, Y, slab);
}

// out[e] (+)= sum_{s < nsplit} slab[s][e]  (fixed order)
__global__ void slab_reduce_kernel(int64_t nelem, int nsplit, const float* slab, float* out, int acc) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nelem; e += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < nsplit; ++k) s += slab[(int64_t)k * nelem + e];
    out[e] = acc ? out[e] + s : s;
  }
}

// The same sums, four adjacent elements per thread (16-B loads) and eight splits in flight per
// thread (loads issued together, adds kept in split order: bitwise the same as slab_reduce_kernel).
// nelem % 4 == 0, 16-B aligned slab and out.
__global__ void slab_reduce4_kernel(int64_t nelem, int nsplit, const float* slab, float* out, int acc) {
  const int64_t n4 = nelem / 4;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n4; e += (int64_t)gridDim.x * blockDim.x) {
    const float4* p = reinterpret_cast<const float4*>(slab) + e;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int k = 0;
    for (; k + 8 <= nsplit; k += 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(k + u) * n4];
#pragma unroll
      for (int u = 0; u < 8; ++u) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
    for (; k < nsplit; ++k) {
      const float4 v = p[(int64_t)k * n4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    float4* o = reinterpret_cast<float4*>(out) + e;
    if (acc) {
      const float4 q = *o;
      s = make_float4(q.x + s.x, q.y + s.y, q.z + s.z, q.w + s.w);
    }
    *o = s;
  }
}

static int launch_slab_reduce(int64_t nelem, int64_t ns, const float* slab, float* out, int accumulate,
                              hipStream_t s) {
  if (nelem % 4 == 0 && aligned16(slab) && aligned16(out)) {
    const int64_t blocks = (nelem / 4 + 255) / 256;
    hipLaunchKernelGGL(slab_reduce4_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0, s,
                       nelem, (int)ns, slab, out, accumulate);
  } else {
    const int64_t blocks = (nelem + 255) / 256;
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s,
                       nelem, (int)ns, slab, out, accumulate);
  }
  IADMM_CHECK_LAUNCH();
  return 0;
}

}  // namespace iadmm

using namespace iadmm;

extern "C" int iadmm_gemm_nt(int64_t M, int64_t Ni, int64_t K, const float* X, const float* W,
                             float* out, int accumulate, void* stream) {
  if (M <= 0 || Ni <= 0 || K <= 0 || !X || !W || !out) return IADMM_E_ARG;
  const int64_t nit = (Ni + 127) / 128, nrt = (M + 255) / 256;
  if (nit * nrt > 0x7fffffffLL || Ni > (1 << 20) || K > (1 << 20)) return IADMM_E_SIZE;
  const dim3 grid((unsigned)(nit * nrt));
  const bool vec = (K % 4 == 0) && (Ni % 4 == 0) && aligned16(X) && aligned16(W) && aligned16(out);
  hipStream_t s = (hipStream_t)stream;
  const bool dma = vec && K * 256 * 4 <= 0x7fffffffLL;  // the DMA kernel's epilogue stores float4 rows
  if (dma) {
    return accumulate ? launch_gemm_nt_dma<true, false>(M, Ni, K, X, W, out, s)
                      : launch_gemm_nt_dma<false, false>(M, Ni, K, X, W, out, s);
  } else if (accumulate) {
    if (vec) hipLaunchKernelGGL((gemm_nt_kernel<true, true>), grid, dim3(256), 0, s, M, (int)Ni, (int)K, X, W, out);
    else hipLaunchKernelGGL((gemm_nt_kernel<true, false>), grid, dim3(256), 0, s, M, (int)Ni, (int)K, X, W, out);
  } else {
    if (vec) hipLaunchKernelGGL((gemm_nt_kernel<false, true>), grid, dim3(256), 0, s, M, (int)Ni, (int)K, X, W, out);
    else hipLaunchKernelGGL((gemm_nt_kernel<false, false>), grid, dim3(256), 0, s, M, (int)Ni, (int)K, X, W, out);
  }
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t iadmm_gemm_packed_a_floats(int64_t Ni, int64_t K) {
  const int ti = gemm_nt_tile(Ni);
  return ((Ni + ti - 1) / ti) * ((K + kBK - 1) / kBK) * ti * kBK;
}

extern "C" int iadmm_gemm_pack_a(int64_t Ni, int64_t K, const float* W, float* Wpk, void* stream) {
  if (Ni <= 0 || K <= 0 || !W || !Wpk) return IADMM_E_ARG;
  if (Ni > (1 << 20) || K > (1 << 20)) return IADMM_E_SIZE;
  if (!aligned16(Wpk)) return IADMM_E_ALIGN;
  const int ti = gemm_nt_tile(Ni);
  hipLaunchKernelGGL(gemm_pack_a_kernel, dim3(2048), dim3(256), 0, (hipStream_t)stream, (int)Ni, (int)K, ti,
                     (int)((Ni + ti - 1) / ti), (int)((K + kBK - 1) / kBK), W, Wpk);
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_gemm_nt_packed(int64_t M, int64_t Ni, int64_t K, const float* X, const float* Wpk,
                                    float* out, int accumulate, void* stream) {
  if (M <= 0 || Ni <= 0 || K <= 0 || !X || !Wpk || !out) return IADMM_E_ARG;
  if (Ni > (1 << 20) || K > (1 << 20) || K * 256 * 4 > 0x7fffffffLL) return IADMM_E_SIZE;
  if (K % 4 || Ni % 4 || !aligned16(X) || !aligned16(Wpk) || !aligned16(out)) return IADMM_E_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  return accumulate ? launch_gemm_nt_dma<true, true>(M, Ni, K, X, Wpk, out, s)
                    : launch_gemm_nt_dma<false, true>(M, Ni, K, X, Wpk, out, s);
}

extern "C" int iadmm_gemm_nt_packed_split(int64_t M, int64_t Ni, int64_t K, int64_t ksplit, const float* X,
                                          const float* Wpk, float* slab, float* out, int accumulate, void* stream) {
  if (M <= 0 || Ni <= 0 || K <= 0 || ksplit <= 0 || !X || !Wpk || !out) return IADMM_E_ARG;
  if (ksplit == 1) return iadmm_gemm_nt_packed(M, Ni, K, X, Wpk, out, accumulate, stream);
  if (!slab) return IADMM_E_ARG;
  if (Ni > (1 << 20) || K > (1 << 20) || K * 256 * 4 > 0x7fffffffLL || ksplit > 65535) return IADMM_E_SIZE;
  if (K % 16 || Ni % 4 || !aligned16(X) || !aligned16(Wpk) || !aligned16(slab) || !aligned16(out)) return IADMM_E_ALIGN;
  const int64_t kpart = iadmm_gemm_nt_kpart(K, ksplit);
  if ((K + kpart - 1) / kpart != ksplit) return IADMM_E_ARG;  // every split non-empty
  const int ti = gemm_nt_tile(Ni);
  const int64_t nit = (Ni + ti - 1) / ti, nrt = (M + 255) / 256;
  if (nit * nrt > 0x7fffffffLL) return IADMM_E_SIZE;
  const dim3 grid((unsigned)(nit * nrt), (unsigned)ksplit);
  hipStream_t s = (hipStream_t)stream;
  if (ti == 160) {
    constexpr int lds = dma_ring_floats<5>() * 4;
    IADMM_ALLOW_LDS(gemm_nt_dma_split_kernel<5>, lds);
    hipLaunchKernelGGL(gemm_nt_dma_split_kernel<5>, grid, dim3(256), lds, s, M, (int)Ni, (int)K, (int)kpart, X, Wpk, slab);
  } else {
    constexpr int lds = dma_ring_floats<4>() * 4;
    IADMM_ALLOW_LDS(gemm_nt_dma_split_kernel<4>, lds);
    hipLaunchKernelGGL(gemm_nt_dma_split_kernel<4>, grid, dim3(256), lds, s, M, (int)Ni, (int)K, (int)kpart, X, Wpk, slab);
  }
  IADMM_CHECK_LAUNCH();
  return launch_slab_reduce(M * Ni, ksplit, slab, out, accumulate, s);
}

extern "C" int64_t iadmm_gemm_nt_kpart(int64_t K, int64_t ksplit) {
  if (K <= 0 || ksplit <= 0) return 0;
  return ((K + ksplit - 1) / ksplit + 31) / 32 * 32;
}

extern "C" int64_t iadmm_gemm_tn_splits(int64_t M, int64_t rows_per_split) {
  return (M + rows_per_split - 1) / rows_per_split;
}

extern "C" int iadmm_gemm_tn(int64_t M, int64_t Ni, int64_t No, int64_t rows_per_split, const float* X,
                             const float* Y, float* slab, float* out, int accumulate, void* stream) {
  if (M <= 0 || Ni <= 0 || No <= 0 || rows_per_split <= 0 || !X || !Y || !slab || !out) return IADMM_E_ARG;
  if (rows_per_split % kGBK) return IADMM_E_ARG;
  const int64_t ns = (M + rows_per_split - 1) / rows_per_split;
  if (ns > 65535 || Ni > (1 << 20) || No > (1 << 20)) return IADMM_E_SIZE;
  hipStream_t s = (hipStream_t)stream;
  switch (Ni) {
    case 1: launch_skinny<1>(M, (int)No, rows_per_split, ns, X, Y, slab, s); break;
    case 2: launch_skinny<2>(M, (int)No, rows_per_split, ns, X, Y, slab, s); break;
    case 3: launch_skinny<3>(M, (int)No, rows_per_split, ns, X, Y, slab, s); break;
    case 4: launch_skinny<4>(M, (int)No, rows_per_split, ns, X, Y, slab, s); break;
    default: {
      const bool dma = Ni % 4 == 0 && No % 4 == 0 && aligned16(X) && aligned16(Y) && rows_per_split % 16 == 0 &&
                       rows_per_split * (Ni > No ? Ni : No) * 4 <= 0x7fffffffLL;
      if (dma && gemm_nt_tile(Ni) == 160) {
        const dim3 grid((unsigned)((Ni + 159) / 160), (unsigned)((No + 255) / 256), (unsigned)ns);
        constexpr int lds = tn_ring_floats<5>() * 4;
        IADMM_ALLOW_LDS(gemm_tn_dma5_kernel, lds);
        hipLaunchKernelGGL(gemm_tn_dma5_kernel, grid, dim3(256), lds, s, M, (int)Ni, (int)No, rows_per_split, X, Y,
                           slab);
      } else if (dma) {
        const dim3 grid((unsigned)((Ni + 127) / 128), (unsigned)((No + 255) / 256), (unsigned)ns);
        constexpr int lds = tn_ring_floats<4>() * 4;
        IADMM_ALLOW_LDS(gemm_tn_dma4_kernel, lds);
        hipLaunchKernelGGL(gemm_tn_dma4_kernel, grid, dim3(256), lds, s, M, (int)Ni, (int)No, rows_per_split, X, Y,
                           slab);
      } else {
        const dim3 grid((unsigned)((Ni + 127) / 128), (unsigned)((No + 127) / 128), (unsigned)ns);
        hipLaunchKernelGGL(gemm_tn_kernel, grid, dim3(256), 0, s, M, (int)Ni, (int)No, rows_per_split, X, Y, slab);
      }
    }
  }
  IADMM_CHECK_LAUNCH();
  return launch_slab_reduce(Ni * No, ns, slab, out, accumulate, s);
}

extern "C" int iadmm_slab_reduce(int64_t nelem, int64_t nsplit, const float* slab, float* out, int accumulate,
                                 void* stream) {
  if (nelem <= 0 || nsplit <= 0 || !slab || !out) return IADMM_E_ARG;
  return launch_slab_reduce(nelem, nsplit, slab, out, accumulate, (hipStream_t)stream);
}
