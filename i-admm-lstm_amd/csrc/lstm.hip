// Fused coordinate-wise LSTM cell on fp32 MFMA (gfx950 v_mfma_f32_32x32x2_f32).
//
// Reference: models/lstm.py:74-80.  For every row r of the M = B*(n+m) coordinate rows and every
// hidden unit j:
//   pre_g[r,j] = (in0[r] W_g[0,j] + in1[r] W_g[1,j]) + sum_k H[r,k] U_g[k,j] + b_g[j]
//   I,F,O = sigmoid(pre_{i,f,o}), U = tanh(pre_u), C' = I U + F C, H' = O tanh(C')
//   part[tile(j)][r] += H'[r,j] W_h[j]      (the output projection, reduced per 32-unit tile)
//
// GEMM shape: rows M (2.048M at the bench config) x 4h gate columns x K = h.  The weights are the
// MFMA "A" operand (M-dim of the instruction = hidden unit), H is the "B" operand (N-dim = data
// row), so the accumulator of one wave holds, for its 64 data rows and 32 hidden units, all FOUR
// gates at the same register index: the whole cell update runs in registers in the epilogue.
//
// Tile: workgroup = 4 waves = 32 hidden units x 256 rows; wave = 32 hidden x 64 rows x 4 gates
// (8 accumulators of 32x32 = 128 acc registers).  K is staged in 16-deep chunks through a 3-stage
// LDS ring filled by LDS-DMA (buffer_load_dwordx4 ... lds; cell_tile.h cell_mainloop_dma), one
// barrier per chunk, fragments double-buffered in registers; the epilogue's C / xv / g operands are
// loaded behind the last chunk's MFMAs.  (h % 4 != 0 or unaligned rows: the register-staged
// 32-deep loop, cell_mainloop, same products in the same order.)  Workgroups are remapped XCD-aware so the njt
// hidden tiles of one 256-row H panel run back to back on the same XCD (panel read from HBM once,
// then served by that XCD's L2).
#include "cell_tile.h"

namespace iadmm {

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Upk[((jt*nkc + kc)*128 + g*32 + jj)*32 + kk] = U_g[kc*32 + kk][jt*32 + jj]  (0 outside h)
__global__ void lstm_pack_kernel(int h, int njt, int nkc, const float* U0, const float* U1,
                                 const float* U2, const float* U3, float* Upk) {
  const int64_t tot = (int64_t)njt * nkc * 128 * kBK;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < tot;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int kk = (int)(i % kBK);
    int64_t t = i / kBK;
    const int row = (int)(t % 128);
    t /= 128;
    const int kc = (int)(t % nkc);
    const int jt = (int)(t / nkc);
    const int g = row >> 5, jj = row & 31;
    const int k = kc * kBK + kk, j = jt * kJT + jj;
    const float* U = g == 0 ? U0 : (g == 1 ? U1 : (g == 2 ? U2 : U3));
    Upk[i] = (k < h && j < h) ? U[(int64_t)k * h + j] : 0.f;
  }
}

struct WxSrc { const float *W[4], *b[4], *Wh; };

__global__ void lstm_pack_wx_kernel(int h, int hp, WxSrc s, float* Wx) {
  const int tot = hp * kWxF;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += gridDim.x * blockDim.x) {
    const int j = i / kWxF, f = i % kWxF;
    float v = 0.f;
    if (j < h) {
      if (f < 12) {
        const int g = f / 3, w = f % 3;
        v = w < 2 ? s.W[g][(int64_t)w * h + j] : s.b[g][j];
      } else if (f == 12) {
        v = s.Wh[j];
      }
    }
    Wx[i] = v;
  }
}

}  // namespace iadmm

using namespace iadmm;

extern "C" int64_t iadmm_lstm_ntiles(int64_t h) { return cdiv(h, kJT); }
extern "C" int64_t iadmm_lstm_packed_floats(int64_t h) { return cdiv(h, kJT) * cdiv(h, kBK) * 128 * kBK; }
extern "C" int64_t iadmm_lstm_wx_floats(int64_t h) { return cdiv(h, kJT) * kJT * kWxF; }

extern "C" int iadmm_lstm_pack(int64_t h, const float* W_i, const float* U_i, const float* b_i,
                               const float* W_f, const float* U_f, const float* b_f,
                               const float* W_o, const float* U_o, const float* b_o,
                               const float* W_u, const float* U_u, const float* b_u,
                               const float* W_h, float* Upk, float* Wx, void* stream) {
  if (h <= 0 || h > (1 << 20)) return IADMM_E_ARG;
  const float* ptrs[] = {W_i, U_i, b_i, W_f, U_f, b_f, W_o, U_o, b_o, W_u, U_u, b_u, W_h, Upk, Wx};
  for (const float* p : ptrs)
    if (!p) return IADMM_E_ARG;
  if (!aligned16(Upk)) return IADMM_E_ALIGN;
  const int njt = (int)cdiv(h, kJT), nkc = (int)cdiv(h, kBK);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(lstm_pack_kernel, dim3(2048), dim3(256), 0, s, (int)h, njt, nkc, U_i, U_f,
                     U_o, U_u, Upk);
  IADMM_CHECK_LAUNCH();
  WxSrc src{{W_i, W_f, W_o, W_u}, {b_i, b_f, b_o, b_u}, W_h};
  hipLaunchKernelGGL(lstm_pack_wx_kernel, dim3(64), dim3(256), 0, s, (int)h, njt * kJT, src, Wx);
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_lstm_cell_fwd(int64_t M, int64_t h, const float* H, const float* C,
                                   const float* xv, const float* g, const float* Upk,
                                   const float* Wx, float* Hn, float* Cn, float* part,
                                   void* stream) {
  if (M <= 0 || h <= 0 || !H || !C || !xv || !g || !Upk || !Wx || !Hn || !Cn || !part) return IADMM_E_ARG;
  if (Hn == H) return IADMM_E_ARG;  // other workgroups still read H rows
  if (!aligned16(Upk)) return IADMM_E_ALIGN;
  const int64_t nrt = cdiv(M, kRows), njt = cdiv(h, kJT);
  if (nrt * njt > 0x7fffffffLL || h > (1 << 16)) return IADMM_E_SIZE;
  // tile order: groups of 4 row panels, hidden tile slowest (cell_tile_of_block_grouped): bitwise
  // the same result as panel-major order, 29 % fewer L2 misses (tools/cellmap.py, profiles/r02_cellmap_*)
  CellArgsT a{M, (int)h, (int)njt, (int)cdiv(h, kBK), H, C, xv, g, Upk, Wx, Hn, Cn, part, 4};
  const bool vec = (h % 4 == 0) && aligned16(H) && aligned16(C) && aligned16(Hn) && aligned16(Cn);
  const dim3 grid((unsigned)(nrt * njt));
  if (vec) {
    // LDS-DMA main loop (cell_tile.h cell_mainloop_dma): 74 KiB of dynamic LDS per workgroup
    if (h % kBKd == 0) {  // no K tail: the VALU-free loop (cell_tile.h mainloop_dma_k16)
      IADMM_ALLOW_LDS((cell_fwd_dma_kernel<0, true>), kDmaLdsBytes);
      hipLaunchKernelGGL((cell_fwd_dma_kernel<0, true>), grid, dim3(256), kDmaLdsBytes, (hipStream_t)stream, a);
    } else {
      IADMM_ALLOW_LDS((cell_fwd_dma_kernel<0, false>), kDmaLdsBytes);
      hipLaunchKernelGGL((cell_fwd_dma_kernel<0, false>), grid, dim3(256), kDmaLdsBytes, (hipStream_t)stream, a);
    }
  } else
    hipLaunchKernelGGL((cell_fwd_kernel<false, 4, 0>), grid, dim3(256), 0, (hipStream_t)stream, a);
  IADMM_CHECK_LAUNCH();
  return 0;
}
