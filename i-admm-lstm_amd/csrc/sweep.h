// Row sweeps over one instance's dense matrix, the building block of every HBM-bound kernel
// (KKT residual gradient, metrics, Ruiz norms).
//
// One workgroup owns one QP instance.  Wave w streams rows w*U, w*U+nw*U, ... of a row-major
// [R x C] matrix; lane L owns a fixed set of columns:
//   VEC  (C % 4 == 0): float4 groups cg = L + 64*i (i < NG)  -> columns 4*cg .. 4*cg+3
//   !VEC            : columns L + 64*j (j < 4*NG)
// so one row is read with coalesced 16-B (or 4-B) loads, 1 KiB per wave-instruction.
// Per row the sweep can produce
//   DOT : dot_s[r] = sum_c M[r,c] * a_s[c]        (wave reduction, written by lane 0)
//   COL : col[c]  += M[r,c] * c_s[r]              (per-lane register accumulators)
// and the column accumulators of all waves are folded in a fixed order by col_reduce, so every
// result is deterministic (no atomics).
#pragma once
#include "common.h"

namespace iadmm {

template <int NG, bool VEC>
IADMM_DEV int col_of(int lane, int idx) {
  if constexpr (VEC) return 4 * (lane + 64 * (idx >> 2)) + (idx & 3);
  else return lane + 64 * idx;
}

template <int NG, bool VEC>
IADMM_DEV void load_row(const float* __restrict__ row, bool rok, int C, int lane, float (&v)[NG * 4]) {
  if constexpr (VEC) {
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const int c = 4 * (lane + 64 * i);
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
      if (rok && c < C) t = *reinterpret_cast<const float4*>(row + c);
      v[4 * i + 0] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4 * NG; ++j) {
      const int c = lane + 64 * j;
      v[j] = (rok && c < C) ? row[c] : 0.f;
    }
  }
}

// DOT/COL sweep over a column panel: rows r < R of the [R x C] panel starting at Mx with row
// stride ld (ld == C for a whole matrix); see the file comment.  ``col`` accumulates in place.
// dot_acc: dot_s[r] += (panel dot) instead of =, so DOT over several panels sums them in panel
// order (each row is always handled by the same wave, so no barrier is needed between panels).
template <int NG, bool VEC, bool DOT, bool COL>
IADMM_DEV void sweep_panel(const float* __restrict__ Mx, int R, int C, int64_t ld, const float* a_s,
                           const float* c_s, float* dot_s, bool dot_acc, float (&col)[NG * 4],
                           int wave, int nw, int lane) {
  constexpr bool HOIST = NG <= 8;
  constexpr int U = NG <= 4 ? 2 : 1;
  float av[HOIST ? NG * 4 : 1];
  if constexpr (DOT && HOIST) {
#pragma unroll
    for (int idx = 0; idx < NG * 4; ++idx) {
      const int c = col_of<NG, VEC>(lane, idx);
      av[idx] = c < C ? a_s[c] : 0.f;
    }
  }
  for (int r0 = wave * U; r0 < R; r0 += nw * U) {
    float v[U][NG * 4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = r0 + u;
      load_row<NG, VEC>(Mx + (size_t)r * ld, r < R, C, lane, v[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = r0 + u;
      if constexpr (COL) {
        const float cr = r < R ? c_s[r] : 0.f;
#pragma unroll
        for (int idx = 0; idx < NG * 4; ++idx) col[idx] = fmaf(v[u][idx], cr, col[idx]);
      }
      if constexpr (DOT) {
        float d = 0.f;
#pragma unroll
        for (int idx = 0; idx < NG * 4; ++idx) {
          float a;
          if constexpr (HOIST) a = av[idx];
          else { const int c = col_of<NG, VEC>(lane, idx); a = c < C ? a_s[c] : 0.f; }
          d = fmaf(v[u][idx], a, d);
        }
        d = wave_sum(d);
        if (lane == 0 && r < R) dot_s[r] = dot_acc ? dot_s[r] + d : d;
      }
    }
  }
}

template <int NG, bool VEC, bool DOT, bool COL>
IADMM_DEV void sweep(const float* __restrict__ Mx, int R, int C, const float* a_s,
                     const float* c_s, float* dot_s, float (&col)[NG * 4], int wave, int nw,
                     int lane) {
  sweep_panel<NG, VEC, DOT, COL>(Mx, R, C, C, a_s, c_s, dot_s, false, col, wave, nw, lane);
}

// Fold the per-wave column accumulators: red_s[c] = ((col_w0 + col_w1) + col_w2) + ...
// Must be reached by every thread of the block.
template <int NG, bool VEC, bool MAX = false>
IADMM_DEV void col_reduce(float (&col)[NG * 4], float* red_s, int C, int wave, int nw, int lane) {
  for (int w = 1; w < nw; ++w) {
    if (wave == w) {
#pragma unroll
      for (int idx = 0; idx < NG * 4; ++idx) {
        const int c = col_of<NG, VEC>(lane, idx);
        if (c < C) red_s[c] = col[idx];
      }
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int idx = 0; idx < NG * 4; ++idx) {
        const int c = col_of<NG, VEC>(lane, idx);
        if (c < C) col[idx] = MAX ? fmaxf(col[idx], red_s[c]) : col[idx] + red_s[c];
      }
    }
    __syncthreads();
  }
  if (wave == 0) {
#pragma unroll
    for (int idx = 0; idx < NG * 4; ++idx) {
      const int c = col_of<NG, VEC>(lane, idx);
      if (c < C) red_s[c] = col[idx];
    }
  }
  __syncthreads();
}

// Column-group count for a given number of columns (template dispatch helper).
inline int ng_for(int64_t C) {
  const int64_t g = (C + 255) / 256;
  if (g <= 1) return 1;
  if (g <= 2) return 2;
  if (g <= 4) return 4;
  if (g <= 8) return 8;
  if (g <= 16) return 16;
  if (g <= 24) return 24;
  return -1;
}

#define IADMM_DISPATCH_NG(ng, vec, ...)                                   \
  do {                                                                    \
    switch (ng) {                                                         \
      case 1: if (vec) { constexpr int NG_ = 1; constexpr bool V_ = true; __VA_ARGS__; } else { constexpr int NG_ = 1; constexpr bool V_ = false; __VA_ARGS__; } break;   \
      case 2: if (vec) { constexpr int NG_ = 2; constexpr bool V_ = true; __VA_ARGS__; } else { constexpr int NG_ = 2; constexpr bool V_ = false; __VA_ARGS__; } break;   \
      case 4: if (vec) { constexpr int NG_ = 4; constexpr bool V_ = true; __VA_ARGS__; } else { constexpr int NG_ = 4; constexpr bool V_ = false; __VA_ARGS__; } break;   \
      case 8: if (vec) { constexpr int NG_ = 8; constexpr bool V_ = true; __VA_ARGS__; } else { constexpr int NG_ = 8; constexpr bool V_ = false; __VA_ARGS__; } break;   \
      case 16: if (vec) { constexpr int NG_ = 16; constexpr bool V_ = true; __VA_ARGS__; } else { constexpr int NG_ = 16; constexpr bool V_ = false; __VA_ARGS__; } break; \
      case 24: if (vec) { constexpr int NG_ = 24; constexpr bool V_ = true; __VA_ARGS__; } else { constexpr int NG_ = 24; constexpr bool V_ = false; __VA_ARGS__; } break; \
      default: return IADMM_E_SIZE;                                       \
    }                                                                     \
  } while (0)

}  // namespace iadmm
