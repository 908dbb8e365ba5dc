// Modified Ruiz equilibration + cost scaling (reference: methods/scaling.py:17-119).
//
// The reference builds dense diagonal matrices and scales with three bmm per round (O(n^3) per
// instance).  Here one workgroup owns one instance and runs all rounds in one launch, O(n^2):
// each round is ONE read+write sweep of Q and A0 that applies the pending cost factor of the
// previous round, the new column/row scalings, and at the same time produces the inf-norms the
// next round needs.  The element arithmetic keeps the reference's rounding order exactly:
//   Q  <- d_i * ((c_prev * Q_ij) * d_j)      (scaling.py:71 then :92 of the previous round)
//   A0 <- e_i * (A0_ij * d_j)                (scaling.py:72)
// and the column norms of c_prev*Q are fl(c_prev * colmax|Q|), which is exact because rounding
// is monotone and c_prev > 0.
#include "sweep.h"

namespace iadmm {

constexpr int kRuizThreads = 256;
constexpr float kMinScaling = 1e-4f;  // scaling.py:12
constexpr float kMaxScaling = 1e4f;   // scaling.py:13

IADMM_DEV float limit_scaling(float v) {  // scaling.py:26-31 (tensor branch)
  float o = fminf(fmaxf(v, kMinScaling), kMaxScaling);
  return o == kMinScaling ? 1.0f : o;
}

IADMM_DEV float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = red[0];
  for (int w = 1; w < nw; ++w) s = fmaxf(s, red[w]);
  __syncthreads();
  return s;
}

struct RuizArgs {
  int n, m, iters;
  const float *Q, *p, *A0, *zl, *zu;
  float *Qo, *po, *A0o, *zlo, *zuo, *D, *E, *c;
};

// Column max |M| over rows (COL) and row max (ROW) of a plain read sweep (round-0 norms).
template <int NG, bool VEC, bool ROW>
IADMM_DEV void norm_sweep(const float* __restrict__ Mx, int R, int C, float (&cm)[NG * 4],
                          float* rowmax_s, int wave, int nw, int lane) {
  for (int r = wave; r < R; r += nw) {
    float v[NG * 4];
    load_row<NG, VEC>(Mx + (size_t)r * C, true, C, lane, v);
    float rm = 0.f;
#pragma unroll
    for (int idx = 0; idx < NG * 4; ++idx) {
      const float av = fabsf(v[idx]);
      cm[idx] = fmaxf(cm[idx], av);
      rm = fmaxf(rm, av);
    }
    if constexpr (ROW) {
      rm = wave_max(rm);
      if (lane == 0) rowmax_s[r] = rm;
    }
  }
}

// Scale-and-write sweep: out = s_r * ((cpre * in) * d_c); tracks column max and row max of out.
template <int NG, bool VEC, bool ROW>
IADMM_DEV void scale_sweep(const float* src, float* dst, int R, int C, const float* rs_s,
                           const float* d_s, float cpre, float (&cm)[NG * 4], float* rowmax_s,
                           int wave, int nw, int lane) {
  constexpr bool HOIST = NG <= 8;
  float dv[HOIST ? NG * 4 : 1];
  if constexpr (HOIST) {
#pragma unroll
    for (int idx = 0; idx < NG * 4; ++idx) {
      const int c = col_of<NG, VEC>(lane, idx);
      dv[idx] = c < C ? d_s[c] : 0.f;
    }
  }
  for (int r = wave; r < R; r += nw) {
    float v[NG * 4];
    const float* srow = src + (size_t)r * C;
    float* drow = dst + (size_t)r * C;
    load_row<NG, VEC>(srow, true, C, lane, v);
    const float sr = rs_s[r];
    float rm = 0.f;
#pragma unroll
    for (int idx = 0; idx < NG * 4; ++idx) {
      float dc;
      if constexpr (HOIST) dc = dv[idx];
      else { const int c = col_of<NG, VEC>(lane, idx); dc = c < C ? d_s[c] : 0.f; }
      const float o = sr * ((cpre * v[idx]) * dc);
      v[idx] = o;
      cm[idx] = fmaxf(cm[idx], fabsf(o));
      rm = fmaxf(rm, fabsf(o));
    }
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < NG; ++i) {
        const int c = 4 * (lane + 64 * i);
        if (c < C) *reinterpret_cast<float4*>(drow + c) = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4 * NG; ++j) {
        const int c = lane + 64 * j;
        if (c < C) drow[c] = v[j];
      }
    }
    if constexpr (ROW) {
      rm = wave_max(rm);
      if (lane == 0) rowmax_s[r] = rm;
    }
  }
}

template <int NG, bool VEC>
__global__ __launch_bounds__(kRuizThreads) void ruiz_kernel(RuizArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n = a.n, m = a.m;
  float* d = sm;          // n  : this round's column scaling
  float* e = d + n;       // m  : this round's row scaling
  float* qcm = e + m;     // n  : column inf-norms of Q (before the pending cost factor)
  float* acm = qcm + n;   // n  : column inf-norms of A0
  float* arm = acm + n;   // m  : row inf-norms of A0
  float* red = arm + m;   // 8  : block reductions
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const size_t b = blockIdx.x;
  const float* Qi = a.Q + b * n * n;
  const float* Ai = a.A0 + b * m * n;
  float* Qb = a.Qo + b * n * n;
  float* Ab = a.A0o + b * m * n;
  float* pb = a.po + b * n;
  float* Db = a.D + b * n;
  float* Eb = a.E + b * m;

  // round-0 norms of the input data
  float cmQ[NG * 4], cmA[NG * 4];
#pragma unroll
  for (int i = 0; i < NG * 4; ++i) { cmQ[i] = 0.f; cmA[i] = 0.f; }
  norm_sweep<NG, VEC, false>(Qi, n, n, cmQ, nullptr, wave, nw, lane);
  if (m > 0) norm_sweep<NG, VEC, true>(Ai, m, n, cmA, arm, wave, nw, lane);
  col_reduce<NG, VEC, true>(cmQ, qcm, n, wave, nw, lane);
  col_reduce<NG, VEC, true>(cmA, acm, n, wave, nw, lane);

  float cpend = 1.0f;  // cost factor of the previous round, not yet applied to the stored Q
  float cacc = 1.0f;   // scaling.py:56 c = 1.0
  for (int it = 0; it < a.iters; ++it) {
    // scaling.py:64-68: KKT column norms -> limit -> 1/sqrt
    for (int j = tid; j < n; j += blockDim.x) {
      const float top = fmaxf(cpend * qcm[j], m > 0 ? acm[j] : 0.f);
      d[j] = 1.0f / sqrtf(limit_scaling(top));
    }
    for (int i = tid; i < m; i += blockDim.x) e[i] = 1.0f / sqrtf(limit_scaling(arm[i]));
    __syncthreads();

    const float* Qs = it == 0 ? Qi : Qb;
    const float* As = it == 0 ? Ai : Ab;
#pragma unroll
    for (int i = 0; i < NG * 4; ++i) { cmQ[i] = 0.f; cmA[i] = 0.f; }
    scale_sweep<NG, VEC, false>(Qs, Qb, n, n, d, d, cpend, cmQ, nullptr, wave, nw, lane);
    if (m > 0) scale_sweep<NG, VEC, true>(As, Ab, m, n, e, d, 1.0f, cmA, arm, wave, nw, lane);

    // vectors (scaling.py:73-79): p = d p, zl/zu = e z, D = d D, E = e E
    float pmax = 0.f;
    for (int j = tid; j < n; j += blockDim.x) {
      const float pv = d[j] * (it == 0 ? a.p[b * n + j] : pb[j]);
      pb[j] = pv;
      pmax = fmaxf(pmax, fabsf(pv));
      Db[j] = it == 0 ? d[j] * 1.0f : d[j] * Db[j];
    }
    for (int i = tid; i < m; i += blockDim.x) {
      const float ei = e[i];
      a.zlo[b * m + i] = ei * (it == 0 ? a.zl[b * m + i] : a.zlo[b * m + i]);
      a.zuo[b * m + i] = ei * (it == 0 ? a.zu[b * m + i] : a.zuo[b * m + i]);
      Eb[i] = it == 0 ? ei * 1.0f : ei * Eb[i];
    }
    col_reduce<NG, VEC, true>(cmQ, qcm, n, wave, nw, lane);
    col_reduce<NG, VEC, true>(cmA, acm, n, wave, nw, lane);

    // cost normalisation (scaling.py:81-96)
    float qs = 0.f;
    for (int j = tid; j < n; j += blockDim.x) qs += qcm[j];
    const float qmean = block_sum(qs, red) / (float)n;
    const float pinf = limit_scaling(block_max(pmax, red));
    const float ck = 1.0f / limit_scaling(fmaxf(pinf, qmean));
    for (int j = tid; j < n; j += blockDim.x) pb[j] = ck * pb[j];
    cacc = ck * cacc;
    cpend = ck;
    __syncthreads();
  }

  // apply the last round's cost factor to Q
  if (a.iters > 0) {
    for (int r = wave; r < n; r += nw) {
      float v[NG * 4];
      float* row = Qb + (size_t)r * n;
      load_row<NG, VEC>(row, true, n, lane, v);
      if constexpr (VEC) {
#pragma unroll
        for (int i = 0; i < NG; ++i) {
          const int c = 4 * (lane + 64 * i);
          if (c < n)
            *reinterpret_cast<float4*>(row + c) = make_float4(cpend * v[4 * i], cpend * v[4 * i + 1],
                                                              cpend * v[4 * i + 2], cpend * v[4 * i + 3]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4 * NG; ++j) {
          const int c = lane + 64 * j;
          if (c < n) row[c] = cpend * v[j];
        }
      }
    }
  } else {  // zero rounds: plain copy (D = E = 1, c = 1)
    for (int64_t k = tid; k < (int64_t)n * n; k += blockDim.x) Qb[k] = Qi[k];
    for (int64_t k = tid; k < (int64_t)m * n; k += blockDim.x) Ab[k] = Ai[k];
    for (int j = tid; j < n; j += blockDim.x) { pb[j] = a.p[b * n + j]; Db[j] = 1.f; }
    for (int i = tid; i < m; i += blockDim.x) {
      a.zlo[b * m + i] = a.zl[b * m + i]; a.zuo[b * m + i] = a.zu[b * m + i]; Eb[i] = 1.f;
    }
  }
  if (tid == 0) a.c[b] = cacc;
}

}  // namespace iadmm

using namespace iadmm;

extern "C" int iadmm_ruiz_scale(int64_t B, int64_t n, int64_t m, int64_t iters, const float* Q,
                                const float* p, const float* A0, const float* zl, const float* zu,
                                float* Q_out, float* p_out, float* A0_out, float* zl_out,
                                float* zu_out, float* D, float* E, float* c, void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || iters < 0) return IADMM_E_ARG;
  if (!Q || !p || !Q_out || !p_out || !D || !c) return IADMM_E_ARG;
  if (m > 0 && (!A0 || !zl || !zu || !A0_out || !zl_out || !zu_out || !E)) return IADMM_E_ARG;
  if (3 * n + 2 * m + 8 > 40960 || B > 0x7fffffff) return IADMM_E_SIZE;
  RuizArgs a{(int)n, (int)m, (int)iters, Q, p, A0, zl, zu, Q_out, p_out, A0_out, zl_out, zu_out, D, E, c};
  const int ng = ng_for(n);
  const bool vec = (n % 4 == 0) && aligned16(Q) && aligned16(Q_out) &&
                   (m == 0 || (aligned16(A0) && aligned16(A0_out)));
  const size_t lds = (3 * n + 2 * m + 8) * sizeof(float);
  IADMM_DISPATCH_NG(ng, vec, {
    IADMM_ALLOW_LDS((ruiz_kernel<NG_, V_>), lds); hipLaunchKernelGGL((ruiz_kernel<NG_, V_>), dim3((unsigned)B), dim3(kRuizThreads), lds,
                       (hipStream_t)stream, a);
  });
  IADMM_CHECK_LAUNCH();
  return 0;
}
