// Stage II: batched dense LU with partial pivoting and the two triangular solves
// (reference: models/lu.py:26-35, torch.lu / torch.lu_solve on K[B,N,N]).
//
// Right-looking blocked LU, panel width kNB = 16, one panel step = two launches:
//   lu_panel_kernel   one workgroup per instance: the (N-k) x 16 panel is factored in LDS
//                     (pivot = first max |a| like LAPACK i?amax; the multipliers use a
//                     reciprocal like ?getf2), the row interchanges are applied to the columns
//                     left and right of the panel (?laswp), and U12 = L11^-1 A12 is solved.
//   lu_update_kernel  B x ceil(rows/64) workgroups: A22 -= L21 U12, each thread owning a 4-column
//                     group with its 16x4 slice of U12 in registers, rows streamed with 16-B
//                     loads (HBM-bound: A22 read and written once per panel).
// lu_solve_kernel: one workgroup per instance; P b, then blocked forward (unit L) and backward
// (U) substitution: 64-row blocks, prefix dot products over coalesced row segments, the 64x64
// diagonal block solved inside one wave.
//
// Pivots are stored 0-based (global row index swapped with row i).  info[b] = first i+1 with a
// zero pivot (0 = non-singular), LAPACK convention.
#include "common.h"

namespace iadmm {

constexpr int kNB = 16;
constexpr int kPS = kNB + 1;       // LDS panel row stride (conflict-free column reads)
constexpr int kLuThreads = 256;
constexpr int kUpdRows = 64;
constexpr int kSolveBlk = 64;

__global__ __launch_bounds__(kLuThreads) void lu_panel_kernel(int N, int k0, float* A, int* piv, int* info) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* P = sm;                             // (N-k0) x kPS
  float* rv = P + (size_t)(N - k0) * kPS;    // reduction scratch: 4 waves x (val, idx)
  int* ri = reinterpret_cast<int*>(rv + 8);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t b = blockIdx.x;
  float* Ab = A + b * (size_t)N * N;
  const int R = N - k0;
  const int nb = min(kNB, R);

  // 16-B loads when the panel is a whole 16-column block of 16-B-aligned rows
  const bool vec = nb == kNB && (N % 4) == 0 && aligned16(Ab);
  if (vec) {
#pragma unroll 4
    for (int q = tid; q < R * 4; q += blockDim.x) {
      const int r = q >> 2, c4 = (q & 3) * 4;
      const float4 v = *reinterpret_cast<const float4*>(Ab + (size_t)(k0 + r) * N + k0 + c4);
      P[r * kPS + c4] = v.x; P[r * kPS + c4 + 1] = v.y; P[r * kPS + c4 + 2] = v.z; P[r * kPS + c4 + 3] = v.w;
    }
  } else {
    for (int idx = tid; idx < R * nb; idx += blockDim.x) {
      const int r = idx / nb, c = idx % nb;
      P[r * kPS + c] = Ab[(size_t)(k0 + r) * N + k0 + c];
    }
  }
  __syncthreads();

  for (int j = 0; j < nb; ++j) {
    // pivot: first index of max |P[r][j]| over r in [j, R)
    float best = -1.f;
    int bi = R;
    for (int r = j + tid; r < R; r += blockDim.x) {
      const float v = fabsf(P[r * kPS + j]);
      if (v > best) { best = v; bi = r; }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if (lane == 0) { rv[wave] = best; ri[wave] = bi; }
    __syncthreads();
    if (tid == 0) {
      float bv = rv[0];
      int bx = ri[0];
      for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
        if (rv[w] > bv || (rv[w] == bv && ri[w] < bx)) { bv = rv[w]; bx = ri[w]; }
      if (bx >= R) bx = j;  // all entries NaN: keep the diagonal
      ri[4] = bx;
      piv[b * N + k0 + j] = k0 + bx;
      if (P[bx * kPS + j] == 0.f && info[b] == 0) info[b] = k0 + j + 1;
    }
    __syncthreads();
    const int p = ri[4];
    if (p != j && tid < nb) {
      const float t = P[j * kPS + tid];
      P[j * kPS + tid] = P[p * kPS + tid];
      P[p * kPS + tid] = t;
    }
    __syncthreads();
    const float pv = P[j * kPS + j];
    if (pv != 0.f) {
      const float rcp = 1.0f / pv;
      for (int r = j + 1 + tid; r < R; r += blockDim.x) {
        const float l = P[r * kPS + j] * rcp;
        P[r * kPS + j] = l;
        for (int c = j + 1; c < nb; ++c) P[r * kPS + c] = P[r * kPS + c] - l * P[j * kPS + c];
      }
    }
    __syncthreads();
  }

  // write the factored panel back
  if (vec) {
#pragma unroll 4
    for (int q = tid; q < R * 4; q += blockDim.x) {
      const int r = q >> 2, c4 = (q & 3) * 4;
      *reinterpret_cast<float4*>(Ab + (size_t)(k0 + r) * N + k0 + c4) =
          make_float4(P[r * kPS + c4], P[r * kPS + c4 + 1], P[r * kPS + c4 + 2], P[r * kPS + c4 + 3]);
    }
  } else {
    for (int idx = tid; idx < R * nb; idx += blockDim.x) {
      const int r = idx / nb, c = idx % nb;
      Ab[(size_t)(k0 + r) * N + k0 + c] = P[r * kPS + c];
    }
  }
  // Row interchanges on the columns outside the panel, in pivot order (?laswp), then
  // U12 = L11^-1 A12 (unit lower forward substitution).  Thread t owns columns t + 256 u: it
  // applies all interchanges to them in order (no barrier between interchanges) with the loads
  // of kSwapCols columns in flight together; the TRSM then solves two columns at a time with
  // their 16 loads issued before the substitution (one memory latency per step instead of one
  // per element: this phase was latency-bound).
  constexpr int kSwapCols = 8;
  int pv[kNB];
#pragma unroll
  for (int j = 0; j < kNB; ++j) pv[j] = j < nb ? piv[b * N + k0 + j] : k0 + j;
  for (int cb = 0; cb < N; cb += kSwapCols * kLuThreads) {
#pragma unroll
    for (int j = 0; j < kNB; ++j) {
      const int rj = k0 + j, p = pv[j];
      if (j >= nb || p == rj) continue;
      float t0[kSwapCols], t1[kSwapCols];
#pragma unroll
      for (int u = 0; u < kSwapCols; ++u) {
        const int c = cb + tid + kLuThreads * u;
        const bool ok = c < N && (c < k0 || c >= k0 + nb);
        t0[u] = ok ? Ab[(size_t)rj * N + c] : 0.f;
        t1[u] = ok ? Ab[(size_t)p * N + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kSwapCols; ++u) {
        const int c = cb + tid + kLuThreads * u;
        if (c < N && (c < k0 || c >= k0 + nb)) {
          Ab[(size_t)rj * N + c] = t1[u];
          Ab[(size_t)p * N + c] = t0[u];
        }
      }
    }
  }
  __syncthreads();  // the TRSM's column owners differ from the interchanges' (c - k0 - nb vs c)
  for (int c = k0 + nb + tid; c < N; c += 2 * kLuThreads) {
    const int c2 = c + kLuThreads;
    const bool ok2 = c2 < N;
    float x[kNB], x2[kNB];
#pragma unroll
    for (int i = 0; i < kNB; ++i) {
      x[i] = i < nb ? Ab[(size_t)(k0 + i) * N + c] : 0.f;
      x2[i] = (i < nb && ok2) ? Ab[(size_t)(k0 + i) * N + c2] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < kNB; ++i) {
      float s = x[i], s2 = x2[i];
      for (int l = 0; l < i; ++l) {
        const float lv = P[i * kPS + l];
        s = s - lv * x[l];
        s2 = s2 - lv * x2[l];
      }
      x[i] = s;
      x2[i] = s2;
    }
#pragma unroll
    for (int i = 0; i < kNB; ++i) {
      if (i < nb) {
        Ab[(size_t)(k0 + i) * N + c] = x[i];
        if (ok2) Ab[(size_t)(k0 + i) * N + c2] = x2[i];
      }
    }
  }
}

// A22 -= L21 U12 for rows [k0+16 + blockIdx.y*64, +64) of instance blockIdx.x.
template <bool VEC>
__global__ __launch_bounds__(256) void lu_update_kernel(int N, int k0, float* A) {
  __shared__ float Ls[kUpdRows][kNB];
  const int nb = kNB;
  const size_t b = blockIdx.x;
  float* Ab = A + b * (size_t)N * N;
  const int c0 = k0 + nb;
  const int r0 = c0 + blockIdx.y * kUpdRows;
  const int rows = min(kUpdRows, N - r0);
  if (rows <= 0) return;
  for (int idx = threadIdx.x; idx < rows * nb; idx += blockDim.x) {
    const int r = idx / nb, l = idx % nb;
    Ls[r][l] = Ab[(size_t)(r0 + r) * N + k0 + l];
  }
  __syncthreads();
  if constexpr (VEC) {
    const int ncg = (N - c0) / 4;  // c0 and N are multiples of 4
    for (int cg = threadIdx.x; cg < ncg; cg += blockDim.x) {
      const int c = c0 + 4 * cg;
      float4 u[kNB];
#pragma unroll
      for (int l = 0; l < kNB; ++l) u[l] = *reinterpret_cast<const float4*>(Ab + (size_t)(k0 + l) * N + c);
      // (HBM-bound on the read + write of A22: software-pipelining the rows or batching four
      // measured no gain, bench_stage2.py; a wider panel is what would halve the traffic)
      for (int r = 0; r < rows; ++r) {
        float4* ap = reinterpret_cast<float4*>(Ab + (size_t)(r0 + r) * N + c);
        float4 a = *ap;
#pragma unroll
        for (int l = 0; l < kNB; ++l) {
          const float lv = Ls[r][l];
          a.x = a.x - lv * u[l].x; a.y = a.y - lv * u[l].y;
          a.z = a.z - lv * u[l].z; a.w = a.w - lv * u[l].w;
        }
        *ap = a;
      }
    }
  } else {
    for (int c = c0 + threadIdx.x; c < N; c += blockDim.x) {
      float u[kNB];
#pragma unroll
      for (int l = 0; l < kNB; ++l) u[l] = Ab[(size_t)(k0 + l) * N + c];
      for (int r = 0; r < rows; ++r) {
        float a = Ab[(size_t)(r0 + r) * N + c];
#pragma unroll
        for (int l = 0; l < kNB; ++l) a = a - Ls[r][l] * u[l];
        Ab[(size_t)(r0 + r) * N + c] = a;
      }
    }
  }
}

// Solve (P^T L U) x = b in place for one instance per workgroup.
constexpr int kDS = kSolveBlk + 1;  // LDS stride of the staged diagonal block
// VEC (N % 4 == 0, 16-B aligned factors): block bounds are multiples of 4, rows 16-B aligned.
template <bool VEC>
__global__ __launch_bounds__(kLuThreads) void lu_solve_kernel(int N, const float* LU, const int* piv,
                                                              float* X) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* x = sm;                  // N
  float* s = x + N;               // kSolveBlk partial sums
  float* D = s + kSolveBlk;       // kSolveBlk x kDS diagonal block
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const size_t b = blockIdx.x;
  const float* M = LU + b * (size_t)N * N;
  float* xb = X + b * N;
  for (int i = tid; i < N; i += blockDim.x) x[i] = xb[i];
  __syncthreads();
  if (tid == 0) {
    for (int i = 0; i < N; ++i) {
      const int p = piv[b * N + i];
      if (p != i) { const float t = x[i]; x[i] = x[p]; x[p] = t; }
    }
  }
  __syncthreads();
  for (int pass = 0; pass < 2; ++pass) {  // 0: forward with unit L, 1: backward with U
    const int nblk = (N + kSolveBlk - 1) / kSolveBlk;
    for (int bb = 0; bb < nblk; ++bb) {
      const int k0 = pass == 0 ? bb * kSolveBlk : max(0, N - (bb + 1) * kSolveBlk);
      const int k1 = pass == 0 ? min(N, k0 + kSolveBlk) : N - bb * kSolveBlk;
      const int nbk = k1 - k0;
      for (int idx = tid; idx < nbk * nbk; idx += blockDim.x) {
        const int r = idx / nbk, c = idx % nbk;
        D[r * kDS + c] = M[(size_t)(k0 + r) * N + k0 + c];
      }
      for (int i = wave; i < nbk; i += nw) {  // prefix (forward) / suffix (backward) dot products
        const float* row = M + (size_t)(k0 + i) * N;
        const int j0 = pass == 0 ? 0 : k1, j1 = pass == 0 ? k0 : N;
        float d = 0.f;
        if constexpr (VEC) {
          // 16-B loads, 4 in flight per lane: a latency-bound scalar stream ran at ~2 TB/s
          const float4* r4 = reinterpret_cast<const float4*>(row);
          const float4* x4 = reinterpret_cast<const float4*>(x);
          const int q1 = j1 >> 2;
          int q = (j0 >> 2) + lane;
          for (; q + 192 < q1; q += 256) {
            const float4 a0 = r4[q], a1 = r4[q + 64], a2 = r4[q + 128], a3 = r4[q + 192];
            const float4 b0 = x4[q], b1 = x4[q + 64], b2 = x4[q + 128], b3 = x4[q + 192];
            d = fmaf(a0.x, b0.x, d); d = fmaf(a0.y, b0.y, d); d = fmaf(a0.z, b0.z, d); d = fmaf(a0.w, b0.w, d);
            d = fmaf(a1.x, b1.x, d); d = fmaf(a1.y, b1.y, d); d = fmaf(a1.z, b1.z, d); d = fmaf(a1.w, b1.w, d);
            d = fmaf(a2.x, b2.x, d); d = fmaf(a2.y, b2.y, d); d = fmaf(a2.z, b2.z, d); d = fmaf(a2.w, b2.w, d);
            d = fmaf(a3.x, b3.x, d); d = fmaf(a3.y, b3.y, d); d = fmaf(a3.z, b3.z, d); d = fmaf(a3.w, b3.w, d);
          }
          for (; q < q1; q += 64) {
            const float4 a0 = r4[q], b0 = x4[q];
            d = fmaf(a0.x, b0.x, d); d = fmaf(a0.y, b0.y, d); d = fmaf(a0.z, b0.z, d); d = fmaf(a0.w, b0.w, d);
          }
        } else {
          for (int j = j0 + lane; j < j1; j += 64) d = fmaf(row[j], x[j], d);
        }
        d = wave_sum(d);
        if (lane == 0) s[i] = d;
      }
      __syncthreads();
      if (wave == 0) {
        float v = lane < nbk ? x[k0 + lane] - s[lane] : 0.f;
        if (pass == 0) {
          for (int j = 0; j < nbk; ++j) {
            const float xj = __shfl(v, j, 64);
            if (lane > j && lane < nbk) v = v - D[lane * kDS + j] * xj;
          }
        } else {
          for (int j = nbk - 1; j >= 0; --j) {
            const float vj = __shfl(v, j, 64) / D[j * kDS + j];
            if (lane == j) v = vj;
            if (lane < j) v = v - D[lane * kDS + j] * vj;
          }
        }
        if (lane < nbk) x[k0 + lane] = v;
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < N; i += blockDim.x) xb[i] = x[i];
}

// b~ = [sigma x - p ; z - y / rho]  (models/lu.py:125,129)
__global__ void kkt_rhs_kernel(int64_t B, int n, int m, int num_ineq, const float* p, const float* x,
                               const float* y, const float* z, float sigma, const float* scal,
                               const float* rho_rows, float* out) {
  const int N = n + m;
  const float irho_in = scal ? scal[IADMM_S_IRHO_IN] : 0.f, irho_eq = scal ? scal[IADMM_S_IRHO_EQ] : 0.f;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < B * N; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = k / N;
    const int i = (int)(k - b * N);
    if (i < n) {
      out[k] = sigma * x[b * n + i] - p[b * n + i];
    } else {
      const int j = i - n;
      const float irho = rho_rows ? 1.0f / rho_rows[b * m + j] : (j < num_ineq ? irho_in : irho_eq);
      out[k] = z[b * m + j] - irho * y[b * m + j];
    }
  }
}

}  // namespace iadmm

using namespace iadmm;

extern "C" int iadmm_lu_factor(int64_t B, int64_t N, float* A, int* piv, int* info, void* stream) {
  if (B <= 0 || N <= 0 || !A || !piv || !info) return IADMM_E_ARG;
  const size_t lds = ((size_t)N * kPS + 16) * sizeof(float);
  if (lds > 160 * 1024 || B > 0x7fffffff) return IADMM_E_SIZE;
  hipStream_t s = (hipStream_t)stream;
  IADMM_ALLOW_LDS(lu_panel_kernel, lds);
  hipError_t e = hipMemsetAsync(info, 0, B * sizeof(int), s);
  if (e != hipSuccess) return (int)e;
  const bool vec = (N % 4 == 0) && aligned16(A);
  for (int k0 = 0; k0 < N; k0 += kNB) {
    hipLaunchKernelGGL(lu_panel_kernel, dim3((unsigned)B), dim3(kLuThreads), lds, s, (int)N, k0, A, piv, info);
    IADMM_CHECK_LAUNCH();
    const int rest = (int)N - k0 - kNB;
    if (rest > 0) {
      const dim3 grid((unsigned)B, (unsigned)((rest + kUpdRows - 1) / kUpdRows));
      if (vec) hipLaunchKernelGGL(lu_update_kernel<true>, grid, dim3(256), 0, s, (int)N, k0, A);
      else hipLaunchKernelGGL(lu_update_kernel<false>, grid, dim3(256), 0, s, (int)N, k0, A);
      IADMM_CHECK_LAUNCH();
    }
  }
  return 0;
}

extern "C" int iadmm_lu_solve(int64_t B, int64_t N, const float* LU, const int* piv, float* x,
                              void* stream) {
  if (B <= 0 || N <= 0 || !LU || !piv || !x) return IADMM_E_ARG;
  const size_t lds = ((size_t)N + kSolveBlk + kSolveBlk * kDS) * sizeof(float);
  if (lds > 64 * 1024 || B > 0x7fffffff) return IADMM_E_SIZE;
  if (N % 4 == 0 && aligned16(LU))
    hipLaunchKernelGGL(lu_solve_kernel<true>, dim3((unsigned)B), dim3(kLuThreads), lds, (hipStream_t)stream,
                       (int)N, LU, piv, x);
  else
    hipLaunchKernelGGL(lu_solve_kernel<false>, dim3((unsigned)B), dim3(kLuThreads), lds, (hipStream_t)stream,
                       (int)N, LU, piv, x);
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_kkt_rhs(int64_t B, int64_t n, int64_t m, int64_t num_ineq, const float* p,
                             const float* x, const float* y, const float* z, float sigma,
                             const float* scal, const float* rho_rows, float* out, void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || !p || !x || !out || (m > 0 && (!y || !z))) return IADMM_E_ARG;
  if (m > 0 && !scal && !rho_rows) return IADMM_E_ARG;
  const int64_t tot = B * (n + m);
  const int64_t blocks = (tot + 255) / 256;
  hipLaunchKernelGGL(kkt_rhs_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                     (hipStream_t)stream, B, (int)n, (int)m, (int)num_ineq, p, x, y, z, sigma, scal,
                     rho_rows, out);
  IADMM_CHECK_LAUNCH();
  return 0;
}
