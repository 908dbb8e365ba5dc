// Implicit-KKT kernels: residual gradient g = K^T (K xv - b~), ||K xv - b~||, and the
// primal/dual/objective metrics.  HBM-bound: each pass streams Q[n,n] and A0[m,n] of one
// instance exactly once with 16-B coalesced loads; K itself is never formed.
//
// Reference: models/lstm.py:67-72 (K, b~, the two dependent bmm), main.py:952 (ls_res),
// utils.py:53-54,68-71 (obj_fn, primal_dual_loss).
#include "sweep.h"

namespace iadmm {

constexpr int kKktThreads = 256;
// Column panel of the KKT sweeps: NG <= 8 float4 groups per lane (<= 2048 columns), so a lane
// holds at most 32 row values + 32 column accumulators whatever n is (NG 16/24 needed 212-256
// VGPRs and ran one wave per SIMD at n = 5000).
constexpr int kPanelNG = 8;

struct KktArgs {
  int n, m, num_ineq;
  const float *Q, *A0, *p, *x, *y, *z, *xv;
  float sigma;
  const float* scal;
  float *g, *btild, *rhovec, *lsres, *rout;
};

// One workgroup = one instance.  LDS: xs[n] (x~ -> r1), vs[m] (v -> r2), t1[n], t3[m], red[n].
// PASS2=false stops after r and writes ||r||_2 (ls_res); PASS2=true computes g.
// Columns are processed in panels of NG*256 (one panel when n <= NG*256); NT threads per
// workgroup is chosen by the launcher so that large instances (whose LDS allows only one or two
// workgroups per CU) still run 4 waves per SIMD.
template <int NG, bool VEC, bool PASS2, int NT>
__global__ __launch_bounds__(NT) void kkt_kernel(KktArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n = a.n, m = a.m, N = n + m;
  float* xs = sm;
  float* vs = xs + n;
  float* t1 = vs + m;
  float* t3 = t1 + n;
  float* red = t3 + m;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const size_t b = blockIdx.x;
  const float* Qb = a.Q + b * n * n;
  const float* Ab = a.A0 + b * m * n;
  const float* xvb = a.xv + b * N;
  for (int i = tid; i < N; i += blockDim.x) {
    if (i < n) xs[i] = xvb[i]; else vs[i - n] = xvb[i];
  }
  __syncthreads();

  const float sigma = a.sigma;
  const float rho_in = a.scal[IADMM_S_RHO_IN], rho_eq = a.scal[IADMM_S_RHO_EQ];
  const float irho_in = a.scal[IADMM_S_IRHO_IN], irho_eq = a.scal[IADMM_S_IRHO_EQ];

  // ---- pass 1: t1 = Q x~, t3 = A0 x~, red = A0^T v  (one read of Q and of A0)
  constexpr int PW = NG * 256;
  float col[NG * 4];
  if constexpr (NG < kPanelNG) {  // n <= PW: one panel, no panel loop (keeps the VGPR count low)
#pragma unroll
    for (int i = 0; i < NG * 4; ++i) col[i] = 0.f;
    sweep<NG, VEC, true, false>(Qb, n, n, xs, nullptr, t1, col, wave, nw, lane);
    if (m > 0) sweep<NG, VEC, true, true>(Ab, m, n, xs, vs, t3, col, wave, nw, lane);
    col_reduce<NG, VEC>(col, red, n, wave, nw, lane);
  } else {
#pragma unroll 1
    for (int c0 = 0; c0 < n; c0 += PW) {
      const int cp = n - c0 < PW ? n - c0 : PW;
#pragma unroll
      for (int i = 0; i < NG * 4; ++i) col[i] = 0.f;
      sweep_panel<NG, VEC, true, false>(Qb + c0, n, cp, n, xs + c0, nullptr, t1, c0 > 0, col, wave, nw, lane);
      if (m > 0) sweep_panel<NG, VEC, true, true>(Ab + c0, m, cp, n, xs + c0, vs, t3, c0 > 0, col, wave, nw, lane);
      col_reduce<NG, VEC>(col, red + c0, cp, wave, nw, lane);
    }
  }

  // ---- r = K xv - b~ (row i < n: (Q+sI) x~ + A0^T v - (s x - p); row n+j: A0 x~ - v/rho - (z - y/rho))
  float ss = 0.f;
  for (int i = tid; i < n; i += blockDim.x) {
    const float b1 = sigma * a.x[b * n + i] - a.p[b * n + i];
    const float r1 = ((t1[i] + sigma * xs[i]) + red[i]) - b1;
    if (a.btild) a.btild[b * N + i] = b1;
    if (a.rout) a.rout[b * N + i] = r1;
    if (PASS2) xs[i] = r1; else ss += r1 * r1;
  }
  for (int j = tid; j < m; j += blockDim.x) {
    const bool ineq = j < a.num_ineq;
    const float rho = ineq ? rho_in : rho_eq, irho = ineq ? irho_in : irho_eq;
    const float b2 = a.z[b * m + j] - irho * a.y[b * m + j];
    const float r2 = (t3[j] + (-irho) * vs[j]) - b2;
    if (a.btild) a.btild[b * N + n + j] = b2;
    if (a.rout) a.rout[b * N + n + j] = r2;
    if (a.rhovec) a.rhovec[b * m + j] = rho;
    if (PASS2) vs[j] = r2; else ss += r2 * r2;
  }
  if constexpr (!PASS2) {
    const float tot = block_sum(ss, red);
    if (tid == 0) a.lsres[b] = sqrtf(tot);
    return;
  } else {
    __syncthreads();
    // ---- pass 2: red = Q^T r1 + A0^T r2 (one column accumulator), t3 = A0 r1
    if constexpr (NG < kPanelNG) {
#pragma unroll
      for (int i = 0; i < NG * 4; ++i) col[i] = 0.f;
      sweep<NG, VEC, false, true>(Qb, n, n, nullptr, xs, nullptr, col, wave, nw, lane);
      if (m > 0) sweep<NG, VEC, true, true>(Ab, m, n, xs, vs, t3, col, wave, nw, lane);
      col_reduce<NG, VEC>(col, red, n, wave, nw, lane);
    } else {
#pragma unroll 1
      for (int c0 = 0; c0 < n; c0 += PW) {
        const int cp = n - c0 < PW ? n - c0 : PW;
#pragma unroll
        for (int i = 0; i < NG * 4; ++i) col[i] = 0.f;
        sweep_panel<NG, VEC, false, true>(Qb + c0, n, cp, n, nullptr, xs, nullptr, false, col, wave, nw, lane);
        if (m > 0) sweep_panel<NG, VEC, true, true>(Ab + c0, m, cp, n, xs + c0, vs, t3, c0 > 0, col, wave, nw, lane);
        col_reduce<NG, VEC>(col, red + c0, cp, wave, nw, lane);
      }
    }
    for (int i = tid; i < n; i += blockDim.x) a.g[b * N + i] = red[i] + sigma * xs[i];
    for (int j = tid; j < m; j += blockDim.x) {
      const float irho = j < a.num_ineq ? irho_in : irho_eq;
      a.g[b * N + n + j] = t3[j] + (-irho) * vs[j];
    }
  }
}

// ---- Row-block split of the residual gradient (any batch size fills the chip).
// The rows of Q and of A0 are cut into fixed blocks of kRB rows (Q blocks 0..nbq-1, then A0
// blocks nbq..nbq+nba-1); a workgroup streams a contiguous range of blocks, so an instance is
// spread over S workgroups (S chosen from B: B*S ~ the chip's 1024 resident workgroup slots).  Row dots are complete
// per row; column sums are formed per block (wave w owns rows w*U + 4U*k of the block; the
// four waves are folded in order) and written as one partial vector per block, and the small
// combine kernels add the partials in block order.  The summation order therefore depends on the
// block structure only, never on S or B: every batch size and shard gives bitwise the same g.
//   kkt_split_p1  dots = [Q x~ ; A0 x~], part[ia] = A0_ia^T v        (one read of Q and A0)
//   kkt_split_c1  r = K xv - b~  (+ b~, rho_vec, r_out)
//   kkt_split_p2  part[blk] = M_blk^T [r1 ; r2]_blk, dots_A0 = A0 r1 (one read of Q and A0)
//   kkt_split_c2  g = [sum part + sigma r1 ; A0 r1 - r2 / rho]
#ifndef IADMM_KKT_RB
#define IADMM_KKT_RB 256
#endif
constexpr int kRB = IADMM_KKT_RB;  // rows per block (variant knob for tools/kktbench.py studies)

struct KktSplitArgs {
  int n, m, num_ineq, S, nbq, nba, dbuf;
  const float *Q, *A0, *p, *x, *y, *z, *xv;
  float sigma;
  const float* scal;
  float *dots, *part, *r;                // workspace: [B][N], [B][nbq+nba][n], [B][N]
  float *g, *btild, *rhovec, *rout;
  // pass-1 input vector [v1 ; v2] (rows of stride ld1 / ld2): xv for the residual gradient, dg
  // for its backward, [x ; y] for the loss
  const float *v1, *v2;
  int ld1, ld2;
  float* aux;                            // workspace [B][nchunk][2]: per-chunk partial sums
  const float *rf, *cp, *cd;             // backward: saved forward residual; loss: coefficients
  float *dxv, *dx, *dy, *dz, *ds_inst, *primal, *dual;
};

// What the two combine kernels compute (the two streaming passes are shared).
enum SplitMode { kResgrad = 0, kKktBwd = 1, kLoss = 2 };

// One block of kRB rows starting at row0 of an [R x n] matrix Mx: wave w sweeps its rows over
// all column panels (DOT: dot_s[r] for the block's rows, accumulated across panels), COL: the
// block's column sums, folded over the 4 waves in order ((w0 + w1) + w2) + w3 into dst[n]
// (global).  The fold is one round: every wave writes its partial panel into fold[wave][.] (LDS),
// one barrier, then each thread sums its columns.  ``fold`` alternates between two buffers
// (*fsel) when two fit, so the next fold's writes never meet this fold's reads without a
// barrier in between; with one buffer a second barrier follows the reads.  c_s / dot_s are
// indexed by the matrix's own row numbers.
template <int NG, bool VEC, bool DOT, bool COL>
IADMM_DEV void split_block(const float* __restrict__ Mx, int R, int n, int row0, const float* a_s,
                           const float* c_s, float* dot_s, float* fold, int fstride, bool dbuf, int* fsel,
                           float* __restrict__ dst, int wave, int lane) {
  constexpr int PW = NG * 256;
  const int rows = min(kRB, R - row0);
  float col[NG * 4];
#pragma unroll 1
  for (int c0 = 0; c0 < n; c0 += PW) {
    const int cp = n - c0 < PW ? n - c0 : PW;
#pragma unroll
    for (int i = 0; i < NG * 4; ++i) col[i] = 0.f;
    // the waves interleave over the block's rows (wave w: rows w*U + 4U*k), so a workgroup reads
    // one contiguous stretch of the matrix at a time (4 separate per-wave streams measured
    // 5.3 TB/s per pass against 6.2 for the interleaved single-workgroup kernel)
    sweep_panel<NG, VEC, DOT, COL>(Mx + (size_t)row0 * n + c0, rows, cp, n, a_s ? a_s + c0 : nullptr,
                                   c_s ? c_s + row0 : nullptr, dot_s ? dot_s + row0 : nullptr, c0 > 0, col, wave, 4,
                                   lane);
    if constexpr (COL) {
      float* f = fold + (dbuf ? *fsel : 0) * 4 * fstride;
#pragma unroll
      for (int idx = 0; idx < NG * 4; ++idx) {
        const int c = col_of<NG, VEC>(lane, idx);
        if (c < cp) f[wave * fstride + c] = col[idx];
      }
      __syncthreads();
      for (int i = threadIdx.x; i < cp; i += blockDim.x) {
        float v = f[i];
        v += f[fstride + i];
        v += f[2 * fstride + i];
        v += f[3 * fstride + i];
        dst[c0 + i] = v;
      }
      if (dbuf) *fsel ^= 1;
      else __syncthreads();
    }
  }
}

// LDS of the split sweeps: two vectors (n + m floats) + the fold buffer(s) (4 x panel width each).
__host__ __device__ inline int split_fstride(int n, int pw) { return n < pw ? n : pw; }

// Variant knobs (tools/kktbench.py studies): minimum workgroups per CU the register allocation
// must allow, and the LDS budget below which the fold is double-buffered.
#ifndef IADMM_KKT_MINWG
#define IADMM_KKT_MINWG 1
#endif
#ifndef IADMM_KKT_WG_TARGET
#define IADMM_KKT_WG_TARGET 1024
#endif
#ifndef IADMM_KKT_DBUF_BYTES
#define IADMM_KKT_DBUF_BYTES (64 * 1024)
#endif

template <int NG, bool VEC>
__global__ __launch_bounds__(256, IADMM_KKT_MINWG) void kkt_split_p1(KktSplitArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n = a.n, m = a.m, N = n + m, nblk = a.nbq + a.nba;
  float* xs = sm;             // x~ [n]
  float* vs = xs + n;         // v  [m]
  float* fold = vs + m;       // [dbuf ? 2 : 1][4][fstride]
  const int fstride = split_fstride(n, NG * 256);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t b = blockIdx.x / a.S;
  const int s = blockIdx.x % a.S;
  const int lo = (int)((int64_t)s * nblk / a.S), hi = (int)((int64_t)(s + 1) * nblk / a.S);
  for (int i = tid; i < N; i += blockDim.x) {
    if (i < n) xs[i] = a.v1[b * a.ld1 + i]; else vs[i - n] = a.v2[b * a.ld2 + (i - n)];
  }
  __syncthreads();
  int fsel = 0;
  float* db = a.dots + b * N;
  for (int blk = lo; blk < hi; ++blk) {
    if (blk < a.nbq) {
      split_block<NG, VEC, true, false>(a.Q + b * n * n, n, n, blk * kRB, xs, nullptr, db, fold, fstride, a.dbuf,
                                        &fsel, nullptr, wave, lane);
    } else {
      const int ia = blk - a.nbq;
      split_block<NG, VEC, true, true>(a.A0 + b * m * n, m, n, ia * kRB, xs, vs, db + n, fold, fstride, a.dbuf,
                                       &fsel, a.part + (b * nblk + ia) * n, wave, lane);
    }
  }
}

// Sum of the per-block partials k in [0, nb) of column i, in block order; the loads are issued
// eight at a time (the adds stay sequential).
IADMM_DEV float sum_partials(const float* __restrict__ pb, int nb, int n, int i) {
  float red = 0.f;
  int k = 0;
  for (; k + 8 <= nb; k += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = pb[(size_t)(k + u) * n + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) red += v[u];
  }
  for (; k < nb; ++k) red += pb[(size_t)k * n + i];
  return red;
}

// Combine kernels: one thread per row of K (grid = B x nchunk chunks of 256 rows).
//   kResgrad  r = K xv - b~ (+ b~, rho_vec, r_out)
//   kKktBwd   dr = K dg (r := dr) and the chunk's share of ds (d s through 1/rho)
//   kLoss     e_d = Qx + p + A0^T y, e_p = A0 x - z (r := [e_d ; e_p]) and the chunk's share of
//             ||e_d||^2, ||e_p||^2
// The chunk partial sums (aux) are block_sum's fixed tree, added in chunk order by kkt_split_c2.
template <int MODE>
__global__ __launch_bounds__(256) void kkt_split_c1(KktSplitArgs a, int nchunk) {
  __shared__ float red_s[4];
  const int n = a.n, m = a.m, N = n + m, nblk = a.nbq + a.nba;
  const size_t b = blockIdx.x / nchunk;
  const int chunk = blockIdx.x % nchunk;
  const int i = chunk * 256 + threadIdx.x;
  if (MODE == kResgrad && i >= N) return;
  const float sigma = a.sigma;
  const float* db = a.dots + b * N;
  float s0 = 0.f, s1 = 0.f;
  if (i < n) {
    const float red = sum_partials(a.part + b * nblk * n, a.nba, n, i);
    if constexpr (MODE == kResgrad) {
      const float xi = a.xv[b * N + i];
      const float b1 = sigma * a.x[b * n + i] - a.p[b * n + i];
      const float r1 = ((db[i] + sigma * xi) + red) - b1;
      a.r[b * N + i] = r1;
      if (a.btild) a.btild[b * N + i] = b1;
      if (a.rout) a.rout[b * N + i] = r1;
    } else if constexpr (MODE == kKktBwd) {
      a.r[b * N + i] = (db[i] + sigma * a.v1[b * a.ld1 + i]) + red;       // dr1
    } else {
      const float e = (db[i] + a.p[b * n + i]) + red;                      // e_d
      a.r[b * N + i] = e;
      s0 = e * e;
    }
  } else if (i < N) {
    const int j = i - n;
    const bool ineq = j < a.num_ineq;
    if constexpr (MODE == kResgrad) {
      const float rho = a.scal[ineq ? IADMM_S_RHO_IN : IADMM_S_RHO_EQ];
      const float irho = a.scal[ineq ? IADMM_S_IRHO_IN : IADMM_S_IRHO_EQ];
      const float b2 = a.z[b * m + j] - irho * a.y[b * m + j];
      const float r2 = (db[i] + (-irho) * a.xv[b * N + i]) - b2;
      a.r[b * N + i] = r2;
      if (a.btild) a.btild[b * N + i] = b2;
      if (a.rout) a.rout[b * N + i] = r2;
      if (a.rhovec) a.rhovec[b * m + j] = rho;
    } else if constexpr (MODE == kKktBwd) {
      // diota = -dg2 r2 + dr2 (y - v) ; ds += kappa * (-diota / rho^2)   (kappa: d rho / d s)
      const float rho = a.scal[ineq ? IADMM_S_RHO_IN : IADMM_S_RHO_EQ];
      const float irho = a.scal[ineq ? IADMM_S_IRHO_IN : IADMM_S_IRHO_EQ];
      const float kappa = ineq ? 1.f : 1e3f;
      const float dg2 = a.v2[b * a.ld2 + j];
      const float dr2 = db[i] + (-irho) * dg2;
      const float diota = -dg2 * a.rf[b * N + i] + dr2 * (a.y[b * m + j] - a.xv[b * N + i]);
      s0 = kappa * (-diota / (rho * rho));
      a.r[b * N + i] = dr2;
    } else {
      const float e = db[i] - a.z[b * m + j];                              // e_p
      a.r[b * N + i] = e;
      s1 = e * e;
    }
  }
  if constexpr (MODE != kResgrad) {
    s0 = block_sum(s0, red_s);
    if constexpr (MODE == kLoss) s1 = block_sum(s1, red_s);
    if (threadIdx.x == 0) {
      a.aux[(b * nchunk + chunk) * 2 + 0] = s0;
      a.aux[(b * nchunk + chunk) * 2 + 1] = s1;
    }
  }
}

template <int NG, bool VEC>
__global__ __launch_bounds__(256, IADMM_KKT_MINWG) void kkt_split_p2(KktSplitArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n = a.n, m = a.m, N = n + m, nblk = a.nbq + a.nba;
  float* r1 = sm;
  float* r2 = r1 + n;
  float* fold = r2 + m;
  const int fstride = split_fstride(n, NG * 256);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t b = blockIdx.x / a.S;
  const int s = blockIdx.x % a.S;
  const int lo = (int)((int64_t)s * nblk / a.S), hi = (int)((int64_t)(s + 1) * nblk / a.S);
  for (int i = tid; i < N; i += blockDim.x) {
    if (i < n) r1[i] = a.r[b * N + i]; else r2[i - n] = a.r[b * N + i];
  }
  __syncthreads();
  int fsel = 0;
  float* db = a.dots + b * N;
  for (int blk = lo; blk < hi; ++blk) {
    float* dst = a.part + (b * nblk + blk) * n;
    if (blk < a.nbq) {
      split_block<NG, VEC, false, true>(a.Q + b * n * n, n, n, blk * kRB, nullptr, r1, nullptr, fold, fstride, a.dbuf,
                                        &fsel, dst, wave, lane);
    } else {
      const int ia = blk - a.nbq;
      split_block<NG, VEC, true, true>(a.A0 + b * m * n, m, n, ia * kRB, r1, r2, db + n, fold, fstride, a.dbuf,
                                       &fsel, dst, wave, lane);
    }
  }
}

//   kResgrad  g = [sum part + sigma r1 ; A0 r1 - r2 / rho]
//   kKktBwd   dxv += K^T dr, dx -= sigma dr1, dz -= dr2, dy += dr2 / rho, ds_inst = sum of chunks
//   kLoss     dx = cd Q^T e_d/|e_d| + cp A0^T e_p/|e_p|, dy = cd A0 e_d/|e_d|, dz = -cp e_p/|e_p|,
//             primal = |e_p|, dual = |e_d|  (e/|e| := 0 when |e| = 0, like torch's norm backward)
template <int MODE>
__global__ __launch_bounds__(256) void kkt_split_c2(KktSplitArgs a, int nchunk) {
  const int n = a.n, m = a.m, N = n + m, nblk = a.nbq + a.nba;
  const size_t b = blockIdx.x / nchunk;
  const int chunk = blockIdx.x % nchunk;
  const int i = chunk * 256 + threadIdx.x;
  const float* pb = a.part + b * nblk * n;
  const float* rb = a.r + b * N;
  if constexpr (MODE == kResgrad) {
    if (i >= N) return;
    if (i < n) {
      a.g[b * N + i] = sum_partials(pb, nblk, n, i) + a.sigma * rb[i];
    } else {
      const float irho = a.scal[(i - n) < a.num_ineq ? IADMM_S_IRHO_IN : IADMM_S_IRHO_EQ];
      a.g[b * N + i] = a.dots[b * N + i] + (-irho) * rb[i];
    }
  } else if constexpr (MODE == kKktBwd) {
    if (chunk == 0 && threadIdx.x == 0) {
      float ds = 0.f;
      for (int c = 0; c < nchunk; ++c) ds += a.aux[(b * nchunk + c) * 2];
      a.ds_inst[b] = ds;
    }
    if (i >= N) return;
    if (i < n) {
      const float dr1 = rb[i];
      a.dxv[b * N + i] += sum_partials(pb, nblk, n, i) + a.sigma * dr1;
      a.dx[b * n + i] += -a.sigma * dr1;
    } else {
      const int j = i - n;
      const float irho = a.scal[j < a.num_ineq ? IADMM_S_IRHO_IN : IADMM_S_IRHO_EQ];
      const float dr2 = rb[i];
      a.dxv[b * N + i] += a.dots[b * N + i] + (-irho) * dr2;
      a.dz[b * m + j] += -dr2;
      a.dy[b * m + j] += irho * dr2;
    }
  } else {
    float dd = 0.f, pp = 0.f;
    for (int c = 0; c < nchunk; ++c) {
      dd += a.aux[(b * nchunk + c) * 2 + 0];
      pp += a.aux[(b * nchunk + c) * 2 + 1];
    }
    const float nd = sqrtf(dd), np = sqrtf(pp);
    if (chunk == 0 && threadIdx.x == 0) {
      if (a.primal) a.primal[b] = np;
      if (a.dual) a.dual[b] = nd;
    }
    if (i >= N) return;
    const float cp = a.cp ? a.cp[b] : 0.f, cd = a.cd ? a.cd[b] : 0.f;
    const float sd = nd > 0.f ? cd / nd : 0.f, sp = np > 0.f ? cp / np : 0.f;
    if (i < n) {
      if (a.dx) a.dx[b * n + i] = sd * sum_partials(pb, a.nbq, n, i) + sp * sum_partials(pb + (size_t)a.nbq * n, a.nba, n, i);
    } else {
      const int j = i - n;
      if (a.dy) a.dy[b * m + j] = sd * a.dots[b * N + i];
      if (a.dz) a.dz[b * m + j] = -sp * rb[i];
    }
  }
}

struct MetricArgs {
  int n, m;
  const float *Q, *p, *A0, *x, *y, *z;
  float *obj, *primal, *dual;
};

// obj = 0.5 x^T(Qx) + p^T x ; primal = ||A0 x - z|| ; dual = ||(Qx + p) + A0^T y||
template <int NG, bool VEC>
__global__ __launch_bounds__(kKktThreads) void metrics_kernel(MetricArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n = a.n, m = a.m;
  float* xs = sm;
  float* ys = xs + n;
  float* t1 = ys + m;
  float* t3 = t1 + n;
  float* red = t3 + m;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const size_t b = blockIdx.x;
  for (int i = tid; i < n; i += blockDim.x) xs[i] = a.x[b * n + i];
  for (int j = tid; j < m; j += blockDim.x) ys[j] = a.y[b * m + j];
  __syncthreads();
  float col[NG * 4];
#pragma unroll
  for (int i = 0; i < NG * 4; ++i) col[i] = 0.f;
  sweep<NG, VEC, true, false>(a.Q + b * n * n, n, n, xs, nullptr, t1, col, wave, nw, lane);
  if (m > 0) sweep<NG, VEC, true, true>(a.A0 + b * m * n, m, n, xs, ys, t3, col, wave, nw, lane);
  col_reduce<NG, VEC>(col, red, n, wave, nw, lane);
  float xqx = 0.f, px = 0.f, dd = 0.f, pp = 0.f;
  for (int i = tid; i < n; i += blockDim.x) {
    const float pi = a.p[b * n + i];
    xqx = fmaf(xs[i], t1[i], xqx);
    px = fmaf(pi, xs[i], px);
    const float d = (t1[i] + pi) + red[i];
    dd = fmaf(d, d, dd);
  }
  for (int j = tid; j < m; j += blockDim.x) {
    const float r = t3[j] - a.z[b * m + j];
    pp = fmaf(r, r, pp);
  }
  // every block_sum is reached by all threads
  const float s_xqx = block_sum(xqx, red);
  const float s_px = block_sum(px, red);
  const float s_dd = block_sum(dd, red);
  const float s_pp = block_sum(pp, red);
  if (tid == 0) {
    if (a.obj) a.obj[b] = 0.5f * s_xqx + s_px;
    if (a.primal) a.primal[b] = sqrtf(s_pp);
    if (a.dual) a.dual[b] = sqrtf(s_dd);
  }
}

__global__ void unscale_kernel(int64_t B, int n, int m, const float* D, const float* E,
                               const float* c, const float* x, const float* y, const float* z,
                               float* xo, float* yo, float* zo) {
  const int64_t tot = B * (int64_t)(n + m);
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < tot;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = k / (n + m);
    const int i = (int)(k - b * (n + m));
    if (i < n) {
      xo[b * n + i] = D[b * n + i] * x[b * n + i];
    } else {
      const int j = i - n;
      const float e = E[b * m + j];
      const float cinv = 1.0f / c[b];
      yo[b * m + j] = (cinv * e) * y[b * m + j];   // bmm(cinv * E, y), main.py:1026
      zo[b * m + j] = (1.0f / e) * z[b * m + j];   // bmm(Einv, z),      main.py:1027
    }
  }
}

// Batched matvec with a metric epilogue (utils.py:56-63 ineq_dist / eq_dist): one block per
// instance, DOT sweep over rows.  mode 0: Mx x; 1: max(Mx x - rhs, 0); 2: |rhs - Mx x|.
template <int NG, bool VEC>
__global__ __launch_bounds__(kKktThreads) void bmv_kernel(int R, int C, const float* Mx,
                                                           const float* x, const float* rhs,
                                                           int mode, float* out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* xs = sm;       // C
  float* ds = xs + C;   // R
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const size_t b = blockIdx.x;
  for (int i = tid; i < C; i += blockDim.x) xs[i] = x[b * C + i];
  __syncthreads();
  float col[NG * 4];
  sweep<NG, VEC, true, false>(Mx + b * R * C, R, C, xs, nullptr, ds, col, wave, nw, lane);
  __syncthreads();
  for (int r = tid; r < R; r += blockDim.x) {
    const float v = ds[r];
    float o = v;
    if (mode == 1) o = fmaxf(v - rhs[b * R + r], 0.f);
    else if (mode == 2) o = fabsf(rhs[b * R + r] - v);
    out[b * R + r] = o;
  }
}

// Implicit K v (TRANS=false) or K^T v (TRANS=true): only the Q block differs.
//   top = (Q or Q^T) v1 + sigma v1 + A0^T v2 ;  bottom = A0 v1 - v2 / rho
template <int NG, bool VEC, bool TRANS>
__global__ __launch_bounds__(kKktThreads) void kkt_matvec_kernel(KktArgs a, const float* rho_rows, float* out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n = a.n, m = a.m, N = n + m;
  float* xs = sm;
  float* vs = xs + n;
  float* t1 = vs + m;
  float* t3 = t1 + n;
  float* red = t3 + m;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const size_t b = blockIdx.x;
  for (int i = tid; i < N; i += blockDim.x) {
    if (i < n) xs[i] = a.xv[b * N + i]; else vs[i - n] = a.xv[b * N + i];
  }
  __syncthreads();
  float col[NG * 4];
#pragma unroll
  for (int i = 0; i < NG * 4; ++i) col[i] = 0.f;
  if constexpr (TRANS) sweep<NG, VEC, false, true>(a.Q + b * n * n, n, n, nullptr, xs, nullptr, col, wave, nw, lane);
  else sweep<NG, VEC, true, false>(a.Q + b * n * n, n, n, xs, nullptr, t1, col, wave, nw, lane);
  if (m > 0) sweep<NG, VEC, true, true>(a.A0 + b * m * n, m, n, xs, vs, t3, col, wave, nw, lane);
  col_reduce<NG, VEC>(col, red, n, wave, nw, lane);
  const float irho_in = a.scal ? a.scal[IADMM_S_IRHO_IN] : 0.f;
  const float irho_eq = a.scal ? a.scal[IADMM_S_IRHO_EQ] : 0.f;
  for (int i = tid; i < n; i += blockDim.x) {
    // TRANS: red already holds Q^T v1 + A0^T v2 (one column accumulator)
    out[b * N + i] = TRANS ? red[i] + a.sigma * xs[i] : (t1[i] + a.sigma * xs[i]) + red[i];
  }
  for (int j = tid; j < m; j += blockDim.x) {
    const float irho = rho_rows ? 1.0f / rho_rows[b * m + j] : (j < a.num_ineq ? irho_in : irho_eq);
    out[b * N + n + j] = t3[j] + (-irho) * vs[j];
  }
}

// Dense K (models/lstm.py:67-68, models/lu.py:28-29) for Stage II and explicit inspection.
// One 64 x 64 tile of K per workgroup (blockIdx.x = instance, blockIdx.y = tile): rows of K are
// written as coalesced 256-B segments; the A0^T block is staged through LDS so that A0 is also read
// along its rows (a direct per-element formula read it with stride n and ran at 1.3 TB/s).
constexpr int kAsmT = 64;
__global__ __launch_bounds__(256) void kkt_assemble_kernel(int n, int m, int num_ineq, int ntile, const float* Q,
                                                           const float* A0, float sigma, const float* scal,
                                                           const float* rho_rows, float* K) {
  __shared__ float T[kAsmT][kAsmT + 1];
  const int N = n + m;
  const size_t b = blockIdx.x;
  const int i0 = (blockIdx.y / ntile) * kAsmT, j0 = (blockIdx.y % ntile) * kAsmT;
  const int tid = threadIdx.x;
  const float* Qb = Q + b * (size_t)n * n;
  const float* Ab = A0 + b * (size_t)m * n;
  float* Kb = K + b * (size_t)N * N;
  const float irho_in = scal ? scal[IADMM_S_IRHO_IN] : 0.f, irho_eq = scal ? scal[IADMM_S_IRHO_EQ] : 0.f;
  if (i0 < n && j0 + kAsmT > n) {  // the tile meets the A0^T block: T[jj][ii] = A0[j - n][i]
    for (int idx = tid; idx < kAsmT * kAsmT; idx += blockDim.x) {
      const int jj = idx / kAsmT, ii = idx % kAsmT, i = i0 + ii, j = j0 + jj;
      if (i < n && j >= n && j < N) T[jj][ii] = Ab[(size_t)(j - n) * n + i];
    }
    __syncthreads();
  }
  for (int idx = tid; idx < kAsmT * kAsmT; idx += blockDim.x) {
    const int ii = idx / kAsmT, jj = idx % kAsmT, i = i0 + ii, j = j0 + jj;
    if (i >= N || j >= N) continue;
    float v;
    if (i < n && j < n) v = Qb[(size_t)i * n + j] + (i == j ? sigma : 0.f);
    else if (i < n) v = T[jj][ii];
    else if (j < n) v = Ab[(size_t)(i - n) * n + j];
    else if (i != j) v = -0.f;
    else if (rho_rows) v = -(1.0f / rho_rows[b * m + (i - n)]);
    else v = -((i - n) < num_ineq ? irho_in : irho_eq);
    Kb[(size_t)i * N + j] = v;
  }
}

// Row-band form (n % 4 == 0, m % 4 == 0, 16-B aligned Q, A0, K): a workgroup writes 32 whole rows
// of K with 16-B stores.  Top rows i < n: [Q_i + sigma e_i | column i of A0], the A0^T part staged
// through LDS 256 constraint rows at a time (A0[j][i0 .. i0+32) read as 128-B row pieces, written
// back as 1-KiB runs of K's row); bottom rows: [A0_{i-n} | -1/rho on the diagonal, 0 elsewhere].
constexpr int kAsmRows = 32;
constexpr int kAsmJ = 256;
__global__ __launch_bounds__(256) void kkt_assemble_rows_kernel(int n, int m, int num_ineq, const float* Q,
                                                                const float* A0, float sigma, const float* scal,
                                                                const float* rho_rows, float* K) {
  __shared__ float T[kAsmJ][kAsmRows + 1];
  const int N = n + m;
  const size_t b = blockIdx.x;
  const int i0 = blockIdx.y * kAsmRows;
  const int tid = threadIdx.x;
  const float* Qb = Q + b * (size_t)n * n;
  const float* Ab = A0 + b * (size_t)m * n;
  float* Kb = K + b * (size_t)N * N;
  const int nr = min(kAsmRows, N - i0);
  const float irho_in = scal ? scal[IADMM_S_IRHO_IN] : 0.f, irho_eq = scal ? scal[IADMM_S_IRHO_EQ] : 0.f;
  // left block columns [0, n): Q rows (+ sigma on the diagonal) or A0 rows
  const int q4 = n >> 2;
  for (int idx = tid; idx < nr * q4; idx += blockDim.x) {
    const int r = idx / q4, c = (idx - r * q4) * 4, i = i0 + r;
    float4 v;
    if (i < n) {
      v = *reinterpret_cast<const float4*>(Qb + (size_t)i * n + c);
      if (i >= c && i < c + 4) {
        if (i == c) v.x += sigma; else if (i == c + 1) v.y += sigma; else if (i == c + 2) v.z += sigma; else v.w += sigma;
      }
    } else {
      v = *reinterpret_cast<const float4*>(Ab + (size_t)(i - n) * n + c);
    }
    *reinterpret_cast<float4*>(Kb + (size_t)i * N + c) = v;
  }
  if (m == 0) return;
  const int m4 = m >> 2;
  if (i0 >= n) {  // bottom rows: -1/rho on the diagonal of the right block
    for (int idx = tid; idx < nr * m4; idx += blockDim.x) {
      const int r = idx / m4, c = (idx - r * m4) * 4, i = i0 + r, d = i - n;
      float4 v = make_float4(-0.f, -0.f, -0.f, -0.f);
      if (d >= c && d < c + 4) {
        const float val = rho_rows ? -(1.0f / rho_rows[b * m + d]) : -(d < num_ineq ? irho_in : irho_eq);
        if (d == c) v.x = val; else if (d == c + 1) v.y = val; else if (d == c + 2) v.z = val; else v.w = val;
      }
      *reinterpret_cast<float4*>(Kb + (size_t)i * N + n + c) = v;
    }
    return;
  }
  // top rows (i0 + nr <= n since n % 32 is not assumed: rows past n in this band take the bottom
  // form below): the A0^T block through LDS
  const int ntop = min(nr, n - i0);
  for (int j0 = 0; j0 < m; j0 += kAsmJ) {
    const int nj = min(kAsmJ, m - j0);
    __syncthreads();
    for (int idx = tid; idx < nj * (kAsmRows / 4); idx += blockDim.x) {
      const int jj = idx >> 3, c = (idx & 7) * 4;
      if (c < ntop) {
        const float* src = Ab + (size_t)(j0 + jj) * n + i0 + c;
        const float4 v = *reinterpret_cast<const float4*>(src);  // n % 4 == 0, i0 + c % 4 == 0
        T[jj][c] = v.x; T[jj][c + 1] = v.y; T[jj][c + 2] = v.z; T[jj][c + 3] = v.w;
      }
    }
    __syncthreads();
    const int nj4 = nj >> 2;
    for (int idx = tid; idx < ntop * nj4; idx += blockDim.x) {
      const int r = idx / nj4, q = (idx - r * nj4) * 4;
      *reinterpret_cast<float4*>(Kb + (size_t)(i0 + r) * N + n + j0 + q) =
          make_float4(T[q][r], T[q + 1][r], T[q + 2][r], T[q + 3][r]);
    }
  }
  // rows of this band at or past n (when n % 32 != 0): the bottom form
  for (int idx = tid; idx < (nr - ntop) * m4; idx += blockDim.x) {
    const int r = ntop + idx / m4, c = (idx % m4) * 4, i = i0 + r, d = i - n;
    float4 v = make_float4(-0.f, -0.f, -0.f, -0.f);
    if (d >= c && d < c + 4) {
      const float val = rho_rows ? -(1.0f / rho_rows[b * m + d]) : -(d < num_ineq ? irho_in : irho_eq);
      if (d == c) v.x = val; else if (d == c + 1) v.y = val; else if (d == c + 2) v.z = val; else v.w = val;
    }
    *reinterpret_cast<float4*>(Kb + (size_t)i * N + n + c) = v;
  }
}

inline bool kkt_fits(int64_t n, int64_t m) { return 3 * n + 2 * m <= 40960; }

template <int NG, bool VEC, bool PASS2, int NT>
int launch_kkt_nt(int64_t B, size_t lds, KktArgs a, hipStream_t s) {
  IADMM_ALLOW_LDS((kkt_kernel<NG, VEC, PASS2, NT>), lds);
  hipLaunchKernelGGL((kkt_kernel<NG, VEC, PASS2, NT>), dim3((unsigned)B), dim3(NT), lds, s, a);
  IADMM_CHECK_LAUNCH();
  return 0;
}

template <bool PASS2>
int launch_kkt(int64_t B, int64_t n, int64_t m, KktArgs a, hipStream_t s) {
  const int ng = ng_for(n < kPanelNG * 256 ? n : kPanelNG * 256);
  const bool vec = (n % 4 == 0) && aligned16(a.Q) && (m == 0 || aligned16(a.A0));
  const size_t lds = (3 * n + 2 * m) * sizeof(float);
  // Workgroups per CU allowed by LDS (160 KiB): >= 4 -> 256 threads, else 512 (8 waves: at
  // n = m = 5000, one 100 KB workgroup per CU, 512 threads measured 6.18 TB/s against 5.98 with
  // 1024 (VGPR-capped, spills) and 5.55 with 256; tools/kktbench.py).
  const size_t per_cu = (160 * 1024) / (lds > 0 ? lds : 1);
  if (ng == 1) return vec ? launch_kkt_nt<1, true, PASS2, 256>(B, lds, a, s) : launch_kkt_nt<1, false, PASS2, 256>(B, lds, a, s);
  if (ng == 2) return vec ? launch_kkt_nt<2, true, PASS2, 256>(B, lds, a, s) : launch_kkt_nt<2, false, PASS2, 256>(B, lds, a, s);
  if (ng == 4) return vec ? launch_kkt_nt<4, true, PASS2, 256>(B, lds, a, s) : launch_kkt_nt<4, false, PASS2, 256>(B, lds, a, s);
  if (per_cu >= 4) {
    if (vec) return launch_kkt_nt<kPanelNG, true, PASS2, 256>(B, lds, a, s);
    return launch_kkt_nt<kPanelNG, false, PASS2, 256>(B, lds, a, s);
  }
  if (vec) return launch_kkt_nt<kPanelNG, true, PASS2, 512>(B, lds, a, s);
  return launch_kkt_nt<kPanelNG, false, PASS2, 512>(B, lds, a, s);
}

}  // namespace iadmm

using namespace iadmm;

template <int NG, bool VEC>
static int launch_split(dim3 grid, size_t lds, const KktSplitArgs& a, hipStream_t s, int pass) {
  if (pass == 1) {
    IADMM_ALLOW_LDS((kkt_split_p1<NG, VEC>), lds);
    hipLaunchKernelGGL((kkt_split_p1<NG, VEC>), grid, dim3(256), lds, s, a);
  } else {
    IADMM_ALLOW_LDS((kkt_split_p2<NG, VEC>), lds);
    hipLaunchKernelGGL((kkt_split_p2<NG, VEC>), grid, dim3(256), lds, s, a);
  }
  IADMM_CHECK_LAUNCH();
  return 0;
}

static int64_t kkt_split_blocks(int64_t n, int64_t m) { return (n + kRB - 1) / kRB + (m + kRB - 1) / kRB; }
static int64_t kkt_split_chunks(int64_t n, int64_t m) { return (n + m + 255) / 256; }

extern "C" int64_t iadmm_kkt_resgrad_ws_bytes(int64_t B, int64_t n, int64_t m) {
  if (B <= 0 || n <= 0 || m < 0) return 0;
  return B * (2 * (n + m) + kkt_split_blocks(n, m) * n + 2 * kkt_split_chunks(n, m)) * (int64_t)sizeof(float);
}

template <int MODE>
static int launch_combine(int pass, int64_t B, int nchunk, const KktSplitArgs& a, hipStream_t s) {
  if (pass == 1) hipLaunchKernelGGL((kkt_split_c1<MODE>), dim3((unsigned)(B * nchunk)), dim3(256), 0, s, a, nchunk);
  else hipLaunchKernelGGL((kkt_split_c2<MODE>), dim3((unsigned)(B * nchunk)), dim3(256), 0, s, a, nchunk);
  IADMM_CHECK_LAUNCH();
  return 0;
}

// LDS of the split sweeps: the two vectors (n + m floats) + one or two fold buffers of 4 panel
// rows each (two while the total stays within IADMM_KKT_DBUF_BYTES, so that at least two
// workgroups share a CU; one otherwise); panel width = min(n, 256 NG).
static int64_t split_lds_bytes(int64_t n, int64_t m, bool* dbuf_out) {
  const int ng = ng_for(n < kPanelNG * 256 ? n : kPanelNG * 256);
  const int64_t fstride = split_fstride((int)n, ng * 256);
  const bool dbuf = (n + m + 8 * fstride) * 4 <= IADMM_KKT_DBUF_BYTES;
  if (dbuf_out) *dbuf_out = dbuf;
  return (n + m + (dbuf ? 8 : 4) * fstride) * (int64_t)sizeof(float);
}

extern "C" int64_t iadmm_kkt_resgrad_lds_bytes(int64_t n, int64_t m) {
  if (n <= 0 || m < 0 || n > 0x7fffffff || m > 0x7fffffff) return 0;
  return split_lds_bytes(n, m, nullptr);
}

// The row-block split pipeline p1 -> c1 -> [p2] -> c2 for one of the three modes.  ``a`` carries
// the mode's inputs/outputs; the geometry, workspace carving and pass-1 vector are filled here.
static int run_split(int mode, int64_t B, int64_t n, int64_t m, KktSplitArgs a, void* ws, int64_t ws_bytes,
                     bool pass2, hipStream_t s) {
  if (!ws || ws_bytes < iadmm_kkt_resgrad_ws_bytes(B, n, m) || !aligned16(ws)) return IADMM_E_ARG;
  const int64_t nbq = (n + kRB - 1) / kRB, nba = (m + kRB - 1) / kRB, nblk = nbq + nba;
  const int ng = ng_for(n < kPanelNG * 256 ? n : kPanelNG * 256);
  bool dbuf = false;
  const int64_t lds = split_lds_bytes(n, m, &dbuf);
  if (lds > 160 * 1024 || B > 0x7fffffff) return IADMM_E_SIZE;
  // workgroups per instance: the batch's workgroups fill the chip's resident slots (4 per CU x
  // 256 CUs) in ONE round -- a second, partial round of long streaming workgroups idles most of
  // the chip at its end -- and at most one workgroup per block
  int64_t S = IADMM_KKT_WG_TARGET / B;
  S = S < 1 ? 1 : (S > nblk ? nblk : S);
  const int64_t nchunk = kkt_split_chunks(n, m);
  if (B * S > 0x7fffffff || B * nchunk > 0x7fffffff) return IADMM_E_SIZE;
  float* w = static_cast<float*>(ws);
  a.n = (int)n; a.m = (int)m; a.S = (int)S; a.nbq = (int)nbq; a.nba = (int)nba; a.dbuf = dbuf ? 1 : 0;
  a.dots = w;
  a.part = w + B * (n + m);
  a.r = a.part + B * nblk * n;
  a.aux = a.r + B * (n + m);
  const bool vec = (n % 4 == 0) && aligned16(a.Q) && (m == 0 || aligned16(a.A0));
  const dim3 grid((unsigned)(B * S));
  auto stream_pass = [&](int pass) {
    if (ng == 1) return vec ? launch_split<1, true>(grid, lds, a, s, pass) : launch_split<1, false>(grid, lds, a, s, pass);
    if (ng == 2) return vec ? launch_split<2, true>(grid, lds, a, s, pass) : launch_split<2, false>(grid, lds, a, s, pass);
    if (ng == 4) return vec ? launch_split<4, true>(grid, lds, a, s, pass) : launch_split<4, false>(grid, lds, a, s, pass);
    return vec ? launch_split<kPanelNG, true>(grid, lds, a, s, pass) : launch_split<kPanelNG, false>(grid, lds, a, s, pass);
  };
  auto combine = [&](int pass) {
    if (mode == kResgrad) return launch_combine<kResgrad>(pass, B, (int)nchunk, a, s);
    if (mode == kKktBwd) return launch_combine<kKktBwd>(pass, B, (int)nchunk, a, s);
    return launch_combine<kLoss>(pass, B, (int)nchunk, a, s);
  };
  int rc = stream_pass(1);
  if (!rc) rc = combine(1);
  if (!rc && pass2) rc = stream_pass(2);
  if (!rc) rc = combine(2);
  return rc;
}

extern "C" int iadmm_kkt_resgrad(int64_t B, int64_t n, int64_t m, int64_t num_ineq,
                                 const float* Q, const float* A0, const float* p, const float* x,
                                 const float* y, const float* z, const float* xv, float sigma,
                                 const float* scal, float* g, float* btild, float* rho_vec,
                                 float* r_out, void* ws, int64_t ws_bytes, void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || num_ineq < 0 || num_ineq > m) return IADMM_E_ARG;
  if (!Q || !p || !x || !xv || !scal || !g || (m > 0 && (!A0 || !y || !z))) return IADMM_E_ARG;
  KktSplitArgs a{};
  a.num_ineq = (int)num_ineq;
  a.Q = Q; a.A0 = A0; a.p = p; a.x = x; a.y = y; a.z = z; a.xv = xv;
  a.sigma = sigma; a.scal = scal;
  a.g = g; a.btild = btild; a.rhovec = rho_vec; a.rout = r_out;
  a.v1 = xv; a.v2 = xv + n; a.ld1 = a.ld2 = (int)(n + m);
  return run_split(kResgrad, B, n, m, a, ws, ws_bytes, true, (hipStream_t)stream);
}

extern "C" int iadmm_kkt_bwd_split(int64_t B, int64_t n, int64_t m, int64_t num_ineq, const float* Q,
                                   const float* A0, const float* xv, const float* y, const float* r,
                                   const float* dg, float sigma, const float* scal, float* dxv, float* dx,
                                   float* dy, float* dz, float* ds_inst, void* ws, int64_t ws_bytes,
                                   void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || num_ineq < 0 || num_ineq > m) return IADMM_E_ARG;
  if (!Q || !xv || !r || !dg || !scal || !dxv || !dx || !ds_inst || (m > 0 && (!A0 || !y || !dy || !dz)))
    return IADMM_E_ARG;
  KktSplitArgs a{};
  a.num_ineq = (int)num_ineq;
  a.Q = Q; a.A0 = A0; a.y = y; a.xv = xv;
  a.sigma = sigma; a.scal = scal;
  a.v1 = dg; a.v2 = dg + n; a.ld1 = a.ld2 = (int)(n + m);
  a.rf = r;
  a.dxv = dxv; a.dx = dx; a.dy = dy; a.dz = dz; a.ds_inst = ds_inst;
  return run_split(kKktBwd, B, n, m, a, ws, ws_bytes, true, (hipStream_t)stream);
}

extern "C" int iadmm_loss_grad_split(int64_t B, int64_t n, int64_t m, const float* Q, const float* p,
                                     const float* A0, const float* x, const float* y, const float* z,
                                     const float* cp, const float* cd, float* primal, float* dual, float* dx,
                                     float* dy, float* dz, void* ws, int64_t ws_bytes, void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || !Q || !p || !x || (m > 0 && (!A0 || !y || !z))) return IADMM_E_ARG;
  KktSplitArgs a{};
  a.Q = Q; a.A0 = A0; a.p = p; a.z = z;
  a.v1 = x; a.v2 = y; a.ld1 = (int)n; a.ld2 = (int)m;
  a.cp = cp; a.cd = cd;
  a.primal = primal; a.dual = dual; a.dx = dx; a.dy = dy; a.dz = dz;
  // the second sweep only feeds the gradient; the norms come out of the first
  return run_split(kLoss, B, n, m, a, ws, ws_bytes, dx || dy || dz, (hipStream_t)stream);
}

extern "C" int iadmm_kkt_lsres(int64_t B, int64_t n, int64_t m, int64_t num_ineq,
                               const float* Q, const float* A0, const float* p, const float* x,
                               const float* y, const float* z, const float* xv, float sigma,
                               const float* scal, float* out, void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || num_ineq < 0 || num_ineq > m) return IADMM_E_ARG;
  if (!Q || !p || !x || !xv || !scal || !out || (m > 0 && (!A0 || !y || !z))) return IADMM_E_ARG;
  if (!kkt_fits(n, m) || B > 0x7fffffff) return IADMM_E_SIZE;
  KktArgs a{(int)n, (int)m, (int)num_ineq, Q, A0, p, x, y, z, xv, sigma, scal, nullptr, nullptr, nullptr, out, nullptr};
  return launch_kkt<false>(B, n, m, a, (hipStream_t)stream);
}

extern "C" int iadmm_metrics(int64_t B, int64_t n, int64_t m, const float* Q, const float* p,
                             const float* A0, const float* x, const float* y, const float* z,
                             float* obj, float* primal, float* dual, void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || !Q || !p || !x || (m > 0 && (!A0 || !y || !z))) return IADMM_E_ARG;
  if (!kkt_fits(n, m) || B > 0x7fffffff) return IADMM_E_SIZE;
  MetricArgs a{(int)n, (int)m, Q, p, A0, x, y, z, obj, primal, dual};
  const int ng = ng_for(n);
  const bool vec = (n % 4 == 0) && aligned16(Q) && (m == 0 || aligned16(A0));
  const size_t lds = (3 * n + 2 * m) * sizeof(float);
  IADMM_DISPATCH_NG(ng, vec, {
    IADMM_ALLOW_LDS((metrics_kernel<NG_, V_>), lds); hipLaunchKernelGGL((metrics_kernel<NG_, V_>), dim3((unsigned)B), dim3(kKktThreads), lds,
                       (hipStream_t)stream, a);
  });
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_unscale(int64_t B, int64_t n, int64_t m, const float* D, const float* E,
                             const float* c, const float* x, const float* y, const float* z,
                             float* x_out, float* y_out, float* z_out, void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || !D || !c || !x || !x_out) return IADMM_E_ARG;
  if (m > 0 && (!E || !y || !z || !y_out || !z_out)) return IADMM_E_ARG;
  const int64_t tot = B * (n + m);
  const unsigned grid = (unsigned)((tot + 255) / 256 < 65536 ? (tot + 255) / 256 : 65536);
  hipLaunchKernelGGL(unscale_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, B, (int)n,
                     (int)m, D, E, c, x, y, z, x_out, y_out, z_out);
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_bmv(int64_t B, int64_t R, int64_t C, const float* Mx, const float* x,
                         const float* rhs, int mode, float* out, void* stream) {
  if (B <= 0 || R <= 0 || C <= 0 || !Mx || !x || !out || mode < 0 || mode > 2) return IADMM_E_ARG;
  if (mode != 0 && !rhs) return IADMM_E_ARG;
  if (R + C > 40960 || B > 0x7fffffff) return IADMM_E_SIZE;
  const int ng = ng_for(C);
  const bool vec = (C % 4 == 0) && aligned16(Mx);
  const size_t lds = (R + C) * sizeof(float);
  IADMM_DISPATCH_NG(ng, vec, {
    IADMM_ALLOW_LDS((bmv_kernel<NG_, V_>), lds); hipLaunchKernelGGL((bmv_kernel<NG_, V_>), dim3((unsigned)B), dim3(kKktThreads), lds,
                       (hipStream_t)stream, (int)R, (int)C, Mx, x, rhs, mode, out);
  });
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_kkt_matvec(int64_t B, int64_t n, int64_t m, int64_t num_ineq, const float* Q,
                                const float* A0, const float* v, float sigma, const float* scal,
                                const float* rho_rows, int transpose, float* out, void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || num_ineq < 0 || num_ineq > m) return IADMM_E_ARG;
  if (!Q || !v || !out || (m > 0 && !A0) || (m > 0 && !scal && !rho_rows)) return IADMM_E_ARG;
  if (!kkt_fits(n, m) || B > 0x7fffffff) return IADMM_E_SIZE;
  KktArgs a{(int)n, (int)m, (int)num_ineq, Q, A0, nullptr, nullptr, nullptr, nullptr, v, sigma, scal,
            nullptr, nullptr, nullptr, nullptr, nullptr};
  const int ng = ng_for(n);
  const bool vec = (n % 4 == 0) && aligned16(Q) && (m == 0 || aligned16(A0));
  const size_t lds = (3 * n + 2 * m) * sizeof(float);
  hipStream_t s = (hipStream_t)stream;
  if (transpose) {
    IADMM_DISPATCH_NG(ng, vec, { IADMM_ALLOW_LDS((kkt_matvec_kernel<NG_, V_, true>), lds); hipLaunchKernelGGL((kkt_matvec_kernel<NG_, V_, true>), dim3((unsigned)B), dim3(kKktThreads), lds, s, a, rho_rows, out); });
  } else {
    IADMM_DISPATCH_NG(ng, vec, { IADMM_ALLOW_LDS((kkt_matvec_kernel<NG_, V_, false>), lds); hipLaunchKernelGGL((kkt_matvec_kernel<NG_, V_, false>), dim3((unsigned)B), dim3(kKktThreads), lds, s, a, rho_rows, out); });
  }
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_kkt_assemble(int64_t B, int64_t n, int64_t m, int64_t num_ineq, const float* Q,
                                  const float* A0, float sigma, const float* scal,
                                  const float* rho_rows, float* K, void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || num_ineq < 0 || num_ineq > m || !Q || !K || (m > 0 && !A0))
    return IADMM_E_ARG;
  if (m > 0 && !scal && !rho_rows) return IADMM_E_ARG;
  if (n % 4 == 0 && m % 4 == 0 && aligned16(Q) && aligned16(K) && (m == 0 || aligned16(A0))) {
    const int64_t nb = (n + m + kAsmRows - 1) / kAsmRows;
    if (B > 0x7fffffff || nb > 65535) return IADMM_E_SIZE;
    hipLaunchKernelGGL(kkt_assemble_rows_kernel, dim3((unsigned)B, (unsigned)nb), dim3(256), 0, (hipStream_t)stream,
                       (int)n, (int)m, (int)num_ineq, Q, A0, sigma, scal, rho_rows, K);
    IADMM_CHECK_LAUNCH();
    return 0;
  }
  const int64_t ntile = (n + m + kAsmT - 1) / kAsmT;
  if (B > 0x7fffffff || ntile * ntile > 65535) return IADMM_E_SIZE;
  hipLaunchKernelGGL(kkt_assemble_kernel, dim3((unsigned)B, (unsigned)(ntile * ntile)), dim3(256), 0,
                     (hipStream_t)stream, (int)n, (int)m, (int)num_ineq, (int)ntile, Q, A0, sigma, scal, rho_rows, K);
  IADMM_CHECK_LAUNCH();
  return 0;
}
