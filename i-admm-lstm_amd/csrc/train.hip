// Training backward of one I-ADMM-LSTM iteration and of the unsupervised loss
// (reference: autograd through models/lstm.py:47-96 and utils.py:68-71, driven by
// main.py:336-358).  Every reduction is a fixed-order slab / per-block partial: gradients are
// bitwise reproducible.
//
// Forward of iteration t (per instance; rho_j = s*kappa_j, s = sigmoid(rho[t]), kappa = 1 on
// inequality rows, 1e3 on equality rows, iota = 1/rho, a = 2 sigmoid(alpha[t])):
//   r = K xv - b~,  g = K^T r,  in = [xv, g],  P_g = in W_g + H U_g + b_g,
//   C' = I*U + F*C,  H' = O*tanh(C'),  q = H' W_h + b_h,  xv' = xv - q,
//   x' = a x~' + (1-a) x,  zt = z + iota(v' - y),  z' = max(min(zt + iota y, zu), zl),
//   y' = y + rho (zt - z').
// Backward kernels (in the order the Python autograd Function calls them):
//   admm_update_bwd   adjoints through x', z', y', xv' -> dq, partial dx/dy/dz, d(xv) pass-through,
//                     and per-block partials of ds (through rho and iota), da and db_h
//   lstm_cell_bwd     recomputes the gate pre-activations on MFMA (same tile as the forward) and
//                     writes dP[M][4h], dC, per-row-tile W_h-gradient slabs and per-hidden-tile
//                     partials of d(in) = dP W^T
//   (gemm.hip)        dH = dP U_cat^T ; [dU_cat ; dW ; db] = [H, xv, g, 1]^T dP
//   in_reduce         sums the d(in) partials: d(xv) += din0, dg = din1
//   kkt_bwd           dr = K dg, d(xv) += K^T dr, dx -= sigma dr1, dz -= dr2, dy += iota dr2 and
//                     diota = -dg2 r2 + dr2 (y - v)   (two sweeps of Q and A0, like the forward)
//   sched_bwd         drho[t] = s(1-s) ds, dalpha[t] = 2 sig'(alpha_t) da, db_h
//   loss_grad         ||A0x-z|| + ||Qx+p+A0^T y|| per instance and its gradient (two sweeps)
#include "cell_tile.h"
#include "sweep.h"

namespace iadmm {

// ------------------------------------------------------------------ ADMM update backward
struct UpdBwdArgs {
  int64_t B;
  int n, m, num_ineq;
  const float *x, *y, *z, *xvn, *zl, *zu, *scal;            // forward inputs / output xv'
  const float *dx, *dy, *dz, *dxv;                          // adjoints of x', y', z', xv' (may be NULL)
  float *dx_o, *dy_o, *dz_o, *dxv_o, *dq;                   // outputs
  float* partials;                                          // [gridDim.x][4]: ds, da, dbh, 0
};

IADMM_DEV float dmin_a(float a, float b) { return a < b ? 1.f : (a == b ? 0.5f : 0.f); }  // d min(a,b)/da
IADMM_DEV float dmax_a(float a, float b) { return a > b ? 1.f : (a == b ? 0.5f : 0.f); }  // d max(a,b)/da

__global__ __launch_bounds__(256) void admm_update_bwd_kernel(UpdBwdArgs a) {
  __shared__ float red[8];
  const int N = a.n + a.m;
  const int64_t M = a.B * (int64_t)N;
  const float rho_in = a.scal[IADMM_S_RHO_IN], rho_eq = a.scal[IADMM_S_RHO_EQ];
  const float irho_in = a.scal[IADMM_S_IRHO_IN], irho_eq = a.scal[IADMM_S_IRHO_EQ];
  const float alpha = a.scal[IADMM_S_ALPHA], oma = a.scal[IADMM_S_1MALPHA];
  float ds = 0.f, da = 0.f, dbh = 0.f;
  for (int64_t R = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; R < M; R += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = R / N;
    const int i = (int)(R - b * N);
    float dxvt = a.dxv ? a.dxv[R] : 0.f;  // adjoint of xv' (total for this row)
    if (i < a.n) {
      const int64_t k = b * a.n + i;
      const float dxp = a.dx ? a.dx[k] : 0.f;
      dxvt += alpha * dxp;
      a.dx_o[k] = oma * dxp;
      da += dxp * (a.xvn[R] - a.x[k]);
    } else {
      const int j = i - a.n;
      const int64_t k = b * a.m + j;
      const bool ineq = j < a.num_ineq;
      const float rho = ineq ? rho_in : rho_eq, iota = ineq ? irho_in : irho_eq;
      const float kappa = ineq ? 1.f : 1e3f;
      const float y = a.y[k], z = a.z[k], v = a.xvn[R];
      const float zt = z + iota * (v - y);
      const float w = zt + iota * y;
      const float u1 = tmin(w, a.zu[k]);
      const float zn = tmax(u1, a.zl[k]);
      const float dyp = a.dy ? a.dy[k] : 0.f;
      const float dzp = a.dz ? a.dz[k] : 0.f;
      // y' = y + rho (zt - z')
      float dyo = dyp, dzt = rho * dyp, drho = dyp * (zt - zn);
      const float dzn = dzp - rho * dyp;
      // z' = max(min(w, zu), zl)
      const float dw = dzn * dmax_a(u1, a.zl[k]) * dmin_a(w, a.zu[k]);
      // w = zt + iota y
      dzt += dw;
      dyo += iota * dw;
      float diota = dw * y;
      // zt = z + iota (v - y)
      const float dzo = dzt;
      const float dv = iota * dzt;
      dyo -= iota * dzt;
      diota += dzt * (v - y);
      dxvt += dv;
      drho += -diota / (rho * rho);
      ds += kappa * drho;
      a.dy_o[k] = dyo;
      a.dz_o[k] = dzo;
    }
    a.dxv_o[R] = dxvt;   // xv' = xv - q: d(xv) gets the total adjoint ...
    a.dq[R] = -dxvt;     // ... and q gets its negative
    dbh += -dxvt;
  }
  const float s_ds = block_sum(ds, red);
  const float s_da = block_sum(da, red);
  const float s_dbh = block_sum(dbh, red);
  if (threadIdx.x == 0) {
    a.partials[blockIdx.x * 4 + 0] = s_ds;
    a.partials[blockIdx.x * 4 + 1] = s_da;
    a.partials[blockIdx.x * 4 + 2] = s_dbh;
    a.partials[blockIdx.x * 4 + 3] = 0.f;
  }
}

// ------------------------------------------------------------------ LSTM cell backward
struct CellBwdArgs {
  int64_t M;
  int h, njt, nkc, nrt;
  const float *H, *C, *xv, *g, *Upk, *Wx;
  const float *dq, *dHn, *dCn;      // adjoint of q (per row), of H', of C' (NULL = 0)
  float *dC, *dP;                   // adjoint of C (may alias dCn), dP[M][4h]
  float *whslab;                    // [nrt][h]: sum over the tile's rows of H' * dq
  float *inpart;                    // [njt][M][2]: sum over the tile's units of dP W^T
};

// Dynamic LDS: VEC: the LDS-DMA ring (cell_tile.h, kRingFloats); otherwise the register-staged
// loop's two padded tiles.
constexpr int kCellBwdLdsVec = kRingFloats * 4;
constexpr int kCellBwdLdsScalar = (128 + kRows) * kLD * 4;

template <bool VEC, bool K16>
IADMM_DEV void cell_bwd_tile(const CellBwdArgs& a, int jt, int rt, float* dsm, float* sW, float (*swh)[kJT]);

template <bool VEC, bool K16 = false>
__global__ __launch_bounds__(256, 2) void lstm_cell_bwd_kernel(CellBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float dsm[];
  __shared__ __attribute__((aligned(16))) float sW[kWxF * kJT];
  __shared__ float swh[4][kJT];
  int jt, rt;
  cell_tile_of_block(a.njt, jt, rt);
  cell_bwd_tile<VEC, K16>(a, jt, rt, dsm, sW, swh);
}

template <bool VEC, bool K16>
IADMM_DEV void cell_bwd_tile(const CellBwdArgs& a, int jt, int rt, float* dsm, float* sW, float (*swh)[kJT]) {
  const int tid = threadIdx.x, lane = tid & 63, jl = lane & 31, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = a.h;
  const int64_t M = a.M;
  const int64_t rbase = (int64_t)rt * kRows;
  if constexpr (VEC) {
    cell_fill_wpairs(a.Wx, jt, sW, tid, 256);  // pair-major, for the packed epilogue
  } else {
    for (int i = tid; i < kWxF * kJT; i += 256) {
      const int f = i / kJT, jj = i % kJT;
      sW[i] = a.Wx[(int64_t)(jt * kJT + jj) * kWxF + f];
    }
  }
  floatx16 acc[4][2];
  if constexpr (VEC) {
    cell_mainloop_dma<K16>(a.H, M, h, a.nkc, a.Upk + (int64_t)jt * a.nkc * 128 * kBK, rbase, dsm, acc, tid, wave, jl,
                      hf, [] {});
    __syncthreads();  // sW visible (the DMA loop's barriers carry no LDS-write fence)
  } else {
    cell_mainloop<VEC>(a.H, M, h, a.nkc, a.Upk + (int64_t)jt * a.nkc * 128 * kBK, rbase, dsm, dsm + 128 * kLD,
                       acc, tid, wave, jl, hf);
  }

  float whp[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) whp[q] = 0.f;
  if constexpr (VEC) {
    // Packed epilogue: unit pairs through v_pk_*_f32 (the forward's gate values bit for bit:
    // same operations as cell_epi_compute_buf).  h % 4 == 0: a lane's 4 units are all valid or not.
    // Global accesses through buffer descriptors based at the workgroup's row panel, ranges ending
    // at its last valid row (rows past M read 0 / are dropped; a NULL dH' / dC' is an empty
    // descriptor reading 0): 32-bit lane offsets and immediates instead of 64-bit address VALU and
    // load-then-select (the forward epilogue's treatment, cell_tile.h CellEpiBuf).
    const int nvalid = (int)((M - rbase) < kRows ? (M - rbase) : kRows);
    const int64_t pan = rbase * h;
    auto rs = [](const float* base, int bytes) {
      return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, bytes, 0x00020000);
    };
    const int pbytes = nvalid * h * 4;
    const __amdgpu_buffer_rsrc_t rC = rs(a.C + pan, pbytes), rdH = rs(a.dHn ? a.dHn + pan : a.C, a.dHn ? pbytes : 0),
                                 rdCn = rs(a.dCn ? a.dCn + pan : a.C, a.dCn ? pbytes : 0), rdC = rs(a.dC + pan, pbytes),
                                 rdP = rs(a.dP + pan * 4, nvalid * 4 * h * 4), rxv = rs(a.xv + rbase, nvalid * 4),
                                 rg = rs(a.g + rbase, nvalid * 4), rdq = rs(a.dq + rbase, nvalid * 4),
                                 rin = rs(a.inpart + ((int64_t)jt * M + rbase) * 2, nvalid * 8);
    const bool full = (jt + 1) * kJT <= h;
    // Eight steps (r, qq), software-pipelined by one: the loads of step st + 1 are issued before the
    // stores of step st (vmcnt counts stores as well as loads and retires them in issue order: a
    // load issued after a store cannot be waited for alone).
    // Stores (r04): the accumulator layout gives each store instruction 32 rows x 32 B (lanes jl,
    // jl + 32 hold units 8qq .. 8qq + 7 of row jl), and such scattered stores are issue-bound at the
    // texture path -- which the partner workgroup's main loop needs for its LDS-DMA (the r03 "no
    // stores" build was 1.2 of 10.4 ms faster, although nothing waited for them).  dP (4 of the 5
    // outputs) is therefore staged per 32-row block in this wave's part of the idle LDS ring,
    // [gate][row][32 units] with a 36-float row stride (conflict-free 16-B writes), and leaves as 16
    // stores of 8 rows x 128 B (whole lines); dC stays a direct store per step.
    unsigned vr[2], vo[2];
    bool rok[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int row = wave * 64 + r * 32 + jl;
      rok[r] = row < nvalid;
      vr[r] = (unsigned)row * 4u;
      vo[r] = ((unsigned)row * (unsigned)h + (unsigned)(jt * kJT + 4 * hf)) * 4u;
    }
    constexpr int kSR = kJT + 4;                    // staging row stride (floats)
    static_assert(4 * 4 * kJT * kSR <= kRingFloats, "dP staging must fit in the ring");
    float* stg = dsm + wave * (4 * kJT * kSR);      // this wave's [4 gates][32 rows][kSR]
    // transposed dP stores: lane -> row (lane >> 3) + 8 i, 16-B chunk lane & 7 of the gate's 32 units
    const int trow = lane >> 3, tch = lane & 7;
    const bool tuok = full || jt * kJT + 4 * tch < h;
    unsigned tvo[2];
#pragma unroll
    for (int r = 0; r < 2; ++r)
      tvo[r] = tuok ? ((unsigned)(wave * 64 + r * 32 + trow) * (unsigned)(4 * h) + (unsigned)(jt * kJT + 4 * tch)) * 4u
                    : 0x80000000u;
    float4 ldv[8][3];
    float rsc[2][3];
    auto qa_of = [&](int qq) -> unsigned {
      const bool uok = full || jt * kJT + 8 * qq + 4 * hf < h;
      return uok ? 32u * qq : 0x80000000u;
    };
    auto issue = [&](int st) {
      const int r = st >> 2, qq = st & 3;
      if (qq == 0) {
        rsc[r][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rxv, vr[r], 0, 0));
        rsc[r][1] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rg, vr[r], 0, 0));
        rsc[r][2] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rdq, vr[r], 0, 0));
      }
      const unsigned qa = qa_of(qq);
      ldv[st][0] = u2f4(__builtin_amdgcn_raw_buffer_load_b128(rC, vo[r] + qa, 0, 0));
      ldv[st][1] = u2f4(__builtin_amdgcn_raw_buffer_load_b128(rdH, vo[r] + qa, 0, 0));
      ldv[st][2] = u2f4(__builtin_amdgcn_raw_buffer_load_b128(rdCn, vo[r] + qa, 0, 0));
    };
    issue(0);
    float2v din0 = splat2(0.f), din1 = splat2(0.f);
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      __builtin_amdgcn_sched_barrier(0);
      const int r = st >> 2, qq = st & 3;
      const float2v in0 = splat2(rsc[r][0]), in1 = splat2(rsc[r][1]), dqv = splat2(rsc[r][2]);
      if (qq == 0) { din0 = splat2(0.f); din1 = splat2(0.f); }
      {
        const int jj0 = 8 * qq + 4 * hf;
        const bool uok = full || jt * kJT + jj0 < h;
        const bool ok4 = rok[r] && uok;
        const float4 cin4 = ldv[st][0], dh4 = ldv[st][1], dc4 = ldv[st][2];
        float4 dC4, dP4[4];
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
          auto half2 = [&](const float4& v) -> float2v { return pp ? float2v{v.z, v.w} : float2v{v.x, v.y}; };
          const int q = qq * 4 + 2 * pp;
          float2v pre[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            pre[g] = cell_pre2(in0, in1, float2v{acc[g][r][q], acc[g][r][q + 1]}, fld(3 * g), fld(3 * g + 1),
                               fld(3 * g + 2));
          }
          const float2v ig = sigmoid_cell2(pre[0]), fg = sigmoid_cell2(pre[1]), og = sigmoid_cell2(pre[2]);
          const float2v ug = tanh_cell2(pre[3]);
          const float2v cin = half2(cin4);
          const float2v c2 = ig * ug + fg * cin;
          const float2v tc = tanh_cell2(c2);
          const float2v h2 = og * tc;
          const float2v one = splat2(1.f);
          const float2v dHt = half2(dh4) + dqv * fld(12);
          const float2v dO = dHt * tc;
          const float2v dCt = half2(dc4) + dHt * og * (one - tc * tc);
          const float2v dI = dCt * ug, dU = dCt * ig, dF = dCt * cin;
          const float2v dPi = dI * ig * (one - ig), dPf = dF * fg * (one - fg);
          const float2v dPo = dO * og * (one - og), dPu = dU * (one - ug * ug);
          const float2v dCo = dCt * fg;
          if (pp == 0) {
            dC4.x = dCo.x; dC4.y = dCo.y;
            dP4[0].x = dPi.x; dP4[0].y = dPi.y; dP4[1].x = dPf.x; dP4[1].y = dPf.y;
            dP4[2].x = dPo.x; dP4[2].y = dPo.y; dP4[3].x = dPu.x; dP4[3].y = dPu.y;
          } else {
            dC4.z = dCo.x; dC4.w = dCo.y;
            dP4[0].z = dPi.x; dP4[0].w = dPi.y; dP4[1].z = dPf.x; dP4[1].w = dPf.y;
            dP4[2].z = dPo.x; dP4[2].w = dPo.y; dP4[3].z = dPu.x; dP4[3].w = dPu.y;
          }
          if (ok4) {
            const float2v wq = h2 * dqv;
            whp[q] += wq.x;
            whp[q + 1] += wq.y;
            din0 += ((dPi * fld(0) + dPf * fld(3)) + dPo * fld(6)) + dPu * fld(9);
            din1 += ((dPi * fld(1) + dPf * fld(4)) + dPo * fld(7)) + dPu * fld(10);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (st + 1 < 8) issue(st + 1);
        __builtin_amdgcn_sched_barrier(0);
        const unsigned qa = qa_of(qq);
        __builtin_amdgcn_raw_buffer_store_b128(f42u(dC4), rdC, vo[r] + qa, 0, 0);
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(stg + (g * kJT + jl) * kSR + jj0) = dP4[g];
      }
      if (qq == 3) {  // this row block's dP: 16 stores of 8 rows x 128 B
        // every value read before the first store (64 VGPRs, free once this block's accumulators
        // are): an LDS return must not land in the registers of a store still queued for issue
        // (measured: reading the next value into a just-stored register made dP nondeterministic)
        float4 tv[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int g = i >> 2, rr = trow + 8 * (i & 3);
          tv[i] = *reinterpret_cast<const float4*>(stg + (g * kJT + rr) * kSR + 4 * tch);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int g = i >> 2;
          const int so = (8 * (i & 3) * 4 * h + g * h) * 4;
          __builtin_amdgcn_raw_buffer_store_b128(f42u(tv[i]), rdP, tvo[r], so, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (qq == 3) {
        float d0 = din0.x + din0.y, d1 = din1.x + din1.y;
        d0 += __shfl_xor(d0, 32, 64);
        d1 += __shfl_xor(d1, 32, 64);
        const unsigned vi = hf ? 0x80000000u : vr[r] * 2u;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(d0), rin, vi, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(d1), rin, vi + 4u, 0, 0);
      }
    }
  } else {
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int64_t R = rbase + wave * 64 + r * 32 + jl;
    const bool rok = R < M;
    const float in0 = rok ? a.xv[R] : 0.f;
    const float in1 = rok ? a.g[R] : 0.f;
    const float dq = rok ? a.dq[R] : 0.f;
    float din0 = 0.f, din1 = 0.f;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int jj0 = 8 * qq + 4 * hf;
      const int j0 = jt * kJT + jj0;
      const int64_t o0 = R * h + j0;
      // C, dH', dC' of the lane's 4 adjacent hidden units (16-B loads when h % 4 == 0)
      float4 cin4, dh4, dc4;
      const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (VEC) {
        const bool ok4 = rok && j0 < h;
        cin4 = ok4 ? *reinterpret_cast<const float4*>(a.C + o0) : z4;
        dh4 = (ok4 && a.dHn) ? *reinterpret_cast<const float4*>(a.dHn + o0) : z4;
        dc4 = (ok4 && a.dCn) ? *reinterpret_cast<const float4*>(a.dCn + o0) : z4;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool ok = rok && j0 + e < h;
          set4(cin4, e, ok ? a.C[o0 + e] : 0.f);
          set4(dh4, e, (ok && a.dHn) ? a.dHn[o0 + e] : 0.f);
          set4(dc4, e, (ok && a.dCn) ? a.dCn[o0 + e] : 0.f);
        }
      }
      float4 wv[13];
#pragma unroll
      for (int f = 0; f < 13; ++f) wv[f] = *reinterpret_cast<const float4*>(&sW[f * kJT + jj0]);
      float4 dC4, dP4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int q = qq * 4 + e;
        const bool ok = rok && j0 + e < h;
        float pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          pre[g] = cell_pre(in0, in1, acc[g][r][q], get4(wv[3 * g], e), get4(wv[3 * g + 1], e),
                            get4(wv[3 * g + 2], e));
        }
        const float ig = sigmoid_cell(pre[0]), fg = sigmoid_cell(pre[1]), og = sigmoid_cell(pre[2]);
        const float ug = tanh_cell(pre[3]);
        const float cin = get4(cin4, e);
        const float c2 = ig * ug + fg * cin;
        const float tc = tanh_cell(c2);
        const float h2 = og * tc;
        const float wh = get4(wv[12], e);
        const float dHt = get4(dh4, e) + dq * wh;
        const float dO = dHt * tc;
        const float dCt = get4(dc4, e) + dHt * og * (1.f - tc * tc);
        const float dI = dCt * ug, dU = dCt * ig, dF = dCt * cin;
        const float dPi = dI * ig * (1.f - ig), dPf = dF * fg * (1.f - fg);
        const float dPo = dO * og * (1.f - og), dPu = dU * (1.f - ug * ug);
        set4(dC4, e, dCt * fg);
        set4(dP4[0], e, dPi); set4(dP4[1], e, dPf); set4(dP4[2], e, dPo); set4(dP4[3], e, dPu);
        if (ok) {
          whp[q] += h2 * dq;
          din0 += dPi * get4(wv[0], e) + dPf * get4(wv[3], e) + dPo * get4(wv[6], e) + dPu * get4(wv[9], e);
          din1 += dPi * get4(wv[1], e) + dPf * get4(wv[4], e) + dPo * get4(wv[7], e) + dPu * get4(wv[10], e);
        }
      }
      float* dp = a.dP + R * (int64_t)(4 * h) + j0;
      if constexpr (VEC) {
        if (rok && j0 < h) {
          *reinterpret_cast<float4*>(a.dC + o0) = dC4;
#pragma unroll
          for (int g = 0; g < 4; ++g) *reinterpret_cast<float4*>(dp + g * h) = dP4[g];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (rok && j0 + e < h) {
            a.dC[o0 + e] = get4(dC4, e);
#pragma unroll
            for (int g = 0; g < 4; ++g) dp[g * h + e] = get4(dP4[g], e);
          }
        }
      }
    }
    din0 += __shfl_xor(din0, 32, 64);
    din1 += __shfl_xor(din1, 32, 64);
    if (hf == 0 && rok) {
      a.inpart[((int64_t)jt * M + R) * 2 + 0] = din0;
      a.inpart[((int64_t)jt * M + R) * 2 + 1] = din1;
    }
  }
  }
  // W_h gradient slab: sum of H' dq over this tile's 256 rows for its 32 units (fixed order)
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    float v = whp[q];
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);  // over the 32 rows of a half
    whp[q] = v;
  }
  if (jl == 0) {
#pragma unroll
    for (int q = 0; q < 16; ++q) swh[wave][(q & 3) + 8 * (q >> 2) + 4 * hf] = whp[q];
  }
  __syncthreads();
  if (tid < kJT) {
    const int j = jt * kJT + tid;
    if (j < h) a.whslab[(int64_t)rt * h + j] = ((swh[0][tid] + swh[1][tid]) + swh[2][tid]) + swh[3][tid];
  }
}

// d(xv)[R] += sum_jt inpart[jt][R][0];  dg[R] = sum_jt inpart[jt][R][1]
__global__ void in_reduce_kernel(int64_t M, int njt, const float* inpart, float* dxv, float* dg) {
  for (int64_t R = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; R < M; R += (int64_t)gridDim.x * blockDim.x) {
    float s0 = 0.f, s1 = 0.f;
    for (int t = 0; t < njt; ++t) {
      s0 += inpart[((int64_t)t * M + R) * 2 + 0];
      s1 += inpart[((int64_t)t * M + R) * 2 + 1];
    }
    dxv[R] += s0;
    dg[R] = s1;
  }
}

// ------------------------------------------------------------------ KKT backward
struct KktBwdArgs {
  int n, m, num_ineq;
  const float *Q, *A0, *xv, *y, *r, *dg;   // r = forward residual K xv - b~ (saved)
  float sigma;
  const float* scal;
  float *dxv, *dx, *dy, *dz;                // accumulated in place
  float* ds_inst;                           // [B] partial ds of this instance
};

// dr = K dg ; d(xv) += K^T dr ; dx -= sigma dr1 ; dz -= dr2 ; dy += iota dr2 ;
// diota = -dg2 r2 + dr2 (y - v)  ->  ds += kappa * (-diota / rho^2)
template <int NG, bool VEC>
__global__ __launch_bounds__(256) void kkt_bwd_kernel(KktBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n = a.n, m = a.m, N = n + m;
  float* us = sm;        // n : dg1 -> dr1
  float* ws = us + n;    // m : dg2 -> dr2
  float* t1 = ws + m;    // n
  float* t3 = t1 + n;    // m
  float* red = t3 + m;   // n
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const size_t b = blockIdx.x;
  const float* Qb = a.Q + b * n * n;
  const float* Ab = a.A0 + b * m * n;
  for (int i = tid; i < N; i += blockDim.x) {
    if (i < n) us[i] = a.dg[b * N + i]; else ws[i - n] = a.dg[b * N + i];
  }
  __syncthreads();
  const float sigma = a.sigma;
  const float rho_in = a.scal[IADMM_S_RHO_IN], rho_eq = a.scal[IADMM_S_RHO_EQ];
  const float irho_in = a.scal[IADMM_S_IRHO_IN], irho_eq = a.scal[IADMM_S_IRHO_EQ];
  float col[NG * 4];
#pragma unroll
  for (int i = 0; i < NG * 4; ++i) col[i] = 0.f;
  // pass A: dr = K dg  (t1 = Q dg1, t3 = A0 dg1, red = A0^T dg2)
  sweep<NG, VEC, true, false>(Qb, n, n, us, nullptr, t1, col, wave, nw, lane);
  if (m > 0) sweep<NG, VEC, true, true>(Ab, m, n, us, ws, t3, col, wave, nw, lane);
  col_reduce<NG, VEC>(col, red, n, wave, nw, lane);
  float ds = 0.f;
  for (int i = tid; i < n; i += blockDim.x) us[i] = ((t1[i] + sigma * us[i]) + red[i]);  // dr1
  for (int j = tid; j < m; j += blockDim.x) {
    const bool ineq = j < a.num_ineq;
    const float rho = ineq ? rho_in : rho_eq, iota = ineq ? irho_in : irho_eq;
    const float kappa = ineq ? 1.f : 1e3f;
    const float dg2 = ws[j];
    const float dr2 = t3[j] + (-iota) * dg2;
    const float r2 = a.r[b * N + n + j];
    const float diota = -dg2 * r2 + dr2 * (a.y[b * m + j] - a.xv[b * N + n + j]);
    ds += kappa * (-diota / (rho * rho));
    ws[j] = dr2;
  }
  __syncthreads();
  // pass B: K^T dr  (red = Q^T dr1 + A0^T dr2, t3 = A0 dr1)
#pragma unroll
  for (int i = 0; i < NG * 4; ++i) col[i] = 0.f;
  sweep<NG, VEC, false, true>(Qb, n, n, nullptr, us, nullptr, col, wave, nw, lane);
  if (m > 0) sweep<NG, VEC, true, true>(Ab, m, n, us, ws, t3, col, wave, nw, lane);
  col_reduce<NG, VEC>(col, red, n, wave, nw, lane);
  for (int i = tid; i < n; i += blockDim.x) {
    a.dxv[b * N + i] += red[i] + sigma * us[i];
    a.dx[b * n + i] += -sigma * us[i];
  }
  for (int j = tid; j < m; j += blockDim.x) {
    const float iota = j < a.num_ineq ? irho_in : irho_eq;
    a.dxv[b * N + n + j] += t3[j] + (-iota) * ws[j];
    a.dz[b * m + j] += -ws[j];
    a.dy[b * m + j] += iota * ws[j];
  }
  const float s = block_sum(ds, red);
  if (tid == 0) a.ds_inst[b] = s;
}

// ------------------------------------------------------------------ schedule backward
// drho[t] += s(1-s) * (sum of ds partials), dalpha[t] += 2 sig(a)(1-sig(a)) * sum da, db_h += sum dbh
__global__ void sched_bwd_kernel(const float* rho_param, const float* alpha_param, int64_t t,
                                 const float* upd_partials, int nblk, const float* kkt_ds, int64_t B,
                                 float* drho, float* dalpha, float* dbh) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float ds = 0.f, da = 0.f, db = 0.f;
  // (r06) loads issued eight partials at a time, adds in the same order: one memory latency per eight
  // partials instead of per partial (27 us of a batch-2 iteration's 1.2 ms were this loop's chain)
  int k = 0;
  const bool al = (reinterpret_cast<uintptr_t>(upd_partials) & 15) == 0;
  for (; al && k + 8 <= nblk; k += 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(upd_partials + 4 * (k + u));
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      ds += v[u].x;
      da += v[u].y;
      db += v[u].z;
    }
  }
  for (; k < nblk; ++k) {
    ds += upd_partials[4 * k + 0];
    da += upd_partials[4 * k + 1];
    db += upd_partials[4 * k + 2];
  }
  int64_t b = 0;
  for (; b + 8 <= B; b += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = kkt_ds[b + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) ds += v[u];
  }
  for (; b < B; ++b) ds += kkt_ds[b];
  const float s = sigmoidf_(rho_param[t]);
  const float sa = sigmoidf_(alpha_param[t]);
  drho[t] += ds * s * (1.f - s);
  dalpha[t] += da * 2.f * sa * (1.f - sa);
  dbh[0] += db;
}

// ------------------------------------------------------------------ loss + gradient
struct LossArgs {
  int n, m;
  const float *Q, *p, *A0, *x, *y, *z, *cp, *cd;   // cp/cd: per-instance upstream coefficients
  float *primal, *dual, *dx, *dy, *dz;
};

// primal = ||A0 x - z||, dual = ||Q x + p + A0^T y||; dx = cp A0^T ep^ + cd Q^T ed^,
// dz = -cp ep^, dy = cd A0 ed^  (e^ = e/||e||, 0 when ||e|| = 0, like torch's norm backward)
template <int NG, bool VEC>
__global__ __launch_bounds__(256) void loss_grad_kernel(LossArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n = a.n, m = a.m;
  float* xs = sm;        // n : x -> ed^
  float* ys = xs + n;    // m : y -> ep^
  float* t1 = ys + m;    // n
  float* t3 = t1 + n;    // m
  float* red = t3 + m;   // n
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const size_t b = blockIdx.x;
  const float* Qb = a.Q + b * n * n;
  const float* Ab = a.A0 + b * m * n;
  for (int i = tid; i < n; i += blockDim.x) xs[i] = a.x[b * n + i];
  for (int j = tid; j < m; j += blockDim.x) ys[j] = a.y[b * m + j];
  __syncthreads();
  float col[NG * 4];
#pragma unroll
  for (int i = 0; i < NG * 4; ++i) col[i] = 0.f;
  sweep<NG, VEC, true, false>(Qb, n, n, xs, nullptr, t1, col, wave, nw, lane);
  if (m > 0) sweep<NG, VEC, true, true>(Ab, m, n, xs, ys, t3, col, wave, nw, lane);
  col_reduce<NG, VEC>(col, red, n, wave, nw, lane);
  float dd = 0.f, pp = 0.f;
  for (int i = tid; i < n; i += blockDim.x) {
    const float e = (t1[i] + a.p[b * n + i]) + red[i];
    t1[i] = e;
    dd = fmaf(e, e, dd);
  }
  for (int j = tid; j < m; j += blockDim.x) {
    const float e = t3[j] - a.z[b * m + j];
    t3[j] = e;
    pp = fmaf(e, e, pp);
  }
  const float nd = sqrtf(block_sum(dd, red));
  const float np = sqrtf(block_sum(pp, red));
  const float cp = a.cp ? a.cp[b] : 0.f, cd = a.cd ? a.cd[b] : 0.f;
  const float sd = nd > 0.f ? cd / nd : 0.f, sp = np > 0.f ? cp / np : 0.f;
  for (int i = tid; i < n; i += blockDim.x) xs[i] = t1[i];  // ed
  for (int j = tid; j < m; j += blockDim.x) {
    ys[j] = t3[j];                                           // ep
    if (a.dz) a.dz[b * m + j] = -sp * t3[j];
  }
  __syncthreads();
  // pass 2: red = Q^T ed (x sd) + A0^T ep (x sp) ; t3 = A0 ed
#pragma unroll
  for (int i = 0; i < NG * 4; ++i) col[i] = 0.f;
  sweep<NG, VEC, false, true>(Qb, n, n, nullptr, xs, nullptr, col, wave, nw, lane);
  float cola[NG * 4];
#pragma unroll
  for (int i = 0; i < NG * 4; ++i) cola[i] = 0.f;
  if (m > 0) sweep<NG, VEC, true, true>(Ab, m, n, xs, ys, t3, cola, wave, nw, lane);
#pragma unroll
  for (int i = 0; i < NG * 4; ++i) col[i] = sd * col[i] + sp * cola[i];
  col_reduce<NG, VEC>(col, red, n, wave, nw, lane);
  for (int i = tid; i < n; i += blockDim.x) if (a.dx) a.dx[b * n + i] = red[i];
  for (int j = tid; j < m; j += blockDim.x) if (a.dy) a.dy[b * m + j] = sd * t3[j];
  if (tid == 0) {
    if (a.primal) a.primal[b] = np;
    if (a.dual) a.dual[b] = nd;
  }
}

}  // namespace iadmm

using namespace iadmm;

extern "C" int iadmm_admm_update_bwd(int64_t B, int64_t n, int64_t m, int64_t num_ineq, const float* x,
                                     const float* y, const float* z, const float* xv_out, const float* zl,
                                     const float* zu, const float* scal, const float* dx_out,
                                     const float* dy_out, const float* dz_out, const float* dxv_out,
                                     float* dx, float* dy, float* dz, float* dxv, float* dq,
                                     float* partials, int64_t nblocks, void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || num_ineq < 0 || num_ineq > m || nblocks <= 0 || nblocks > 65535) return IADMM_E_ARG;
  if (!x || !xv_out || !scal || !dx || !dxv || !dq || !partials) return IADMM_E_ARG;
  if (m > 0 && (!y || !z || !zl || !zu || !dy || !dz)) return IADMM_E_ARG;
  UpdBwdArgs a{B, (int)n, (int)m, (int)num_ineq, x, y, z, xv_out, zl, zu, scal, dx_out, dy_out, dz_out, dxv_out,
               dx, dy, dz, dxv, dq, partials};
  hipLaunchKernelGGL(admm_update_bwd_kernel, dim3((unsigned)nblocks), dim3(256), 0, (hipStream_t)stream, a);
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_lstm_cell_bwd(int64_t M, int64_t h, const float* H, const float* C, const float* xv,
                                   const float* g, const float* Upk, const float* Wx, const float* dq,
                                   const float* dHn, const float* dCn, float* dC, float* dP, float* whslab,
                                   float* inpart, void* stream) {
  if (M <= 0 || h <= 0 || !H || !C || !xv || !g || !Upk || !Wx || !dq || !dC || !dP || !whslab || !inpart)
    return IADMM_E_ARG;
  const int64_t nrt = (M + kRows - 1) / kRows, njt = (h + kJT - 1) / kJT;
  if (nrt * njt > 0x7fffffffLL || h > (1 << 16)) return IADMM_E_SIZE;
  CellBwdArgs a{M, (int)h, (int)njt, (int)((h + kBK - 1) / kBK), (int)nrt, H, C, xv, g, Upk, Wx, dq, dHn, dCn,
                dC, dP, whslab, inpart};
  const bool vec = (h % 4 == 0) && aligned16(H) && aligned16(C) && aligned16(dC) && aligned16(dP) &&
                   (!dHn || aligned16(dHn)) && (!dCn || aligned16(dCn));
  const dim3 grid((unsigned)(nrt * njt));
  if (vec) {
    if (h % kBKd == 0) {  // no K tail: the VALU-free DMA loop (cell_tile.h mainloop_dma_k16)
      IADMM_ALLOW_LDS((lstm_cell_bwd_kernel<true, true>), kCellBwdLdsVec);
      hipLaunchKernelGGL((lstm_cell_bwd_kernel<true, true>), grid, dim3(256), kCellBwdLdsVec, (hipStream_t)stream, a);
    } else {
      IADMM_ALLOW_LDS((lstm_cell_bwd_kernel<true, false>), kCellBwdLdsVec);
      hipLaunchKernelGGL((lstm_cell_bwd_kernel<true, false>), grid, dim3(256), kCellBwdLdsVec, (hipStream_t)stream, a);
    }
  } else {
    hipLaunchKernelGGL(lstm_cell_bwd_kernel<false>, grid, dim3(256), kCellBwdLdsScalar, (hipStream_t)stream, a);
  }
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_in_reduce(int64_t M, int64_t njt, const float* inpart, float* dxv, float* dg, void* stream) {
  if (M <= 0 || njt <= 0 || !inpart || !dxv || !dg) return IADMM_E_ARG;
  const int64_t blocks = (M + 255) / 256;
  hipLaunchKernelGGL(in_reduce_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                     (hipStream_t)stream, M, (int)njt, inpart, dxv, dg);
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_kkt_bwd(int64_t B, int64_t n, int64_t m, int64_t num_ineq, const float* Q, const float* A0,
                             const float* xv, const float* y, const float* r, const float* dg, float sigma,
                             const float* scal, float* dxv, float* dx, float* dy, float* dz, float* ds_inst,
                             void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || num_ineq < 0 || num_ineq > m) return IADMM_E_ARG;
  if (!Q || !xv || !r || !dg || !scal || !dxv || !dx || !ds_inst || (m > 0 && (!A0 || !y || !dy || !dz)))
    return IADMM_E_ARG;
  if (3 * n + 2 * m > 40960 || B > 0x7fffffff) return IADMM_E_SIZE;
  KktBwdArgs a{(int)n, (int)m, (int)num_ineq, Q, A0, xv, y, r, dg, sigma, scal, dxv, dx, dy, dz, ds_inst};
  const int ng = ng_for(n);
  const bool vec = (n % 4 == 0) && aligned16(Q) && (m == 0 || aligned16(A0));
  const size_t lds = (3 * n + 2 * m) * sizeof(float);
  IADMM_DISPATCH_NG(ng, vec, {
    IADMM_ALLOW_LDS((kkt_bwd_kernel<NG_, V_>), lds); hipLaunchKernelGGL((kkt_bwd_kernel<NG_, V_>), dim3((unsigned)B), dim3(256), lds, (hipStream_t)stream, a);
  });
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_sched_bwd(const float* rho_param, const float* alpha_param, int64_t t,
                               const float* upd_partials, int64_t nblk, const float* kkt_ds, int64_t B,
                               float* drho, float* dalpha, float* dbh, void* stream) {
  if (!rho_param || !alpha_param || !upd_partials || !kkt_ds || !drho || !dalpha || !dbh || t < 0) return IADMM_E_ARG;
  hipLaunchKernelGGL(sched_bwd_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, rho_param, alpha_param, t,
                     upd_partials, (int)nblk, kkt_ds, B, drho, dalpha, dbh);
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_loss_grad(int64_t B, int64_t n, int64_t m, const float* Q, const float* p, const float* A0,
                               const float* x, const float* y, const float* z, const float* cp, const float* cd,
                               float* primal, float* dual, float* dx, float* dy, float* dz, void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || !Q || !p || !x || (m > 0 && (!A0 || !y || !z))) return IADMM_E_ARG;
  if (3 * n + 2 * m > 40960 || B > 0x7fffffff) return IADMM_E_SIZE;
  LossArgs a{(int)n, (int)m, Q, p, A0, x, y, z, cp, cd, primal, dual, dx, dy, dz};
  const int ng = ng_for(n);
  const bool vec = (n % 4 == 0) && aligned16(Q) && (m == 0 || aligned16(A0));
  const size_t lds = (3 * n + 2 * m) * sizeof(float);
  IADMM_DISPATCH_NG(ng, vec, {
    IADMM_ALLOW_LDS((loss_grad_kernel<NG_, V_>), lds); hipLaunchKernelGGL((loss_grad_kernel<NG_, V_>), dim3((unsigned)B), dim3(256), lds, (hipStream_t)stream, a);
  });
  IADMM_CHECK_LAUNCH();
  return 0;
}
