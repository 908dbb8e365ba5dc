/*
 * iadmm.h — C-ABI of the MI355X-native I-ADMM-LSTM solve loop (libiadmm.so, gfx950).
 *
 * The reference (NetSysOpt/I-ADMM-LSTM) is pure PyTorch with no FFI; its operator API is the
 * Python module surface ``models/lstm.py:LSTM.forward``, ``models/lu.py:LU.forward``,
 * ``methods/scaling.py:Scaling.scale_data`` and ``utils.py:primal_dual_loss``.  Each entry point
 * below replaces the ATen-op sequence named in its comment; the Python drop-ins under
 * ``models/``, ``methods/`` and ``utils.py`` bind them through ``ctypes``.
 *
 * Conventions
 *   - Every pointer is a DEVICE pointer to contiguous row-major fp32, batch-major
 *     ([B][rows][cols]), unless documented as host.  Integers are int64_t sizes.
 *   - ``stream`` is a hipStream_t passed as void* (0 = legacy default stream).  Calls are
 *     stream-ordered and asynchronous: no allocation, no host synchronisation, no global mutable
 *     state, no environment reads; safe to capture in a hipGraph and to call from several threads
 *     on distinct streams (tests/test_abi_concurrency_gpu.py).
 *   - Every buffer (outputs and workspaces) is caller-owned, and so are the only HIP objects the
 *     library ever creates: the look-ahead streams / events of an iadmm_lu_ctx, made and destroyed
 *     by the two (not stream-ordered) context calls below.
 *   - Return value: 0 on success; a negative IADMM_E* code for a bad argument or a size beyond
 *     a kernel's limit (nothing is launched); a positive hipError_t if a launch failed.
 *     No C++ exception crosses this boundary.
 *   - Iteration scalars (rho, 1/rho, alpha, ...) live in a small DEVICE buffer ``scal`` written by
 *     iadmm_schedule, so a whole iteration runs without a host round trip.
 */
#ifndef IADMM_H
#define IADMM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  IADMM_OK = 0,
  IADMM_E_ARG = -1,      /* null pointer / non-positive size                   */
  IADMM_E_SIZE = -2,     /* size beyond the kernel's on-chip limit            */
  IADMM_E_ALIGN = -3     /* pointer not 16-B aligned where the kernel needs it */
};

/* Layout of the per-iteration scalar buffer ``scal`` (IADMM_NSCAL floats, device). */
enum {
  IADMM_S_RHO_IN = 0,    /* sigmoid(rho[t])                        models/lstm.py:60   */
  IADMM_S_RHO_EQ = 1,    /* rho * 1e3 on equality rows             models/lstm.py:18,62 */
  IADMM_S_IRHO_IN = 2,   /* 1 / rho_in                             models/lstm.py:68-69 */
  IADMM_S_IRHO_EQ = 3,   /* 1 / rho_eq                                                  */
  IADMM_S_ALPHA = 4,     /* 2 * sigmoid(alpha[t])                  models/lstm.py:63   */
  IADMM_S_1MALPHA = 5,   /* 1 - alpha                              models/lstm.py:88   */
  IADMM_NSCAL = 8
};

/* Library / device info.  Returns the number of exported compute entry points. */
int iadmm_version(void);

/* Iteration scalars of step t from the raw parameters rho[T,1], alpha[T,1]
 * (replaces models/lstm.py:60-63).  ``scal`` gets IADMM_NSCAL floats. */
int iadmm_schedule(const float* rho_param, const float* alpha_param, int64_t t, float* scal,
                   void* stream);

/* Fixed-alpha scalars for Stage II (models/lu.py:24): copies rho entries of ``scal_in`` and
 * sets alpha / 1-alpha from the host value. */
int iadmm_schedule_fixed_alpha(const float* scal_in, float alpha, float* scal_out, void* stream);

/* Implicit-KKT residual gradient  g = K^T (K xv - b~)  (replaces models/lstm.py:67-72: the
 * K materialisation, the RHS and the two dependent bmm).  K is never formed:
 *   K = [[Q + sigma I, A0^T], [A0, -diag(1/rho_vec)]],  b~ = [sigma x - p ; z - y / rho_vec].
 * Q[B,n,n], A0[B,m,n], p/x[B,n], y/z[B,m], xv[B,n+m] -> g[B,n+m];
 * btild[B,n+m], rho_vec[B,m] and r_out[B,n+m] (= K xv - b~, kept for the training backward)
 * are optional outputs (may be NULL).
 * Rows [0,num_ineq) of A0 use rho_in, rows [num_ineq,m) rho_eq.
 * The rows of Q and A0 are split into fixed 256-row blocks spread over enough workgroups to fill
 * the chip at any B; column sums are combined per block in block order, so g does not depend on
 * B (or on how a batch is sharded).  ws: caller-owned, 16-B aligned device workspace of at least
 * iadmm_kkt_resgrad_ws_bytes(B, n, m) bytes (the same size serves iadmm_kkt_bwd_split and
 * iadmm_loss_grad_split).  Limit: iadmm_kkt_resgrad_lds_bytes(n, m) <= 160 KiB (IADMM_E_SIZE
 * otherwise); that is (n + m + k min(n, 2048)) floats with k = 8 while the sum stays within 64 KiB
 * and k = 4 above (n = m = 1000: 39 KiB; n = m = 5000: 71 KiB; n = m <= 16384). */
int64_t iadmm_kkt_resgrad_ws_bytes(int64_t B, int64_t n, int64_t m);
int64_t iadmm_kkt_resgrad_lds_bytes(int64_t n, int64_t m);
int iadmm_kkt_resgrad(int64_t B, int64_t n, int64_t m, int64_t num_ineq,
                      const float* Q, const float* A0, const float* p,
                      const float* x, const float* y, const float* z, const float* xv,
                      float sigma, const float* scal,
                      float* g, float* btild, float* rho_vec, float* r_out,
                      void* ws, int64_t ws_bytes, void* stream);

/* ||K xv - b~||_2 per instance (main.py:952 ``ls_res``), same implicit K. out[B]. */
int iadmm_kkt_lsres(int64_t B, int64_t n, int64_t m, int64_t num_ineq,
                    const float* Q, const float* A0, const float* p,
                    const float* x, const float* y, const float* z, const float* xv,
                    float sigma, const float* scal, float* out, void* stream);

/* Implicit K v (transpose=0) or K^T v (transpose=1), v/out [B,n+m]; the operator behind the
 * A_tild object the drop-in forward returns (models/lstm.py:96, used as bmm(A_tild, xv) at
 * main.py:952).  rho per class from ``scal`` or per row from ``rho_rows`` [B,m] when non-NULL.
 * Limit: 3n + 2m <= 40960. */
int iadmm_kkt_matvec(int64_t B, int64_t n, int64_t m, int64_t num_ineq, const float* Q,
                     const float* A0, const float* v, float sigma, const float* scal,
                     const float* rho_rows, int transpose, float* out, void* stream);

/* Dense K[B,n+m,n+m] (models/lstm.py:67-68, models/lu.py:28-29): for Stage II and tests.
 * rho from ``scal`` (two classes) or per row from ``rho_rows`` [B,m] when non-NULL. */
int iadmm_kkt_assemble(int64_t B, int64_t n, int64_t m, int64_t num_ineq, const float* Q,
                       const float* A0, float sigma, const float* scal, const float* rho_rows,
                       float* K, void* stream);

/* b~ = [sigma x - p ; z - y / rho] (models/lu.py:30,34) into out[B,n+m]; rho as above. */
int iadmm_kkt_rhs(int64_t B, int64_t n, int64_t m, int64_t num_ineq, const float* p,
                  const float* x, const float* y, const float* z, float sigma,
                  const float* scal, const float* rho_rows, float* out, void* stream);

/* Stage II batched LU with partial pivoting, in place (replaces torch.lu, models/lu.py:31):
 * A[B,N,N] -> packed L\U; piv[B,N] int32, 1-based like LAPACK getrf / torch.linalg.lu_factor
 * (row i was swapped with row piv[i]-1);
 * info[B] = first 1-based zero pivot or 0.  Right-looking in 128-column blocks (two 64-column halves; 16-column
 * panels up to N = 2048, 8-column panels on 1024-thread workgroups above, held in registers up to 10240 panel
 * rows and in HBM beyond; fp32-MFMA trailing updates -- rank 256 per pair of blocks at N <= 2048, rank 128
 * above -- with the block's interchanges as gathered loads up to N = 36736, as a pass of their own above;
 * limit N <= 46340, N * N < 2^31).
 * N <= 2048 (r04): the interchanges left of each block are applied once at the end.
 * ws: caller-owned, 16-B aligned device workspace of at least iadmm_lu_factor_ws_bytes(B, N) bytes
 * (per-instance block permutations -- one per 128-column block for N <= 2048, with the composed
 * left permutations, two for N <= 36736 -- and the 128x128 two-level L11^-1 blocks, two for N <= 36736,
 * one above);
 * nothing is allocated inside.
 * iadmm_lu_factor runs every launch in order on `stream`.  iadmm_lu_factor_ex with a context (N <= 36736)
 * factors the next block beside the rest of each trailing update (look-ahead) on the context's two
 * streams (high / low priority), forked from and joined back into `stream` on every path, errors
 * included: the call stays asynchronous and ordered on `stream`, and the factors are bit for bit
 * those of iadmm_lu_factor.  Under stream capture (hipGraph) the call ignores the context and runs
 * every launch on `stream` (the cross-stream fork / join crashed the HIP 7.2 runtime at capture end).
 * A context belongs to the device current at its creation (IADMM_E_ARG on another) and serves one
 * factorization at a time in its streams' order: give each concurrent caller (thread / stream) its own.
 * Block pairs (r05, the default for N <= 2048 with N % 4 == 0 and 16-B aligned rows): two 128-column
 * blocks share one rank-256 update of the columns right of them; no look-ahead there (measured slower:
 * the rank-256 update fills the GPU by itself); instead, with a context and B >= 512, the two halves
 * of the batch are factored concurrently on the context's streams (forked from and joined back into
 * `stream`), bit for bit the one-stream factors.
 * flags: 0, or any of IADMM_LU_FORCE_HBM (tests: the forms for N above the LDS-table limits -- the
 * interchange pass instead of the gathered loads -- at any N), IADMM_LU_RANK128 (one rank-128 update
 * per block at every N, with the look-ahead: the r04 form; different rounding, same accuracy),
 * IADMM_LU_PAIRS (accepted for compatibility: the default since r05). */
typedef struct iadmm_lu_ctx iadmm_lu_ctx;
enum { IADMM_LU_FORCE_HBM = 1, IADMM_LU_PAIRS = 2, IADMM_LU_RANK128 = 4 };
int iadmm_lu_ctx_create(iadmm_lu_ctx** ctx);   /* on the current device; *ctx = NULL on failure */
int iadmm_lu_ctx_destroy(iadmm_lu_ctx* ctx);   /* waits for the context's streams; NULL is a no-op */
int64_t iadmm_lu_factor_ws_bytes(int64_t B, int64_t N);
int iadmm_lu_factor(int64_t B, int64_t N, float* A, int* piv, int* info, void* ws, int64_t ws_bytes,
                    void* stream);
int iadmm_lu_factor_ex(int64_t B, int64_t N, float* A, int* piv, int* info, void* ws, int64_t ws_bytes,
                       iadmm_lu_ctx* ctx, int flags, void* stream);

/* Solve with the factors in place (replaces torch.lu_solve, models/lu.py:32,35): x[B,N] holds b
 * on entry and the solution on exit.  x lives in LDS while (N + 4224) floats fit 160 KiB (N <= 36736), in
 * HBM above (several launches per 64-row block); limit N <= 46340.  flags (_ex): 0 or IADMM_LU_FORCE_HBM
 * (the HBM form at any N, tests). */
int iadmm_lu_solve(int64_t B, int64_t N, const float* LU, const int* piv, float* x, void* stream);
int iadmm_lu_solve_ex(int64_t B, int64_t N, const float* LU, const int* piv, float* x, int flags, void* stream);

/* Pack the LSTM gate weights for the cell kernel (models/lstm.py:21-38 parameter layout).
 * W_g[2,h], U_g[h,h], b_g[h] for g in (i,f,o,u), W_h[h,1].
 * Upk: iadmm_lstm_packed_floats(h) floats; Wx: iadmm_lstm_wx_floats(h) floats. */
int64_t iadmm_lstm_packed_floats(int64_t h);
int64_t iadmm_lstm_wx_floats(int64_t h);
int iadmm_lstm_pack(int64_t h,
                    const float* W_i, const float* U_i, const float* b_i,
                    const float* W_f, const float* U_f, const float* b_f,
                    const float* W_o, const float* U_o, const float* b_o,
                    const float* W_u, const float* U_u, const float* b_u,
                    const float* W_h, float* Upk, float* Wx, void* stream);

/* Number of hidden tiles (partial-projection slabs) the cell kernel writes. */
int64_t iadmm_lstm_ntiles(int64_t h);

/* Fused coordinate-wise LSTM cell over M = B*(n+m) rows (replaces models/lstm.py:74-80):
 *   pre_g = [xv,g] W_g + H U_g + b_g ; I,F,O = sigmoid ; U = tanh
 *   C' = I*U + F*C ; H' = O*tanh(C') ; part[tile][row] = sum_{j in tile} H'[row,j] W_h[j]
 * H[M,h], C[M,h], xv[M], g[M] -> Hn[M,h], Cn[M,h], part[ntiles][M].
 * Cn may alias C (in-place cell state); Hn must not alias H.
 * The hidden x gate contraction runs on fp32 MFMA (v_mfma_f32_32x32x2_f32). */
int iadmm_lstm_cell_fwd(int64_t M, int64_t h, const float* H, const float* C,
                        const float* xv, const float* g, const float* Upk, const float* Wx,
                        float* Hn, float* Cn, float* part, void* stream);

/* ---- Optional split-precision cell ("f16x3"; not the default path) ----------------------------
 * The same cell with the hidden x gate contraction on the fp16 matrix cores
 * (v_mfma_f32_32x32x16_f16) using a 3-term split x = hi + lo of both operands
 * (U.H ~= U_hi H_hi + U_hi H_lo + U_lo H_hi, fp32 accumulation; error analysis in
 * csrc/lstm_f16x3.hip).  Half buffers are passed as void* (IEEE binary16). */

/* Halfs of the split weight layout for hidden size h (2 planes of the iadmm_lstm_pack layout). */
int64_t iadmm_lstm_packed16_halfs(int64_t h);

/* Split, power-of-two-scaled U_{i,f,o,u}[h,h] -> Upk16; wscale[2] = {2^s, 2^-s} (device). */
int iadmm_lstm_pack_f16x3(int64_t h, const float* U_i, const float* U_f, const float* U_o,
                          const float* U_u, void* Upk16, float* wscale, void* stream);

/* Y16[0..n) = fp16(x), Y16[n..2n) = fp16(x - fp16(x)) (the split planes of an fp32 tensor). */
int iadmm_split_f16(int64_t n, const float* X, void* Y16, void* stream);

/* Cell with split H: H16[2][M][h] -> Hn16[2][M][h] (must not alias H16), Cn[M,h] (may alias C),
 * part[ntiles][M]; the fp32 H' is written to Hn only when Hn != NULL.  Requires h % 8 == 0 and
 * 16-B aligned H16, Hn16, Upk16, C, Cn, Hn.  Wx from iadmm_lstm_pack. */
int iadmm_lstm_cell_fwd_f16x3(int64_t M, int64_t h, const void* H16, const float* C, const float* xv,
                              const float* g, const void* Upk16, const float* Wx, const float* wscale,
                              float* Hn, void* Hn16, float* Cn, float* part, void* stream);

/* ADMM update (replaces models/lstm.py:80 ``+ b_h`` and :82-94):
 * grad = sum_tiles part + b_h ; xv' = xv - grad ; x' = alpha xv'[:n] + (1-alpha) x ;
 * z~ = z + (v - y)/rho ; z' = clamp(z~ + y/rho, zl, zu) ; y' = y + rho (z~ - z').
 * relax_z != 0 applies alpha to z as well (models/lu.py:43, Stage II); then ``part`` is NULL
 * and ``xv`` already holds the solved xv'.  ``rho_rows`` [B,m] (optional) overrides the two-class
 * rho of ``scal`` per row (the explicit rho_vec of models/lu.py:13).  Outputs must not alias
 * inputs. rho_vec (optional output) receives the rho used per row. */
int iadmm_admm_update(int64_t B, int64_t n, int64_t m, int64_t num_ineq, int64_t ntiles,
                      const float* part, const float* b_h, const float* xv,
                      const float* x, const float* y, const float* z,
                      const float* zl, const float* zu, const float* scal,
                      const float* rho_rows, int relax_z,
                      float* xv_out, float* x_out, float* y_out, float* z_out,
                      float* rho_vec, void* stream);

/* Modified Ruiz equilibration + cost scaling, ``iters`` rounds (replaces
 * methods/scaling.py:50-119 without its dense-diagonal bmm).  Inputs may alias outputs.
 * Outputs: scaled Q,p,A0,zl,zu; diagonal vectors D[B,n], E[B,m]; c[B].
 * Limit: 3n + 2m <= 40952. */
int iadmm_ruiz_scale(int64_t B, int64_t n, int64_t m, int64_t iters,
                     const float* Q, const float* p, const float* A0,
                     const float* zl, const float* zu,
                     float* Q_out, float* p_out, float* A0_out, float* zl_out, float* zu_out,
                     float* D, float* E, float* c, void* stream);

/* Unscale iterates (main.py:1025-1027): x=D x, y=(c^-1 E) y, z=E^-1 z.  May run in place. */
int iadmm_unscale(int64_t B, int64_t n, int64_t m, const float* D, const float* E,
                  const float* c, const float* x, const float* y, const float* z,
                  float* x_out, float* y_out, float* z_out, void* stream);

/* Metrics on one batch (utils.py:53-54, 68-71): obj = 1/2 x^T Q x + p^T x,
 * primal = ||A0 x - z||_2, dual = ||Q x + p + A0^T y||_2; each out[B] (any may be NULL).
 * Limit: 3n + 2m <= 40960. */
int iadmm_metrics(int64_t B, int64_t n, int64_t m, const float* Q, const float* p,
                  const float* A0, const float* x, const float* y, const float* z,
                  float* obj, float* primal, float* dual, void* stream);

/* Batched matvec with a metric epilogue (utils.py:56-63): out[B,R] =
 *   mode 0: M x ; mode 1: max(M x - rhs, 0) (ineq_dist) ; mode 2: |rhs - M x| (eq_dist).
 * M[B,R,C], x[B,C], rhs[B,R] (unused for mode 0).  Limit: R + C <= 40960. */
int iadmm_bmv(int64_t B, int64_t R, int64_t C, const float* M, const float* x, const float* rhs,
              int mode, float* out, void* stream);

/* Backward primitives of the reporting metrics (utils.py:53-60 obj_fn / ineq_dist / eq_dist under
 * autograd; iadmm/autograd.py ObjFn, IneqDistFn, EqDistFn):
 *   iadmm_bmv_t: out[B,C] = M[B,R,C]^T v[B,R] (fixed-order sums over r; R floats of LDS <= 160 KiB)
 *   iadmm_bger:  out[B,R,C] = (accumulate ? out : 0) + u[B,R] v[B,C]^T (per-instance rank 1) */
int iadmm_bmv_t(int64_t B, int64_t R, int64_t C, const float* M, const float* v, float* out, void* stream);
int iadmm_bger(int64_t B, int64_t R, int64_t C, const float* u, const float* v, int accumulate, float* out,
               void* stream);

/* ------------------------------------------------------------------------------------------
 * Training backward (autograd through models/lstm.py:47-96 and utils.py:68-71; main.py:336-358).
 * All reductions are fixed-order partial slabs: gradients are bitwise reproducible.
 * ---------------------------------------------------------------------------------------- */

/* out[M,Ni] (+)= X[M,K] . W[Ni,K]^T on fp32 MFMA (dH = dP . U_cat^T). */
int iadmm_gemm_nt(int64_t M, int64_t Ni, int64_t K, const float* X, const float* W, float* out,
                  int accumulate, void* stream);

/* The same with W pre-packed by iadmm_gemm_pack_a into iadmm_gemm_packed_a_floats(Ni, K) floats
 * ([ceil(Ni/128)][ceil(K/32)][128][32], zero-padded): every LDS-DMA piece of W is one contiguous
 * KiB.  Requires K % 4 == 0, Ni % 4 == 0, 16-B aligned X, Wpk, out (IADMM_E_ALIGN otherwise). */
int64_t iadmm_gemm_packed_a_floats(int64_t Ni, int64_t K);
int iadmm_gemm_pack_a(int64_t Ni, int64_t K, const float* W, float* Wpk, void* stream);
int iadmm_gemm_nt_packed(int64_t M, int64_t Ni, int64_t K, const float* X, const float* Wpk, float* out,
                         int accumulate, void* stream);

/* The packed form split over K (r06: small M, e.g. the recipe's batch 2 with 80 output tiles): split y
 * takes K columns [kpart y, kpart (y + 1)), kpart = iadmm_gemm_nt_kpart(K, ksplit) (a multiple of 32;
 * every split non-empty, IADMM_E_ARG otherwise), writes slab[ksplit][M][Ni] (caller-owned scratch),
 * and the slabs are summed in split order into out (+= when accumulate).  ksplit = 1 is
 * iadmm_gemm_nt_packed (slab unused).  K % 16 == 0 with ksplit > 1. */
int64_t iadmm_gemm_nt_kpart(int64_t K, int64_t ksplit);
int iadmm_gemm_nt_packed_split(int64_t M, int64_t Ni, int64_t K, int64_t ksplit, const float* X, const float* Wpk,
                               float* slab, float* out, int accumulate, void* stream);

/* out[Ni,No] (+)= X[M,Ni]^T . Y[M,No], split over M in slices of rows_per_split (multiple of 32):
 * slab[iadmm_gemm_tn_splits(M, rows_per_split)][Ni][No] is caller-owned scratch.  fp32 MFMA for
 * Ni > 4 (dU_cat = H^T dP); Ni <= 4 (d[W_x; b] = [xv, g, 1]^T dP) streams Y once on the VALU. */
int64_t iadmm_gemm_tn_splits(int64_t M, int64_t rows_per_split);
int iadmm_gemm_tn(int64_t M, int64_t Ni, int64_t No, int64_t rows_per_split, const float* X,
                  const float* Y, float* slab, float* out, int accumulate, void* stream);

/* out[e] (+)= sum_s slab[s][e], s < nsplit, fixed order. */
int iadmm_slab_reduce(int64_t nelem, int64_t nsplit, const float* slab, float* out, int accumulate,
                      void* stream);

/* Backward of iadmm_admm_update (Stage I form): adjoints dx_out/dy_out/dz_out/dxv_out of
 * (x', y', z', xv') (NULL = 0) -> dx, dy, dz (written), dxv (written, pass-through), dq = -dxv
 * (adjoint of the projection q = H'W_h + b_h) and per-block partials[nblocks][4] =
 * (d s, d alpha-scalar a, d b_h, 0) for iadmm_sched_bwd. */
int iadmm_admm_update_bwd(int64_t B, int64_t n, int64_t m, int64_t num_ineq, const float* x,
                          const float* y, const float* z, const float* xv_out, const float* zl,
                          const float* zu, const float* scal, const float* dx_out,
                          const float* dy_out, const float* dz_out, const float* dxv_out,
                          float* dx, float* dy, float* dz, float* dxv, float* dq,
                          float* partials, int64_t nblocks, void* stream);

/* Backward of iadmm_lstm_cell_fwd: recomputes the gates (fp32 MFMA), consumes dq[M] and the
 * adjoints dHn, dCn [M,h] of H', C' (NULL = 0) and writes dC [M,h] (may alias dCn),
 * dP [M][4h] (gate pre-activation adjoints, gate-major columns g*h + j),
 * whslab [ceil(M/256)][h] (per-row-tile sums of H' dq, reduce -> dW_h) and
 * inpart [ntiles][M][2] (per-hidden-tile sums of dP W^T, reduce with iadmm_in_reduce). */
int iadmm_lstm_cell_bwd(int64_t M, int64_t h, const float* H, const float* C, const float* xv,
                        const float* g, const float* Upk, const float* Wx, const float* dq,
                        const float* dHn, const float* dCn, float* dC, float* dP, float* whslab,
                        float* inpart, void* stream);

/* dxv[R] += sum_t inpart[t][R][0] ; dg[R] = sum_t inpart[t][R][1]. */
int iadmm_in_reduce(int64_t M, int64_t ntiles, const float* inpart, float* dxv, float* dg,
                    void* stream);

/* Backward of iadmm_kkt_resgrad given dg: dr = K dg, dxv += K^T dr, dx += -sigma dr1,
 * dz += -dr2, dy += dr2 / rho, ds_inst[B] = this instance's d s through 1/rho (r = saved r_out). */
int iadmm_kkt_bwd(int64_t B, int64_t n, int64_t m, int64_t num_ineq, const float* Q,
                  const float* A0, const float* xv, const float* y, const float* r, const float* dg,
                  float sigma, const float* scal, float* dxv, float* dx, float* dy, float* dz,
                  float* ds_inst, void* stream);

/* iadmm_kkt_bwd on the row-block split of iadmm_kkt_resgrad (the same two streaming passes over
 * Q and A0, spread over enough workgroups to fill the chip at any B, e.g. the training
 * micro-batch of 128); same outputs, block-order summation (bitwise independent of B).
 * ws: >= iadmm_kkt_resgrad_ws_bytes(B, n, m) bytes, 16-B aligned. */
int iadmm_kkt_bwd_split(int64_t B, int64_t n, int64_t m, int64_t num_ineq, const float* Q,
                        const float* A0, const float* xv, const float* y, const float* r,
                        const float* dg, float sigma, const float* scal, float* dxv, float* dx,
                        float* dy, float* dz, float* ds_inst, void* ws, int64_t ws_bytes,
                        void* stream);

/* drho[t] += s(1-s) sum(ds), dalpha[t] += 2 sig(alpha_t)(1-sig(alpha_t)) sum(da), dbh += sum(db). */
int iadmm_sched_bwd(const float* rho_param, const float* alpha_param, int64_t t,
                    const float* upd_partials, int64_t nblk, const float* kkt_ds, int64_t B,
                    float* drho, float* dalpha, float* dbh, void* stream);

/* Loss of utils.py:68-71 and its gradient: primal[B] = ||A0 x - z||, dual[B] = ||Qx + p + A0^T y||,
 * dx = cp A0^T e_p/|e_p| + cd Q^T e_d/|e_d|, dy = cd A0 e_d/|e_d|, dz = -cp e_p/|e_p| with
 * per-instance upstream coefficients cp[B], cd[B] (any output may be NULL). */
int iadmm_loss_grad(int64_t B, int64_t n, int64_t m, const float* Q, const float* p,
                    const float* A0, const float* x, const float* y, const float* z,
                    const float* cp, const float* cd, float* primal, float* dual, float* dx,
                    float* dy, float* dz, void* stream);

/* iadmm_loss_grad on the row-block split (see iadmm_kkt_bwd_split); with dx = dy = dz = NULL only
 * the first streaming pass runs (primal/dual only).  ws as for iadmm_kkt_bwd_split. */
int iadmm_loss_grad_split(int64_t B, int64_t n, int64_t m, const float* Q, const float* p,
                          const float* A0, const float* x, const float* y, const float* z,
                          const float* cp, const float* cd, float* primal, float* dual, float* dx,
                          float* dy, float* dz, void* ws, int64_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Box-ceiling probes (bench.py roofline.box_ceiling; not on the solve path).
 *   iadmm_probe_mfma: ``blocks`` 256-thread workgroups, each wave issuing ``iters`` x 8
 *     v_mfma_f32_32x32x2_f32 from registers; iadmm_probe_mfma_flop(blocks, iters) flop in all;
 *     out[blocks*256] receives per-thread sums (keeps the MFMAs live).
 *   iadmm_probe_copy: float4 copy of ``bytes`` (multiple of 16, 16-B aligned src/dst): 2*bytes of
 *     HBM traffic.
 *   iadmm_probe_read: float4 read-only sweep of ``bytes`` by wg_per_cu (1..32) x CUs workgroups of 256
 *     threads, ``unroll`` (8 or 16) loads in flight per thread; out[wg_per_cu * CUs * 256] gets the
 *     per-thread sums (keeps the loads live). */
int64_t iadmm_probe_mfma_flop(int64_t blocks, int64_t iters);
int iadmm_probe_mfma(int64_t blocks, int64_t iters, float* out, void* stream);
int iadmm_probe_copy(int64_t bytes, const void* src, void* dst, void* stream);
int iadmm_probe_read(int64_t bytes, const void* src, float* out, int64_t wg_per_cu, int64_t unroll, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* IADMM_H */
