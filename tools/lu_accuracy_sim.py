"""CPU emulation of csrc/lu.hip's rounding, to find what sets the HIP factor's backward error
(||PLU - K||_F / ||K||_F at 1.8x MKL sgetrf on the N = 2000 KKT matrices).

Every rounding step of the HIP factorization is replayed in numpy on one KKT matrix
(K = [[Q + sigma I, A0^T], [A0, -diag(1/rho)]], the bench's instance distribution, rho_in = 0.5,
rho_eq = 500): an fmaf is an fp64 a - l*u rounded once to fp32 (the product of two fp32 values is
exact in fp64); a v_mfma_f32_32x32x2_f32 step is acc + a0 b0 + a1 b1 rounded once (the k pairs in
the kernels' order); everything else as the kernels write it.  Row interchanges are applied to
whole rows at once (they only move values).  Variants of the U12 = L11^-1 A12 step of the
128-column blocks (lu_linv_kernel + lu_trail128_kernel's prologue):

  linv     the explicit 128 x 128 inverse (r04: forward substitution per column with four partial
           sums), then U12 = L11^-1 A12 as MFMA pairs from zero           (the r04 kernels)
  trsm     U12 by forward substitution on A12 (one fmaf chain per element, l in order)
  twolevel inverted 32 x 32 diagonal blocks; per 32-row block j: A12_j - sum_{i<j} L_ji U_i
           (MFMA pairs, accumulated onto A12_j), then U_j = Linv_jj (.) (MFMA pairs from zero)
  linv64   the explicit inverse of each 64 x 64 half only (the in-half factors), U12 by two-level
           with 64-row blocks

and, for calibration, the same structure with every U12 / trailing product in fp64 ("exact").
Prints the backward error of each against MKL sgetrf (torch.linalg.lu_factor, fp32) and LAPACK
dgetrf, and the growth.

    python tools/lu_accuracy_sim.py [--n 1000] [--seeds 0 1] [--variants linv trsm twolevel]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "i-admm-lstm_amd"))

f32, f64 = np.float32, np.float64
NB, HALF, OB = 16, 64, 128


def r32(x):
    return np.asarray(x, dtype=f64).astype(f32)


def fma(a, l, u):
    """fmaf(-l, u, a) elementwise (broadcasting): one rounding."""
    return r32(a.astype(f64) - l.astype(f64) * u.astype(f64))


def mfma_pairs(acc, Lp, Up, pairs, sign=1.0):
    """acc[r, c] = fl(acc + sign * (L[r, k] U[k, c] + L[r, k'] U[k', c])) for (k, k') in order."""
    acc = acc.astype(f32)
    L64, U64 = Lp.astype(f64), Up.astype(f64)
    for k, k2 in pairs:
        acc = r32(acc.astype(f64) + sign * (np.outer(L64[:, k], U64[k]) + np.outer(L64[:, k2], U64[k2])))
    return acc


def kkt(n, mi, me, seed, rho_in=0.5, rho_eq=500.0, sigma=6e-6):
    from iadmm import data
    d = data.make_qp_batch(n, mi, me, 1, first_index=seed, device="cpu")
    Q, A0 = d["Q"][0].double().numpy(), d["A0"][0].double().numpy()
    m = mi + me
    rho = np.r_[np.full(mi, rho_in), np.full(me, rho_eq)]
    K = np.zeros((n + m, n + m))
    K[:n, :n] = Q + sigma * np.eye(n)
    K[:n, n:] = A0.T
    K[n:, :n] = A0
    K[n:, n:] = -np.diag(r32(1.0 / r32(rho)).astype(f64))
    return r32(K)


def panel(A, k0, cend, piv):
    """lu_panel_kernel (16 columns, rank-1 fmaf updates) + panel_finish (substitution on the half's
    columns right of the panel) + lu_update_block_vec_kernel (rank 16, one fmaf chain per element)."""
    N = A.shape[0]
    nb = min(NB, cend - k0)
    for j in range(nb):
        c = k0 + j
        p = c + int(np.argmax(np.abs(A[c:, c])))
        piv.append(p)
        if p != c:
            A[[c, p]] = A[[p, c]]
        pv = A[c, c]
        if pv != 0:
            rcp = f32(f32(1.0) / pv)
            l = r32(A[c + 1:, c].astype(f64) * f64(rcp))
            A[c + 1:, c] = l
            if c + 1 < k0 + nb:
                A[c + 1:, c + 1:k0 + nb] = fma(A[c + 1:, c + 1:k0 + nb], l[:, None], A[c, c + 1:k0 + nb][None, :])
    c0 = k0 + nb
    if c0 < cend:
        L11 = A[k0:k0 + nb, k0:k0 + nb]
        X = A[k0:k0 + nb, c0:cend].copy()
        for i in range(1, nb):
            s = X[i]
            for l_ in range(i):
                s = fma(s, L11[i, l_], X[l_])
            X[i] = s
        A[k0:k0 + nb, c0:cend] = X
        v = A[c0:, c0:cend]
        for li in range(nb):
            v = fma(v, A[c0:, k0 + li][:, None], X[li][None, :])
        A[c0:, c0:cend] = v


def factor_half(A, K0, cend, piv):
    for k0 in range(K0, cend, NB):
        panel(A, k0, cend, piv)


def subst(L, X):
    """Unit-lower forward substitution, one fmaf chain per element (l in order)."""
    X = X.copy()
    for i in range(1, L.shape[0]):
        s = X[i]
        for l_ in range(i):
            s = fma(s, L[i, l_], X[l_])
        X[i] = s
    return X


def linv_partial4(L):
    """lu_linv_kernel: X = L^-1 (unit lower, n x n), column j by substitution with four partial sums."""
    n = L.shape[0]
    X = np.zeros((n, n), f32)
    for i in range(n):
        s = [np.zeros(n, f32) for _ in range(4)]
        for k4 in range(0, i & ~3, 4):
            for q in range(4):
                s[q] = r32(s[q].astype(f64) + f64(L[i, k4 + q]) * X[k4 + q].astype(f64))
        for k in range(i & ~3, i):
            s[0] = r32(s[0].astype(f64) + f64(L[i, k]) * X[k].astype(f64))
        v = -r32(r32(s[0].astype(f64) + s[1]).astype(f64) + r32(s[2].astype(f64) + s[3]))
        row = np.where(np.arange(n) > i, f32(0), np.where(np.arange(n) == i, f32(1), v))
        X[i] = row
    return X


PRO_PAIRS = [(32 * p + t, 64 + 32 * p + t) for p in range(2) for t in range(32)]  # trail128 prologue
MAIN_PAIRS = [(t, 64 + t) for t in range(64)]                                     # trail128 main loop
MID_PAIRS = [(s, 32 + s) for s in range(32)]                                      # lu_trail_kernel


def u12(A, P, c2, variant):
    L = np.tril(A[P:c2, P:c2], -1)
    A12 = A[P:c2, c2:]
    nbk = c2 - P
    if variant == "exact":
        Lu = L.astype(f64) + np.eye(nbk)
        return np.linalg.solve(Lu, A12.astype(f64))
    if variant == "linv":
        Li = linv_partial4(L)
        return mfma_pairs(np.zeros_like(A12), Li, A12, PRO_PAIRS)
    if variant == "trsm":
        return subst(L, A12)
    if variant in ("twolevel", "linv64"):
        bs = 32 if variant == "twolevel" else 64
        U = np.zeros_like(A12)
        for j in range(0, nbk, bs):
            rhs = A12[j:j + bs].copy()
            if j:
                rhs = mfma_pairs(rhs, L[j:j + bs, :j], U[:j], [(k, k + j // 2) for k in range(j // 2)], sign=-1.0)
            Li = linv_partial4(L[j:j + bs, j:j + bs])
            U[j:j + bs] = mfma_pairs(np.zeros_like(rhs), Li, rhs, [(t, bs // 2 + t) for t in range(bs // 2)])
        return U
    raise ValueError(variant)


def hip_lu(K, variant):
    A = K.copy()
    N = A.shape[0]
    piv = []
    for P in range(0, N, OB):
        c1, c2 = min(N, P + HALF), min(N, P + OB)
        factor_half(A, P, c1, piv)
        if c1 < N:
            # first half's U12 on the second half's columns (lu_swap_kernel TRSM), then the rank-64 mid
            # update (lu_trail_kernel: acc from A22, -L21 (.) U12 as MFMA pairs)
            A[P:c1, c1:c2] = subst(np.tril(A[P:c1, P:c1], -1), A[P:c1, c1:c2])
            A[c1:, c1:c2] = mfma_pairs(A[c1:, c1:c2], A[c1:, P:c1], A[P:c1, c1:c2], MID_PAIRS, sign=-1.0)
            factor_half(A, c1, c2, piv)
        if c2 >= N:
            break
        U = u12(A, P, c2, variant)
        if variant == "exact":
            A[c2:, c2:] = r32(A[c2:, c2:].astype(f64) - A[c2:, P:c2].astype(f64) @ U)
            A[P:c2, c2:] = r32(U)
        else:
            prod = mfma_pairs(np.zeros((N - c2, N - c2), f32), A[c2:, P:c2], U, MAIN_PAIRS)
            A[c2:, c2:] = r32(A[c2:, c2:].astype(f64) - prod)
            A[P:c2, c2:] = U
    return A, np.array(piv)


def berr(K, LU, piv):
    N = K.shape[0]
    L = np.tril(LU.astype(f64), -1) + np.eye(N)
    U = np.triu(LU.astype(f64))
    PA = K.astype(f64).copy()
    for i, p in enumerate(piv):
        if p != i:
            PA[[i, p]] = PA[[p, i]]
    R = L @ U - PA
    return float(np.linalg.norm(R) / np.linalg.norm(K.astype(f64))), float(np.abs(U).max() / np.abs(K).max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--seeds", type=int, nargs="+", default=[0])
    ap.add_argument("--variants", nargs="+", default=["linv", "trsm", "twolevel", "linv64", "exact"])
    a = ap.parse_args()
    torch.set_num_threads(1)
    for seed in a.seeds:
        K = kkt(a.n, a.n // 2, a.n // 2, seed)
        lu, pv = torch.linalg.lu_factor(torch.from_numpy(K))
        pv = pv.numpy() - 1
        b_mkl, g_mkl = berr(K, lu.numpy(), pv)
        lu64, pv64 = torch.linalg.lu_factor(torch.from_numpy(K.astype(f64)))
        b64, _ = berr(K, lu64.numpy().astype(f64), pv64.numpy() - 1)
        print(f"seed {seed} N {K.shape[0]}: MKL sgetrf berr {b_mkl:.3e} growth {g_mkl:.1f} | dgetrf {b64:.1e}", flush=True)
        for v in a.variants:
            t = time.time()
            LU, piv = hip_lu(K, v)
            b, g = berr(K, LU, piv)
            same = np.array_equal(piv, pv)
            print(f"  {v:9s} berr {b:.3e} = {b / b_mkl:.2f} x MKL, growth {g:.1f}, pivots = MKL's: {same} ({time.time() - t:.0f} s)",
                  flush=True)


if __name__ == "__main__":
    main()
