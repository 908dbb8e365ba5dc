"""Synthetic QP instances (restating the QP branch of generate_data.py:67-76 + main.py:718).

Per instance i (global index): Q = diag(u), u ~ U[0,1) (the reference draws 0.5*diag(rand) and
doubles it at load, main.py:718: exact in fp32), p ~ U[0,1)^n, A ~ N(0,1)^{me x n},
b ~ U(-1,1)^me, G ~ N(0,1)^{mi x n}, c = rowsum |G pinv(A)|, A0 = [G; A], zl = [-inf; b],
zu = [c; b].  The OSQP "solved" filter is not applied (OSQP is not available; it only drops
instances).  Each instance uses its own generator seeded ``seed + global_index`` so any shard of
the batch reproduces the same instances on any device count.

pinv(A) is computed as A^T (A A^T)^-1 in fp64 (A has full row rank almost surely); this is data
generation, outside every timed region.
"""
from __future__ import annotations

import torch


def _spd_solve(S, R, iters=200, rtol=1e-13):
    """S^-1 R for SPD S (columns of R solved independently) by conjugate gradients in fp64.

    Only batched matmuls: no LAPACK/rocSOLVER call (this torch build's multi-threaded MKL LASWP
    hangs on some CPU inputs and hipblasDgetrfBatched failed to allocate on the box).
    S = A A^T of a Gaussian A (m_e x n, n = 2 m_e) has condition number ~34, so CG converges to
    ~1e-13 in well under 200 steps."""
    X = torch.zeros_like(R)
    Rr = R.clone()
    P = Rr.clone()
    rr = (Rr * Rr).sum(1, keepdim=True)
    r0 = rr.clamp_min(1e-300)
    for _ in range(iters):
        SP = S @ P
        a = rr / (P * SP).sum(1, keepdim=True).clamp_min(1e-300)
        X += a * P
        Rr -= a * SP
        rn = (Rr * Rr).sum(1, keepdim=True)
        if bool((rn <= (rtol * rtol) * r0).all()):
            break
        P = Rr + (rn / rr.clamp_min(1e-300)) * P
        rr = rn
    return X


def make_qp_batch(n, num_ineq, num_eq, B, first_index=0, seed=17, device="cuda", chunk=64):
    """Returns dict(Q[B,n,n], p[B,n,1], A0[B,m,n], zl[B,m,1], zu[B,m,1]) fp32 on ``device``."""
    m = num_ineq + num_eq
    dev = torch.device(device)
    Q = torch.zeros(B, n, n, dtype=torch.float32, device=dev)
    p = torch.empty(B, n, 1, dtype=torch.float32, device=dev)
    A0 = torch.empty(B, m, n, dtype=torch.float32, device=dev)
    zl = torch.empty(B, m, 1, dtype=torch.float32, device=dev)
    zu = torch.empty(B, m, 1, dtype=torch.float32, device=dev)
    for i in range(B):
        g = torch.Generator(device=dev).manual_seed(int(seed) + int(first_index) + i)
        Q[i].diagonal().copy_(torch.rand(n, generator=g, device=dev))
        p[i, :, 0] = torch.rand(n, generator=g, device=dev)
        A0[i, num_ineq:] = torch.randn(num_eq, n, generator=g, device=dev)
        zl[i, num_ineq:, 0] = 2 * torch.rand(num_eq, generator=g, device=dev) - 1
        A0[i, :num_ineq] = torch.randn(num_ineq, n, generator=g, device=dev)
    zu[:, num_ineq:] = zl[:, num_ineq:]
    zl[:, :num_ineq] = -float("inf")
    for s in range(0, B, chunk):
        e = min(B, s + chunk)
        G = A0[s:e, :num_ineq].double()
        if num_eq > 0:
            A = A0[s:e, num_ineq:].double()
            X = _spd_solve(A @ A.transpose(1, 2), A @ G.transpose(1, 2))  # (AA^T)^-1 A G^T
            c = X.transpose(1, 2).abs().sum(dim=2)                                # |G A^T (AA^T)^-1|
        else:
            c = 0.5 * G.abs().sum(dim=2)
        zu[s:e, :num_ineq, 0] = c.float()
    return dict(Q=Q, p=p, A0=A0, zl=zl, zu=zu)


def init_lstm_params(hidden, length, input_dim=2, seed=17, device="cuda"):
    """Random-init weights with the reference's distribution and draw order
    (models/lstm.py:21-41: N(0, 0.01) for W/U/W_h/rho/alpha, zeros for biases)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    nrm = lambda *s: torch.normal(0.0, 0.01, size=s, generator=g)  # noqa: E731
    out = {}
    for gate in ("i", "f", "o", "u"):
        out["W_" + gate] = nrm(input_dim, hidden)
        out["U_" + gate] = nrm(hidden, hidden)
        out["b_" + gate] = torch.zeros(hidden)
    out["W_h"] = nrm(hidden, 1)
    out["b_h"] = torch.zeros(1)
    out["rho"] = nrm(length, 1)
    out["alpha"] = nrm(length, 1)
    return {k: v.to(device) for k, v in out.items()}
