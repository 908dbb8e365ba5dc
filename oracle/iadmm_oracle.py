"""CPU ORACLE for the I-ADMM-LSTM solve loop — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / the CPU baseline.  The product path (``iadmm`` + the HIP
library) never imports it and has no CPU fallback.

It is a PyTorch-CPU fp32 restatement of the reference algorithm that keeps the reference's op
structure (explicit KKT matrix, ``bmm`` matvecs, four gate GEMMs, dense-diagonal Ruiz), so that
(a) its outputs are pinned bit-for-bit (or to a stated ulp tolerance) against the golden vectors
in ``tests/golden/*.npz`` that were produced by importing the reference itself
(``tests/golden/make_golden.py``), and (b) its run time is the reference's CPU cost.

Reference anchors (``/root/reference``):
  * ``models/lstm.py:47-96``  one Stage-I iteration  -> :func:`lstm_iteration`
  * ``models/lu.py:13-47``    one Stage-II iteration -> :func:`lu_iteration`
  * ``methods/scaling.py:17-119`` modified Ruiz     -> :func:`ruiz`
  * ``utils.py:53-78``        metrics               -> :func:`primal_dual`, :func:`objective`,
                                                       :func:`ineq_dist`, :func:`eq_dist`, :func:`aug_lagr`
  * ``main.py:818-1031``      test-mode solve loop  -> :func:`solve`
"""
from __future__ import annotations

import torch

RHO_EQ_OVER_RHO_INEQ = 1e03  # models/lstm.py:18
GATES = ("i", "f", "o", "u")  # models/lstm.py:21-35 (input, forget, output, update/cell)


# ----------------------------------------------------------------------------- schedule
def schedule(params, t, y_like, num_ineq, num_eq):
    """rho_vec and alpha of iteration t (models/lstm.py:60-63).

    Returns (rho_vec [B,m,1], alpha [1]).  Inequality rows get sigmoid(rho[t]); equality rows
    [num_ineq, num_ineq+num_eq) get 1e3 * that.
    """
    r = torch.sigmoid(params["rho"][t, :])
    rv = torch.ones(size=y_like.shape, device=y_like.device, dtype=y_like.dtype) * r
    lo, hi = num_ineq, num_ineq + num_eq
    rv[:, lo:hi, :] = rv[:, lo:hi, :] * RHO_EQ_OVER_RHO_INEQ
    return rv, 2 * torch.sigmoid(params["alpha"][t, :])


# ----------------------------------------------------------------------------- KKT system
def kkt_matrix(Q, A0, sigma, rho_vec):
    """Dense K = [[Q + sigma I, A0^T], [A0, -diag(1/rho_vec)]] (models/lstm.py:67-68)."""
    Bsz, n, _ = Q.shape
    m = A0.shape[1]
    K = torch.empty((Bsz, n + m, n + m), dtype=Q.dtype)
    K[:, :n, :n] = Q + sigma * torch.diag_embed(torch.ones(size=(Bsz, n), dtype=Q.dtype))
    K[:, :n, n:] = A0.permute(0, 2, 1)
    K[:, n:, :n] = A0
    K[:, n:, n:] = -(1 / rho_vec) * torch.diag_embed(torch.ones(size=(Bsz, m), dtype=Q.dtype))
    return K


def kkt_rhs(x, z, y, p, sigma, rho_vec):
    """b~ = [sigma x - p ; z - y / rho_vec] (models/lstm.py:69, models/lu.py:30)."""
    return torch.cat((sigma * x - p, z - (1 / rho_vec) * y), dim=1)


def kkt_resgrad(K, b, xv):
    """g = K^T (K xv - b~) (models/lstm.py:72)."""
    return torch.bmm(K.permute(0, 2, 1), torch.bmm(K, xv) - b)


# ----------------------------------------------------------------------------- Stage I
def lstm_cell(params, inputs, H, C):
    """Coordinate-wise LSTM cell + output projection (models/lstm.py:74-80)."""
    pre = {}
    for gname in GATES:
        pre[gname] = inputs @ params["W_" + gname] + H @ params["U_" + gname] + params["b_" + gname]
    ig, fg, og = (torch.sigmoid(pre[k]) for k in ("i", "f", "o"))
    ug = torch.tanh(pre["u"])
    C_new = ig * ug + fg * C
    H_new = og * torch.tanh(C_new)
    step = H_new @ params["W_h"] + params["b_h"]
    return H_new, C_new, step


def admm_relax_project(xv_new, x, y, z, zl, zu, rho_vec, alpha, relax_z=False):
    """x/z/y updates shared by both stages (models/lstm.py:84-94, models/lu.py:38-45)."""
    n = x.shape[1]
    x_t, v = xv_new[:, :n, :], xv_new[:, n:, :]
    z_t = z + (1 / rho_vec) * (v - y)
    x_out = alpha * x_t + (1 - alpha) * x
    z_rel = alpha * z_t + (1 - alpha) * z if relax_z else z_t  # lstm.py:91-92 vs lu.py:43
    z_out = torch.max(torch.min(z_rel + (1 / rho_vec) * y, zu), zl)
    y_out = y + rho_vec * (z_rel - z_out)
    return x_out, y_out, z_out


def lstm_iteration(params, t, num_ineq, num_eq, x, y, z, xv, sigma, H, C, Q, p, A0, zl, zu):
    """One I-ADMM-LSTM iteration; same return tuple as models/lstm.py:96."""
    rho_vec, alpha = schedule(params, t, y, num_ineq, num_eq)
    K = kkt_matrix(Q, A0, sigma, rho_vec)
    b = kkt_rhs(x, z, y, p, sigma, rho_vec)
    inputs = torch.cat([xv, kkt_resgrad(K, b, xv)], dim=-1)
    H, C, step = lstm_cell(params, inputs, H, C)
    xv = xv - step
    x, y, z = admm_relax_project(xv, x, y, z, zl, zu, rho_vec, alpha)
    return x, y, z, xv, H, C, K, b, rho_vec


# ----------------------------------------------------------------------------- Stage II
def lu_iteration(rho_vec, x, y, z, xv, sigma, K, lu, piv, Q, p, A0, zl, zu, alpha=1.6):
    """Exact ADMM iteration with a cached LU of K (models/lu.py:13-47)."""
    b = kkt_rhs(x, z, y, p, sigma, rho_vec)
    if lu is None and piv is None:
        K = kkt_matrix(Q, A0, sigma, rho_vec)
        lu, piv = torch.linalg.lu_factor(K)
    xv = torch.linalg.lu_solve(lu, piv, b)
    x, y, z = admm_relax_project(xv, x, y, z, zl, zu, rho_vec, alpha, relax_z=True)
    return x, y, z, xv, K, b, lu, piv


# ----------------------------------------------------------------------------- Ruiz
def _clamp_scaling(v, lo=1e-4, hi=1e4):
    """methods/scaling.py:26-46 (tensor branch): clamp, and values that hit the floor -> 1."""
    out = torch.clamp(v, min=lo, max=hi)
    out[out == lo] = 1.0
    return out


def ruiz(Q, p, A0, zl, zu, iters=10):
    """Modified Ruiz equilibration + cost scaling (methods/scaling.py:50-119).

    Keeps the reference's dense-diagonal ``bmm`` formulation (its cost is part of the CPU
    baseline).  Returns the scaled data and the dense D, E, Einv, cinv, c.
    """
    Bsz, n, _ = Q.shape
    m = A0.shape[1]
    eye_n = torch.diag_embed(torch.ones(size=(Bsz, n), dtype=Q.dtype))
    D = eye_n
    E = torch.diag_embed(torch.ones(size=(Bsz, m), dtype=Q.dtype))
    c = 1.0
    for _ in range(iters):
        col_top = torch.max(torch.linalg.norm(Q, ord=torch.inf, dim=1),
                            torch.linalg.norm(A0, ord=torch.inf, dim=1))
        col_bot = torch.linalg.norm(A0, ord=torch.inf, dim=2)
        s = torch.reciprocal(torch.sqrt(_clamp_scaling(torch.cat((col_top, col_bot), dim=-1))))
        Dk = torch.diag_embed(s[:, :n])
        Ek = torch.diag_embed(s[:, n:])
        Q = torch.bmm(Dk, torch.bmm(Q, Dk))
        A0 = torch.bmm(Ek, torch.bmm(A0, Dk))
        p = torch.bmm(Dk, p)
        e = Ek.diagonal(dim1=1, dim2=2).unsqueeze(-1)
        zl = e * zl
        zu = e * zu
        D = torch.bmm(Dk, D)
        E = torch.bmm(Ek, E)
        qcol = torch.linalg.norm(Q, ord=torch.inf, dim=1).mean(-1, keepdim=True)
        pinf = _clamp_scaling(torch.linalg.norm(p, ord=torch.inf, dim=1))
        ck = 1.0 / _clamp_scaling(torch.max(pinf, qcol))
        Q = ck.unsqueeze(-1) * Q
        p = ck.unsqueeze(-1) * p
        c = ck.unsqueeze(-1) * c
    Einv = torch.diag_embed(torch.reciprocal(E.diagonal(dim1=-2, dim2=-1)))
    return dict(Q=Q, p=p, A0=A0, zl=zl, zu=zu, D=D, E=E, Einv=Einv, c=c, cinv=1.0 / c)


# ----------------------------------------------------------------------------- metrics
def objective(x, Q, p):
    """utils.py:53-54."""
    return 0.5 * torch.bmm(x.permute(0, 2, 1), torch.bmm(Q, x)) + torch.bmm(p.permute(0, 2, 1), x)


def ineq_dist(x, G, c):
    """utils.py:56-57."""
    return torch.clamp(torch.bmm(G, x) - c, 0)


def eq_dist(x, A, b):
    """utils.py:59-60."""
    return torch.abs(b - torch.bmm(A, x))


def aug_lagr(x, z, y, Q, p, A0, rho_vec):
    """utils.py:74-78 (with its Q p term)."""
    r = torch.bmm(A0, x) - z
    fx = 0.5 * torch.bmm(x.permute(0, 2, 1), torch.bmm(Q, p)) + torch.bmm(p.permute(0, 2, 1), x)
    dual_item = torch.bmm(y.permute(0, 2, 1), r)
    aug_item = 0.5 * torch.bmm(r.permute(0, 2, 1), torch.bmm(torch.diag_embed(rho_vec.squeeze(-1)), r))
    return fx + dual_item + aug_item


def primal_dual(x, y, z, Q, p, A0):
    """utils.py:68-71: per-instance ||A0 x - z||_2 and ||Q x + p + A0^T y||_2, [B,1,1]."""
    pr = torch.linalg.vector_norm(torch.bmm(A0, x) - z, dim=(1, 2), keepdim=True)
    du = torch.linalg.vector_norm(torch.bmm(Q, x) + p + torch.bmm(A0.permute(0, 2, 1), y),
                                  dim=(1, 2), keepdim=True)
    return pr, du, pr + du


def unscale(sc, x, y, z):
    """main.py:1025-1027."""
    return torch.bmm(sc["D"], x), torch.bmm(sc["cinv"] * sc["E"], y), torch.bmm(sc["Einv"], z)


# ----------------------------------------------------------------------------- driver
def solve(params, Q, p, A0, zl, zu, num_ineq, num_eq, T, sigma, hidden, scaling=True,
          scaling_iters=10, history=False, trace=False):
    """Test-mode solve of one batch (main.py:818-1031): scale, T Stage-I iterations, unscale.

    Returns a dict with the unscaled final iterate, the scaled state and the final primal/dual
    residuals on the unscaled data.  ``history=True`` also records per-iteration residuals;
    ``trace=True`` the unscaled iterate of every iteration (``trace_x/y/z`` [T,B,*,1]).  The
    arithmetic type is that of the inputs: fp64 data and parameters give the fp64 trajectory the
    K = 100 envelope test (tests/k100_envelope.py) measures both fp32 paths against.
    """
    Bsz, n, _ = Q.shape
    m = A0.shape[1]
    Qu, pu, A0u = Q, p, A0
    sc = None
    if scaling:
        sc = ruiz(Q, p, A0, zl, zu, scaling_iters)
        Q, p, A0, zl, zu = sc["Q"], sc["p"], sc["A0"], sc["zl"], sc["zu"]
    dt = dict(dtype=Q.dtype)
    x = torch.zeros(Bsz, n, 1, **dt)
    y = torch.zeros(Bsz, m, 1, **dt)
    z = torch.zeros(Bsz, m, 1, **dt)
    xv = torch.zeros(Bsz, n + m, 1, **dt)
    H = torch.zeros(Bsz, n + m, hidden, **dt)
    C = torch.zeros(Bsz, n + m, hidden, **dt)
    hist = []
    tr = []
    rho_vec = None
    for t in range(T):
        x, y, z, xv, H, C, _, _, rho_vec = lstm_iteration(params, t, num_ineq, num_eq, x, y, z, xv,
                                                          sigma, H, C, Q, p, A0, zl, zu)
        if history or trace:
            xs, ys, zs = unscale(sc, x, y, z) if scaling else (x, y, z)
            if trace:
                tr.append((xs, ys, zs))
        if history:
            pr, du, _ = primal_dual(xs, ys, zs, Qu, pu, A0u)
            hist.append((pr.reshape(-1), du.reshape(-1)))
    out = dict(x_scaled=x, y_scaled=y, z_scaled=z, xv=xv, H=H, C=C, rho_vec=rho_vec, scaling=sc)
    if scaling:
        x, y, z = unscale(sc, x, y, z)
    pr, du, _ = primal_dual(x, y, z, Qu, pu, A0u)
    out.update(x=x, y=y, z=z, primal=pr.reshape(-1), dual=du.reshape(-1))
    if history:
        out["hist_primal"] = torch.stack([h[0] for h in hist])
        out["hist_dual"] = torch.stack([h[1] for h in hist])
    if trace:
        for i, k in enumerate(("x", "y", "z")):
            out["trace_" + k] = torch.stack([t[i] for t in tr])
    return out


def params_from_npz(f):
    """The 16 reference parameters (models/lstm.py:21-41) from a golden fixture."""
    names = [f"{a}_{g}" for g in GATES for a in ("W", "U", "b")] + ["W_h", "b_h", "rho", "alpha"]
    return {k: torch.from_numpy(f["param_" + k]) for k in names}
