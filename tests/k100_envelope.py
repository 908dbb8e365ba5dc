"""Stage-I K = 100 parity against an fp64 envelope (models/lstm.py:47-96,
main.py:874-988, utils.py:68-71), for any weight set.

From identical inputs (the bench's instances, one weight set) three trajectories run the whole
solve -- Ruiz, T Stage-I iterations, unscale after every iteration:

* the HIP path (``iadmm.solver.solve`` with an ``iter_hook`` that keeps every unscaled iterate);
* the CPU oracle in fp32 (the reference's op structure, MKL ``sgemm``/``bmm``);
* the same oracle in fp64 (data and parameters promoted; the "exact" trajectory).

The bound (stated before it was measured, modelled on tests/stage2_envelope.py), per iteration t
and per instance b:

* iterates x, y, z:  rel-L2(GPU - fp64) <= FACTOR * rel-L2(fp32 oracle - fp64) + FLOOR;
* residual vectors r_p = A0 x - z and r_d = Q x + p + A0^T y (each trajectory's state evaluated
  in fp64 on the unscaled data):  ||r(GPU) - r(fp64)|| <= FACTOR * ||r(fp32) - r(fp64)|| +
  FLOOR * ||r(fp64)||;
* the reported metrics (the GPU's on-device primal / dual history, the numbers main.py prints):
  |primal_GPU - ||r_p(fp64)||| within the same vector bound (| ||a|| - ||b|| | <= ||a - b||).

So the fp32 oracle -- the reference's own arithmetic in another summation order -- defines how far
an fp32 implementation may land from the exact trajectory at each iteration; a weight set whose
dynamics amplify rounding widens the envelope for the oracle exactly as for the GPU, and one
that does not keeps it tight.  No fixed relative tolerance, so a choice of weights cannot turn the
test green or red by itself.  The worst ratio (distance / bound) is reported with its iteration
and instance, and for the primal residual the cancellation ratio ||A0 x|| / ||r_p|| there.
"""
from __future__ import annotations

import os

import torch

from oracle import iadmm_oracle as orc

FACTOR = 2.0
FLOOR = 1e-7


def oracle_run(params, cpu, num_ineq, num_eq, T, sigma, hidden, dtype):
    """Oracle solve in ``dtype`` with per-iteration unscaled iterates and residual histories."""
    threads = torch.get_num_threads()
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    try:
        pc = {k: v.detach().cpu().to(dtype) for k, v in params.items()}
        d = {k: v.cpu().to(dtype) for k, v in cpu.items()}
        with torch.no_grad():
            return orc.solve(pc, d["Q"], d["p"], d["A0"], d["zl"], d["zu"], num_ineq, num_eq, T, sigma, hidden,
                             history=True, trace=True)
    finally:
        torch.set_num_threads(threads)


def gpu_run(params, dev_data, num_ineq, num_eq, T, sigma):
    """HIP solve with every unscaled iterate copied out (the hook runs in the untimed history span)."""
    from iadmm import solver
    tr = {"x": [], "y": [], "z": []}

    def hook(t, ux, uy, uz):
        tr["x"].append(ux.clone())
        tr["y"].append(uy.clone())
        tr["z"].append(uz.clone())

    d = dev_data
    with torch.no_grad():
        out = solver.solve(params, d["Q"], d["p"], d["A0"], d["zl"], d["zu"], num_ineq, num_eq, T, sigma,
                           history=True, iter_hook=hook)
    for k in tr:
        out["trace_" + k] = torch.stack(tr[k]).double().cpu()
    return out


def _rel(a, b):
    """Per-instance rel-L2 over the trailing dims: a, b [B, ...] -> [B]."""
    B = b.shape[0]
    a, b = a.reshape(B, -1), b.reshape(B, -1)
    return (a - b).norm(dim=1) / b.norm(dim=1).clamp_min(1e-30)


def check(gpu, r32, r64, cpu, tag, verbose=True, factor=FACTOR):
    """Evaluates the envelope; returns (fails, summary).  ``summary`` holds the worst ratio per
    quantity with its (iteration, instance) and, for the primal residual, ||A0 x|| / ||r_p||."""
    Qd, pd, Ad = (cpu[k].double() for k in ("Q", "p", "A0"))
    B = Qd.shape[0]
    T = r64["trace_x"].shape[0]

    def resid(x, y, z):
        x, y, z = (v.reshape(B, -1, 1).double() for v in (x, y, z))
        Ax = Ad @ x
        return Ax - z, Qd @ x + pd + Ad.transpose(1, 2) @ y, Ax

    fails = []
    worst = {}

    def note(key, ratio, t, extra=None):
        r = float(ratio.max())
        b = int(ratio.argmax())
        if key not in worst or r > worst[key][0]:
            worst[key] = (r, t, b, extra[b] if extra is not None else None)

    for t in range(T):
        line = []
        for k in ("x", "y", "z"):
            g, a, e = (tr["trace_" + k][t].reshape(B, -1).double() for tr in (gpu, r32, r64))
            dg, d32 = _rel(g, e), _rel(a, e)
            bound = factor * d32 + FLOOR
            note(k, dg / bound, t)
            if bool((dg > bound).any()):
                fails.append((tag, t, k, dg.tolist(), bound.tolist()))
            line.append(f"{k} {float(dg.max()):.1e}/{float(d32.max()):.1e}")
        st = {}
        for name, tr in (("gpu", gpu), ("f32", r32), ("f64", r64)):
            st[name] = resid(tr["trace_x"][t], tr["trace_y"][t], tr["trace_z"][t])
        for i, k in enumerate(("primal", "dual")):
            v64 = st["f64"][i].flatten(1)
            n64 = v64.norm(dim=1)
            eg = (st["gpu"][i].flatten(1) - v64).norm(dim=1)
            e32 = (st["f32"][i].flatten(1) - v64).norm(dim=1)
            bound = factor * e32 + FLOOR * n64
            metric = gpu["hist_" + k][t].double().cpu().reshape(B)
            sg = (metric - n64).abs()
            canc = st["f64"][2].flatten(1).norm(dim=1) / n64.clamp_min(1e-30) if k == "primal" else None
            note(k + " vector", eg / bound, t, canc)
            note(k + " metric", sg / bound, t, canc)
            if bool((eg > bound).any()):
                fails.append((tag, t, k + " vector", eg.tolist(), bound.tolist()))
            if bool((sg > bound).any()):
                fails.append((tag, t, k + " metric", sg.tolist(), bound.tolist()))
            line.append(f"r_{k[0]} {float(eg.max()):.1e}/{float(e32.max()):.1e} metric {float((sg / bound).max()):.2f}")
        if verbose and (t < 3 or t % 10 == 9 or t == T - 1):
            print(f"[k100 {tag} it {t:3d}] gpu/f32 dist to f64: " + " | ".join(line))
    summary = ", ".join(
        f"{k} {v[0]:.2f} @it{v[1]} inst{v[2]}" + (f" (|A0x|/|r_p| {v[3]:.1f})" if v[3] is not None else "")
        for k, v in worst.items())
    print(f"[k100 {tag} worst distance/bound] {summary}")
    return fails, worst
