"""Stage-II error attribution (VERDICT r03 "next" item 1, second step): which piece of the GPU
Stage-II iteration moves the dual residual away from the fp64 trajectory.

From one Stage-I end state (as tools/stage2_diag.py), ITERS Stage-II iterations are run with every
combination of factor in {hip, mkl}, solve in {hip, mkl}, rhs+update in {hip, oracle} (all fp32),
plus the fp64 oracle.  Per iteration and combination: the dual and primal residuals of the state
evaluated in fp64 minus the fp64 trajectory's, per instance, and the dual's first-order split
into the x and y contributions (u . Q dx and u . A0^T dy, u = the fp64 dual direction).

  python tools/stage2_blame.py --n 5000 --hidden 2048 --length 200 --batch 3 --iters 5
"""
import argparse
import itertools
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=5000)
    ap.add_argument("--hidden", type=int, default=2048)
    ap.add_argument("--length", type=int, default=200)
    ap.add_argument("--T", type=int, default=2)
    ap.add_argument("--batch", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    from iadmm import data, ops, solver
    from oracle import iadmm_oracle as orc
    n, B = args.n, args.batch
    mi = me = n // 2
    m = mi + me
    N = n + m
    sigma = 6e-6
    d = data.make_qp_batch(n, mi, me, B, first_index=0, device="cuda")
    cpu = {k: v.cpu() for k, v in d.items()}
    params = data.init_lstm_params(args.hidden, args.length, device="cuda")
    with torch.no_grad():
        out = solver.solve(params, d["Q"].clone(), d["p"].clone(), d["A0"].clone(), d["zl"].clone(), d["zu"].clone(),
                           mi, me, args.T, sigma, keep_unscaled=False)
    rho_vec, _ = orc.schedule({k: v.cpu() for k, v in params.items()}, args.T - 1, torch.zeros(B, m, 1), mi, me)
    st0 = {"x": out["x"].cpu().reshape(B, n, 1), "y": out["y"].cpu().reshape(B, m, 1),
           "z": out["z"].cpu().reshape(B, m, 1)}
    del out
    torch.cuda.empty_cache()
    torch.set_num_threads(1)
    rho_rows = rho_vec.reshape(B, m).contiguous()

    # factors
    K32 = orc.kkt_matrix(cpu["Q"], cpu["A0"], sigma, rho_vec)
    Kg = ops.kkt_assemble(d["Q"], d["A0"], sigma, None, 0, rho_rows=rho_rows.cuda())
    asm_diff = float((Kg.cpu() - K32).abs().max())
    LUg, pivg, _ = ops.lu_factor(Kg)
    LUm, pivm = torch.linalg.lu_factor(K32)
    fac = {"hip": (LUg, pivg), "mkl": (LUm, pivm)}
    dev_fac = {"hip": (LUg, pivg), "mkl": (LUm.cuda().contiguous(), pivm.cuda().int().contiguous())}
    cpu_fac = {"hip": (LUg.cpu().contiguous(), pivg.cpu()), "mkl": (LUm, pivm)}
    K64 = orc.kkt_matrix(cpu["Q"].double(), cpu["A0"].double(), sigma, rho_vec.double())
    LU64, piv64 = torch.linalg.lu_factor(K64)
    scal = solver.fixed_alpha_scal(1.6, "cuda")

    def solve(fk, sk, b):  # b [B,N] fp32 cpu -> xv [B,N,1] cpu
        if sk == "hip":
            LU, piv = dev_fac[fk]
            return ops.lu_solve(LU, piv, b.cuda().contiguous()).cpu().reshape(B, N, 1)
        LU, piv = cpu_fac[fk]
        return torch.linalg.lu_solve(LU, piv, b.reshape(B, N, 1))

    def step(st, fk, sk, uk):
        x, y, z = st["x"], st["y"], st["z"]
        if uk == "hip":
            b = ops.kkt_rhs(d["p"].reshape(B, n), x.cuda().reshape(B, n), y.cuda().reshape(B, m), z.cuda().reshape(B, m),
                            sigma, rho_rows=rho_rows.cuda()).cpu()
        else:
            b = orc.kkt_rhs(x, z, y, cpu["p"], sigma, rho_vec).reshape(B, N)
        xv = solve(fk, sk, b)
        if uk == "hip":
            _, xo, yo, zo = ops.admm_update(n, m, 0, None, None, xv.cuda().reshape(B, N), x.cuda().reshape(B, n),
                                            y.cuda().reshape(B, m), z.cuda().reshape(B, m), d["zl"].reshape(B, m),
                                            d["zu"].reshape(B, m), scal, relax_z=True, rho_rows=rho_rows.cuda())
            return {"x": xo.cpu().reshape(B, n, 1), "y": yo.cpu().reshape(B, m, 1), "z": zo.cpu().reshape(B, m, 1)}
        xo, yo, zo = orc.admm_relax_project(xv, x, y, z, cpu["zl"], cpu["zu"], rho_vec, 1.6, relax_z=True)
        return {"x": xo, "y": yo, "z": zo}

    # fp64 trajectory
    ref = []
    st = {k: v.double() for k, v in st0.items()}
    d64 = {k: v.double() for k, v in cpu.items()}
    for _ in range(args.iters):
        b = orc.kkt_rhs(st["x"], st["z"], st["y"], d64["p"], sigma, rho_vec.double())
        xv = torch.linalg.lu_solve(LU64, piv64, b)
        xo, yo, zo = orc.admm_relax_project(xv, st["x"], st["y"], st["z"], d64["zl"], d64["zu"], rho_vec.double(), 1.6,
                                            relax_z=True)
        st = {"x": xo, "y": yo, "z": zo}
        ref.append(st)

    Qd, pd, Ad = (cpu[k].double().cuda() for k in ("Q", "p", "A0"))

    def resid(s):
        x, y, z = (s[k].double().cuda() for k in ("x", "y", "z"))
        rd = Qd @ x + pd + Ad.transpose(1, 2) @ y
        rp = Ad @ x - z
        return rd, rp

    combos = list(itertools.product(("hip", "mkl"), ("hip", "mkl"), ("hip", "oracle")))
    trajs = {}
    for c in combos:
        st = dict(st0)
        tr = []
        for _ in range(args.iters):
            st = step(st, *c)
            tr.append(st)
        trajs["+".join(c)] = tr
    print(json.dumps({"N": N, "B": B, "assemble_maxabs_diff_vs_oracle_K": asm_diff}), flush=True)
    for it in range(args.iters):
        rd64, rp64 = resid(ref[it])
        u = rd64 / rd64.norm(dim=(1, 2), keepdim=True)
        rec = {"it": it, "dual64": rd64.norm(dim=(1, 2)).cpu().tolist()}
        for name, tr in trajs.items():
            s = tr[it]
            rd, rp = resid(s)
            dx = s["x"].double().cuda() - ref[it]["x"].cuda()
            dy = s["y"].double().cuda() - ref[it]["y"].cuda()
            cx = (u * (Qd @ dx)).sum(dim=(1, 2))
            cy = (u * (Ad.transpose(1, 2) @ dy)).sum(dim=(1, 2))
            rec[name] = {"d_dual": (rd.norm(dim=(1, 2)) - rd64.norm(dim=(1, 2))).cpu().tolist(),
                         "d_primal": (rp.norm(dim=(1, 2)) - rp64.norm(dim=(1, 2))).cpu().tolist(),
                         "from_x": cx.cpu().tolist(), "from_y": cy.cpu().tolist(),
                         "x_rel": ((dx.norm(dim=(1, 2)) / ref[it]["x"].cuda().norm(dim=(1, 2)))).cpu().tolist(),
                         "y_rel": ((dy.norm(dim=(1, 2)) / ref[it]["y"].cuda().norm(dim=(1, 2)))).cpu().tolist()}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
