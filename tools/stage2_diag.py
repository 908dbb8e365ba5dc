"""Stage-II trajectory diagnosis (VERDICT r03 "next" item 1): where the GPU's distance to the fp64
trajectory comes from.

From one Stage-I end state (the GPU's T-iteration solve, unscaled x, y, z, xv and the scaled
rho_vec, copied to the host so every path starts from identical inputs), ITERS exact Stage-II
iterations (models/lu.py) run three ways: the drop-in LU module on the GPU, oracle.lu_iteration in
fp32 (MKL sgetrf/sgetrs, one thread) and in fp64.  Per iteration and trajectory it prints

  * the distances of x, y, z, xv to the fp64 trajectory (rel-L2 per instance, max over the batch),
  * the dual residual ||Q x + p + A0^T y|| of the trajectory's state evaluated three ways: the
    GPU metric kernel (fp32), the oracle's fp32 expression (MKL), fp64 -- so the metric's own
    rounding is separated from the state's,
  * the KKT solve residual ||K xv - b~|| / (||K|| ||xv||) of the iteration, in fp64.

  python tools/stage2_diag.py --n 5000 --hidden 2048 --length 200 --batch 1 --iters 5
"""
import argparse
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
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    from iadmm import data, ops, solver
    from models.lu import LU
    from oracle import iadmm_oracle as orc
    n, B = args.n, args.batch
    mi = me = n // 2
    m = mi + me
    sigma = 6e-6
    d = data.make_qp_batch(n, mi, me, B, first_index=0, device="cuda")
    cpu = {k: v.cpu() for k, v in d.items()}
    params = data.init_lstm_params(args.hidden, args.length, device="cuda")
    with torch.no_grad():
        out = solver.solve(params, d["Q"].clone(), d["p"].clone(), d["A0"].clone(), d["zl"].clone(), d["zu"].clone(),
                           mi, me, args.T, sigma, keep_unscaled=False)
    rho_vec, _ = orc.schedule({k: v.cpu() for k, v in params.items()}, args.T - 1, torch.zeros(B, m, 1), mi, me)
    st0 = {"x": out["x"].cpu().reshape(B, n, 1), "y": out["y"].cpu().reshape(B, m, 1),
           "z": out["z"].cpu().reshape(B, m, 1), "xv": out["xv"].cpu().reshape(B, n + m, 1), "rho_vec": rho_vec}
    del out
    torch.set_num_threads(1)

    def oracle_run(dtype):
        st = {k: v.to(dtype) for k, v in st0.items()}
        dd = {k: v.to(dtype) for k, v in cpu.items()}
        K = lu = piv = None
        traj = []
        for _ in range(args.iters):
            b = orc.kkt_rhs(st["x"], st["z"], st["y"], dd["p"], sigma, st["rho_vec"])
            x, y, z, xv, K, _, lu, piv = orc.lu_iteration(st["rho_vec"], st["x"], st["y"], st["z"], st["xv"], sigma,
                                                          K, lu, piv, dd["Q"], dd["p"], dd["A0"], dd["zl"], dd["zu"])
            st.update(x=x, y=y, z=z, xv=xv)
            traj.append(dict(x=x, y=y, z=z, xv=xv, b=b))
        return traj

    r32, r64 = oracle_run(torch.float32), oracle_run(torch.float64)
    g = {k: v.cuda() for k, v in st0.items()}
    x, y, z, xv = g["x"], g["y"], g["z"], g["xv"]
    model = LU("cuda")
    A_t = lu = piv = None
    gpu = []
    with torch.no_grad():
        for _ in range(args.iters):
            x, y, z, xv, A_t, b, lu, piv = model(g["rho_vec"], x, y, z, xv, sigma, A_t, lu, piv, Q=d["Q"], p=d["p"],
                                                 A0=d["A0"], lb=None, ub=None, zl=d["zl"], zu=d["zu"])
            gpu.append({k: v.cpu() for k, v in dict(x=x, y=y, z=z, xv=xv, b=b).items()})
    del lu, A_t
    torch.cuda.empty_cache()
    Kd = orc.kkt_matrix(cpu["Q"].double(), cpu["A0"].double(), sigma, st0["rho_vec"].double()).cuda()
    Qd, pd, Ad = cpu["Q"].double().cuda(), cpu["p"].double().cuda(), cpu["A0"].double().cuda()

    def rel(a, b):
        a = a.double().reshape(B, -1)
        b = b.double().reshape(B, -1)
        return float(((a - b).norm(dim=1) / b.norm(dim=1).clamp_min(1e-30)).max())

    def duals(st):
        xs, ys, zs = (st[k].float().reshape(B, -1, 1) for k in ("x", "y", "z"))
        _, _, du_gpu = ops.metrics(d["Q"], d["p"].reshape(B, n), d["A0"], xs.cuda().reshape(B, n), ys.cuda().reshape(B, m),
                                   zs.cuda().reshape(B, m))
        _, du32, _ = orc.primal_dual(xs, ys, zs, cpu["Q"], cpu["p"], cpu["A0"])
        xd, yd = st["x"].double().cuda().reshape(B, n, 1), st["y"].double().cuda().reshape(B, m, 1)
        du64 = (Qd @ xd + pd + Ad.transpose(1, 2) @ yd).norm(dim=(1, 2))
        return du_gpu.cpu().reshape(-1).double(), du32.reshape(-1).double(), du64.cpu().reshape(-1)

    def kkt_res(st):
        xvd = st["xv"].double().cuda().reshape(B, -1, 1)
        bd = st["b"].double().cuda().reshape(B, -1, 1)
        r = Kd @ xvd - bd
        return float((r.norm(dim=(1, 2)) / (Kd.flatten(1).norm(dim=1) * xvd.norm(dim=(1, 2)))).max())

    for it in range(args.iters):
        rec = {"N": n + m, "it": it}
        for name, tr in (("gpu", gpu), ("f32", r32), ("f64", r64)):
            st = tr[it]
            e = {k: rel(st[k], r64[it][k]) for k in ("x", "y", "z", "xv")}
            dg, d32, d64 = duals(st)
            e["dual_by_gpu_metric"] = dg.tolist()
            e["dual_by_f32_metric"] = d32.tolist()
            e["dual_by_f64_metric"] = d64.tolist()
            e["kkt_res"] = kkt_res(st)
            rec[name] = e
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
