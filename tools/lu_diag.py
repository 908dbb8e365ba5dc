"""Stage-II LU diagnosis on the real KKT matrix (VERDICT r03 "next" item 1).

For the config-2 (N = 2000) and config-4 (N = 10000) KKT shapes (K assembled on the device from
the generator's instances, rho_in = 0.5, rho_eq = 500 as at the Stage-I end state, sigma = 6e-6):
factor K with the HIP LU (iadmm_lu_factor), with single-threaded MKL sgetrf and with MKL dgetrf,
and print per factorisation

  * the factorisation's backward error ||P L U - K||_F / ||K||_F (fp64 on the device),
  * the growth factor max|U| / max|K| and the largest |L11^-1| over the 128-column blocks,
  * the first pivot where it departs from sgetrf,

and per solve (b = K x_t for a random fp64 x_t, rounded to fp32)

  * the normwise backward error ||b - K x||_inf / (||K||_inf ||x||_inf + ||b||_inf),
  * the forward error ||x - x64|| / ||x64|| against the dgetrf/dgetrs solution,

for: HIP factor + HIP solve, MKL sgetrf + sgetrs, HIP factor + fp64 getrs (the factor's share),
MKL factors + HIP solve (the solve kernel's share).  One JSON line per (N, instance).

  python tools/lu_diag.py --N 2000 10000 --batch 2
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))


def unpack(LU, piv):
    """(P, L, U) in fp64 on the device from LAPACK-style factors (1-based int32 pivots)."""
    P, L, U = torch.lu_unpack(LU.double().cuda(), piv.cuda().int())
    return P, L, U


def factor_stats(K, LU, piv, ref_piv):
    P, L, U = unpack(LU, piv)
    R = P @ (L @ U) - K
    N = K.shape[0]
    # where the residual sits: the U12 rows right of each 128-column block (rows [P, P + 128),
    # columns >= P + 128: U12 = L11^-1 A12 in the HIP flow), the rest of U, and L
    ii = torch.arange(N, device=K.device)
    blk = (ii // 128) * 128
    u12 = (ii.unsqueeze(1) < N) & (ii.unsqueeze(0) >= (blk + 128).unsqueeze(1))
    upper = ii.unsqueeze(0) >= ii.unsqueeze(1)
    parts = {"R_U12": float(R[u12].norm() / K.norm()), "R_Udiag": float(R[upper & ~u12].norm() / K.norm()),
             "R_L": float(R[~upper].norm() / K.norm())}
    out = {"factor_berr": float(R.norm() / K.norm()), **parts,
           "factor_berr_max": float(R.abs().max() / K.abs().max()),
           "growth": float(U.abs().max() / K.abs().max())}
    linv = 0.0
    for P0 in range(0, N, 128):
        e = min(N, P0 + 128)
        L11 = L[P0:e, P0:e]
        I = torch.eye(e - P0, dtype=L11.dtype, device=L11.device)
        Li = torch.linalg.solve_triangular(L11, I, upper=False, unitriangular=True)
        linv = max(linv, float(Li.abs().max()))
    out["max_abs_L11inv"] = linv
    d = (piv.cpu() != ref_piv.cpu()).nonzero()
    out["first_piv_diff"] = int(d[0]) if len(d) else -1
    return out


def solve_stats(K, b, x, x64):
    x = x.double().reshape(-1).cuda()
    r = b - K @ x
    berr = float(r.abs().max() / (K.abs().sum(1).max() * x.abs().max() + b.abs().max()))
    ferr = float((x - x64).norm() / x64.norm())
    return {"berr": berr, "ferr": ferr}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, nargs="+", default=[2000, 10000])
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--rho", type=float, default=0.5)
    args = ap.parse_args()
    from iadmm import data, ops
    torch.set_num_threads(1)  # multi-threaded MKL ?LASWP hangs on some KKT matrices in this build
    for N in args.N:
        n = N // 2
        mi = me = n // 2
        B = args.batch
        d = data.make_qp_batch(n, mi, me, B, device="cuda")
        rho = torch.full((B, mi + me), args.rho, device="cuda")
        rho[:, mi:] = 1e3 * args.rho
        K32 = ops.kkt_assemble(d["Q"], d["A0"], 6e-6, None, 0, rho_rows=rho)
        Kc = K32.cpu()
        LUg, pivg, info = ops.lu_factor(K32.clone())
        torch.cuda.synchronize()
        g = torch.Generator().manual_seed(5)
        for i in range(B):
            Kd = Kc[i].double().cuda()
            LUc, pivc = torch.linalg.lu_factor(Kc[i])
            LUd, pivd = torch.linalg.lu_factor(Kc[i].double())
            xt = torch.randn(N, dtype=torch.float64, generator=g)
            b32 = (Kc[i].double() @ xt).float()
            bd = b32.double().cuda()
            x64 = torch.linalg.lu_solve(LUd, pivd, b32.double().unsqueeze(-1)).reshape(-1).cuda()
            rec = {"N": N, "instance": i, "info": int(info[i]),
                   "K_inf": float(Kd.abs().sum(1).max()), "K_maxabs": float(Kd.abs().max())}
            rec["hip_factor"] = factor_stats(Kd, LUg[i], pivg[i], pivc)
            rec["mkl_sgetrf"] = factor_stats(Kd, LUc, pivc, pivc)
            rec["mkl_dgetrf"] = factor_stats(Kd, LUd, pivd, pivc)
            xs = {
                "hip_factor+hip_solve": ops.lu_solve(LUg[i:i + 1], pivg[i:i + 1], b32.cuda().reshape(1, N)),
                "mkl_sgetrf+sgetrs": torch.linalg.lu_solve(LUc, pivc, b32.unsqueeze(-1)),
                "hip_factor+fp64_getrs": torch.linalg.lu_solve(LUg[i].double().cpu(), pivg[i].cpu(),
                                                               b32.double().unsqueeze(-1)),
                "mkl_sgetrf+fp64_getrs": torch.linalg.lu_solve(LUc.double(), pivc, b32.double().unsqueeze(-1)),
                "mkl_factors+hip_solve": ops.lu_solve(LUc.cuda().unsqueeze(0).contiguous(), pivc.cuda().reshape(1, N).int(),
                                                      b32.cuda().reshape(1, N)),
                "mkl_dgetrf+dgetrs": x64,
            }
            rec["solves"] = {k: solve_stats(Kd, bd, v, x64) for k, v in xs.items()}
            rec["x64_vs_xt"] = float((x64.cpu() - xt).norm() / xt.norm())
            print(json.dumps(rec), flush=True)
            del Kd, LUc, LUd
        del K32, LUg, Kc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
