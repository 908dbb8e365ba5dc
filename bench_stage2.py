"""Stage II benchmark (models/lu.py:13-47 driven by main.py:1035-1066):
assemble K, factor it once (batched blocked LU with partial pivoting), then ``feas_rest_num``
exact ADMM iterations (RHS, two triangular solves, alpha = 1.6 update), at the BASELINE config-2
shape (n = 1000, 500 + 500 rows, N = 2000, B = 1024 per GPU), inputs resident in HBM.

Prints one JSON line: instances/s of the whole Stage II, the factor and per-iteration times,
the LU trailing-update and solve kernels against the HBM roofline (algorithmic bytes: the
rank-64 trailing update reads and writes the trailing matrix once per 64-column block; a solve reads L and U
once), and the CPU reference path (torch.linalg.lu_factor / lu_solve, the oracle) timed on a
bounded sample on the host.

  python bench_stage2.py [--batch 1024] [--iters 20] [--cpu-sample 2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0
LU_BLOCK = 64  # csrc/lu.hip kBlk: rank of the MFMA trailing update


def update_bytes(N, nb=LU_BLOCK):
    """Algorithmic HBM bytes of the rank-64 trailing updates of one N x N factorization:
    A22 read + written, L21 and U12 read, once per 64-column block."""
    tot = 0.0
    for k0 in range(0, N, nb):
        rest = N - k0 - nb
        if rest > 0:
            tot += 4.0 * (2 * rest * rest + 2 * rest * nb)
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--num_var", type=int, default=1000)
    ap.add_argument("--num_ineq", type=int, default=500)
    ap.add_argument("--num_eq", type=int, default=500)
    ap.add_argument("--iters", type=int, default=20, help="feas_rest_num (configs/QP.yaml)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-sample", type=int, default=2)
    ap.add_argument("--chunk", type=int, default=0,
                    help="instances per factorisation chunk (0: solver.stage2_chunk, balanced under the memory cap)")
    args = ap.parse_args()
    from iadmm import data, ops, solver
    n, mi, me, B = args.num_var, args.num_ineq, args.num_eq, args.batch
    m = mi + me
    N = n + m
    torch.cuda.set_device(0)
    d = data.make_qp_batch(n, mi, me, B, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(B, n, device="cuda", generator=g)
    y = torch.randn(B, m, device="cuda", generator=g)
    z = torch.randn(B, m, device="cuda", generator=g)
    rho = torch.full((B, m), 0.5, device="cuda")
    rho[:, mi:] = 500.0
    args_dev = (d["Q"], d["p"].reshape(B, n).contiguous(), d["A0"], d["zl"].reshape(B, m).contiguous(),
                d["zu"].reshape(B, m).contiguous(), rho, x, y, z, 6e-6, args.iters)

    def step(timer):
        return solver.stage2(*args_dev, timer=timer, chunk=args.chunk or None)

    for _ in range(args.warmup):
        out = step(None)
        del out
    torch.cuda.synchronize()
    timer = solver.Timer(True)
    el = 0.0
    for _ in range(args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = step(timer)
        torch.cuda.synchronize()
        el += time.perf_counter() - t0
        info = int(out["info"].abs().sum())
        del out
    spans = {k: v / args.steps for k, v in timer.totals_ms().items()}
    # per-kernel: time the factor's kernels and one solve separately with events, on the first
    # chunk of instances whose dense K fits (all of them at config 2; config 4's 205 GB does not)
    c = solver.stage2_chunk(B, N)
    K = ops.kkt_assemble(d["Q"][:c], d["A0"][:c], 6e-6, None, 0, rho_rows=rho[:c].contiguous())
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    e[0].record()
    LU, piv, _ = ops.lu_factor(K)
    e[1].record()
    b = ops.kkt_rhs(args_dev[1][:c], x[:c], y[:c], z[:c], 6e-6, rho_rows=rho[:c].contiguous())
    e[2].record()
    for _ in range(10):
        ops.lu_solve(LU, piv, b)
    e[3].record()
    torch.cuda.synchronize()
    fac_ms, solve_ms = e[0].elapsed_time(e[1]), e[2].elapsed_time(e[3]) / 10
    upd_bytes = c * update_bytes(N)          # trailing updates, read + write
    solve_bytes = c * (4.0 * N * N + 3 * 4.0 * N)  # L and U once, b in / x out
    res = {
        "metric": f"Stage II (feasibility restoration) QP instances/s at n={n} m={m}, "
                  f"factor once + {args.iters} LU-solve iterations",
        "value": B * args.steps / el, "unit": "QP instances/s", "ms_per_step": 1e3 * el / args.steps,
        "n_gpus": 1, "dtype": "f32", "data": "synthetic (generate_data.py:67-76 distribution), random iterate",
        "config": {"workload": f"Stage II n={n} ineq={mi} eq={me} N={N} batch={B} feas_rest_num={args.iters}"},
        "phase_ms_per_step": spans, "singular_instances": info,
        "factor": {"ms": fac_ms, "instances": c, "chunks_per_step": -(-B // c),
                   "trailing_update_GB": upd_bytes / 1e9,
                   "trailing_update_GBps_over_whole_factor": upd_bytes / fac_ms / 1e6,
                   "note": "a lower bound on the trailing-update kernel's own rate (the factor also runs panels, "
                           "interchanges and U12 solves); per-kernel times: profiles/r01_stage2_kernel_stats.csv",
                   "tflops_equiv": c * (2.0 / 3.0) * N ** 3 / fac_ms / 1e9},
        "roofline_solve": {"kernel": "iadmm_lu_solve", "bound": "hbm", "achieved": solve_bytes / solve_ms / 1e6,
                           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": solve_bytes / solve_ms / 1e6 / HBM_PEAK_GBS,
                           "avg_launch_ms": solve_ms},
    }
    if args.cpu_sample > 0:
        torch.set_num_threads(1)  # multi-threaded MKL getrf hangs on some KKT matrices
        c = min(args.cpu_sample, B)
        del K, LU
        Kc = ops.kkt_assemble(d["Q"][:c], d["A0"][:c], 6e-6, None, 0, rho_rows=rho[:c].contiguous()).cpu()
        bc = b[:c].cpu().unsqueeze(-1)
        t0 = time.perf_counter()
        lu, pv = torch.linalg.lu_factor(Kc)
        t1 = time.perf_counter()
        for _ in range(args.iters):
            torch.linalg.lu_solve(lu, pv, bc)
        t2 = time.perf_counter()
        per = (t1 - t0) / c + (t2 - t1) / c
        res["cpu_baseline"] = {"value": 1.0 / per, "unit": "QP instances/s", "cores": 1, "kind": "port",
                               "sample": f"{c} instances: torch.linalg.lu_factor + {args.iters} lu_solve "
                                         f"(the reference's torch.lu path), factor {1e3 * (t1 - t0) / c:.0f} ms/inst"}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
