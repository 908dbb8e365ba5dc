"""A/B of the batched LU factorization (csrc/lu.hip) between library builds, on the GPU box.

For each library (IADMM_LIB_PATH) in a child process: factor a batch of KKT matrices at the given
shape a few times and one solve five times (hipEvents), and check the backward error of one solve against fp64.  Prints one
JSON line per library.

  python tools/lu_ab.py --libs i-admm-lstm_amd/iadmm/libiadmm.so variants/lu64.so --batch 1024 --N 2000
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(args):
    sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))
    import torch
    from iadmm import _abi, data, ops
    if getattr(_abi.lib(), "iadmm_lu_factor_ex", None) is None:  # an r04-ABI build (A/B against it)
        def lu_factor(K, ws=None, **_):
            B, N = K.shape[0], K.shape[1]
            piv = torch.empty(B, N, dtype=torch.int32, device=K.device)
            info = torch.empty(B, dtype=torch.int32, device=K.device)
            _abi.call("iadmm_lu_factor", B, N, K.data_ptr(), piv.data_ptr(), info.data_ptr(), ws.data_ptr(),
                      ws.numel() * 4, torch.cuda.current_stream().cuda_stream)
            return K, piv, info

        def lu_solve(LU, piv, b, **_):
            x = b.clone()
            _abi.call("iadmm_lu_solve", LU.shape[0], LU.shape[1], LU.data_ptr(), piv.data_ptr(), x.data_ptr(),
                      torch.cuda.current_stream().cuda_stream)
            return x
        ops.lu_factor, ops.lu_solve = lu_factor, lu_solve
    n = args.N // 2
    mi = me = n // 2
    B = args.batch
    d = data.make_qp_batch(n, mi, me, B, device="cuda")
    rho = torch.full((B, mi + me), 0.5, device="cuda")
    rho[:, mi:] = 500.0
    ws = ops.lu_factor_ws(B, args.N, "cuda")
    times = []
    for r in range(args.reps + 1):
        K = ops.kkt_assemble(d["Q"], d["A0"], 6e-6, None, 0, rho_rows=rho)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        LU, piv, info = ops.lu_factor(K, ws=ws, flags=args.flags) if args.flags else ops.lu_factor(K, ws=ws)
        e1.record()
        torch.cuda.synchronize()
        if r:
            times.append(e0.elapsed_time(e1))
        if r < args.reps:
            del K, LU
    g = torch.Generator(device="cuda").manual_seed(1)
    b = torch.randn(B, args.N, device="cuda", generator=g)
    x = ops.lu_solve(LU, piv, b)
    solve_ms = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.lu_solve(LU, piv, b)
        e1.record()
        torch.cuda.synchronize()
        solve_ms.append(e0.elapsed_time(e1))
    K = ops.kkt_assemble(d["Q"][:4], d["A0"][:4], 6e-6, None, 0, rho_rows=rho[:4].contiguous()).double()
    xd, bd = x[:4].double(), b[:4].double()
    res = torch.bmm(K, xd.unsqueeze(-1)).squeeze(-1) - bd
    berr = (res.norm(dim=1) / (K.flatten(1).norm(dim=1) * xd.norm(dim=1))).max().item()
    N = args.N
    ms = min(times)
    # bitwise fingerprint of the factors (A/B variants that claim the same arithmetic must agree)
    lu_sum = sum(int(torch.sum(LU[i:i + 64].view(torch.int32), dtype=torch.int64)) for i in range(0, B, 64))
    piv_sum = int(torch.sum(piv, dtype=torch.int64))
    print(json.dumps({"lib": os.environ.get("IADMM_LIB_PATH", "default"), "flags": args.flags, "B": B, "N": N, "factor_ms": times,
                      "best_ms": ms, "tflops": B * 2.0 / 3.0 * N ** 3 / ms / 1e9, "frac_fp32_mfma": B * 2.0 / 3.0 * N ** 3 / ms / 1e9 / 157.3,
                      "info_max": int(info.max()), "solve_ms": solve_ms,
                      "solve_tbps": B * args.N * args.N * 4 / min(solve_ms) / 1e9, "backward_error": berr, "piv_head": piv[0, :8].tolist(),
                      "lu_bits_sum": lu_sum, "piv_sum": piv_sum}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", default=[os.path.join(ROOT, "i-admm-lstm_amd", "iadmm", "libiadmm.so")])
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--N", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--flags", type=int, default=0, help="iadmm_lu_factor_ex flags (4 = IADMM_LU_RANK128: the r04 form)")
    args = ap.parse_args()
    if args.child:
        return child(args)
    for lib in args.libs:
        env = dict(os.environ, IADMM_LIB_PATH=os.path.abspath(lib))
        cmd = [sys.executable, os.path.abspath(__file__), "--child", "--batch", str(args.batch), "--N", str(args.N),
               "--reps", str(args.reps), "--flags", str(args.flags)]
        rc = subprocess.run(cmd, env=env, timeout=600).returncode
        if rc != 0:
            print(json.dumps({"lib": lib, "rc": rc}), flush=True)
            return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
