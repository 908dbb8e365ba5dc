"""A/B of the optional f16x3 cell (iadmm_lstm_cell_fwd_f16x3) between library builds at the bench
shape (M = 1024 x 2000 rows, h = 800): hipEvent time per launch, the fp32-equivalent TF/s of the
gate GEMM (8 M h^2), and the rel-L2 of H' / C' against the fp32 kernel's on the same inputs.

  python tools/f16x3_ab.py --libs variants/f16x3_old.so i-admm-lstm_amd/iadmm/libiadmm.so
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))
    import torch
    from iadmm import data, ops, solver
    h, M = a.h, a.rows
    g = torch.Generator(device="cuda").manual_seed(3)
    p = data.init_lstm_params(h, 100, device="cuda")
    H = torch.tanh(torch.randn(M, h, device="cuda", generator=g))
    C = torch.randn(M, h, device="cuda", generator=g)
    xv, gg = (torch.randn(M, device="cuda", generator=g) for _ in range(2))
    packed = solver.PackedWeights()
    Upk, Wx = packed.get(p, h)
    Hf, Cf, _ = ops.lstm_cell(H, C, xv, gg, Upk, Wx)
    Upk16, ws, Wx = packed.get_f16x3(p, h)
    H16 = ops.split_f16(H)
    Hn = torch.empty(M, h, device="cuda")
    ts = []
    for r in range(a.reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        Hn16, Cs, parts, _ = ops.lstm_cell_f16x3(H16, C, xv, gg, Upk16, ws, Wx, Hn=Hn)
        e1.record()
        torch.cuda.synchronize()
        if r:
            ts.append(e0.elapsed_time(e1))
    ms = min(ts)
    rel = lambda x, y: float((x.double() - y.double()).norm() / y.double().norm())  # noqa: E731
    print(json.dumps({"lib": os.environ.get("IADMM_LIB_PATH", "default"), "ms": ts, "best_ms": ms,
                      "tflops_f32_equiv": 8.0 * M * h * h / ms / 1e9, "H_vs_fp32": rel(Hn, Hf),
                      "C_vs_fp32": rel(Cs, Cf)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--rows", type=int, default=1024 * 2000)
    ap.add_argument("--h", type=int, default=800)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a)
    for _ in range(2):  # interleaved rounds
        for lib in a.libs:
            env = dict(os.environ, IADMM_LIB_PATH=os.path.abspath(lib))
            rc = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--libs", lib, "--rows",
                                 str(a.rows), "--h", str(a.h), "--reps", str(a.reps)], env=env, timeout=300).returncode
            if rc:
                print(json.dumps({"lib": lib, "rc": rc}), flush=True)


if __name__ == "__main__":
    main()
