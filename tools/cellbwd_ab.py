"""A/B of the LSTM cell backward kernel (iadmm_lstm_cell_bwd) between library builds at the
config-5 micro-batch shape (M = 128 x 2000 rows, h = 800): hipEvent time per launch, TF/s of the
recompute GEMM (8 M h^2), and a bitwise comparison of the outputs across builds.

  python tools/cellbwd_ab.py --libs i-admm-lstm_amd/iadmm/libiadmm.so variants/cellbwd_old.so
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
    from iadmm import data, ops
    h, M = a.h, a.rows
    g = torch.Generator(device="cuda").manual_seed(3)
    p = data.init_lstm_params(h, 100, device="cuda")
    for k in p:
        if k.startswith(("U_", "W_")):
            p[k] = p[k] * 20
    H = torch.tanh(torch.randn(M, h, device="cuda", generator=g))
    C = torch.randn(M, h, device="cuda", generator=g)
    xv, gg, dq = (torch.randn(M, device="cuda", generator=g) for _ in range(3))
    dH, dC = torch.randn(M, h, device="cuda", generator=g), torch.randn(M, h, device="cuda", generator=g)
    Upk, Wx = ops.lstm_pack(p, h)
    ts = []
    for r in range(a.reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = ops.lstm_cell_bwd(H, C, xv, gg, Upk, Wx, dq, dH, dC)
        e1.record()
        torch.cuda.synchronize()
        if r:
            ts.append(e0.elapsed_time(e1))
    ms = min(ts)
    dig = [float(t.double().sum()) for t in out]
    print(json.dumps({"lib": os.environ.get("IADMM_LIB_PATH", "default"), "ms": ts, "best_ms": ms,
                      "tflops": 8.0 * M * h * h / ms / 1e9, "checksums": dig}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--rows", type=int, default=128 * 2000)
    ap.add_argument("--h", type=int, default=800)
    ap.add_argument("--reps", type=int, default=10)
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
                return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
