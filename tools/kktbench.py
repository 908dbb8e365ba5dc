"""Residual-matvec (iadmm_kkt_resgrad) bandwidth sweep over batch sizes and instance shapes.

  python tools/kktbench.py [--shapes B,n,mi,me ...]

Times 10 calls per shape with hipEvents on the current stream and prints the algorithmic GB/s
(2 reads of Q and A0 + the vectors) and the fraction of the 8 TB/s spec.  The
default sweep covers the training micro-batch (B = 128), the bench batch (1024), a single instance
and the config-4 shape.  Run it under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))
import torch  # noqa: E402
from iadmm import ops  # noqa: E402

HBM_PEAK_GBS = 8000.0


def run(B, n, mi, me, iters=10):
    m = mi + me
    N = n + m
    torch.manual_seed(0)
    Q = torch.randn(B, n, n, device="cuda")
    A0 = torch.randn(B, m, n, device="cuda")
    p, x = torch.randn(B, n, device="cuda"), torch.randn(B, n, device="cuda")
    y, z = torch.randn(B, m, device="cuda"), torch.randn(B, m, device="cuda")
    xv = torch.randn(B, N, device="cuda")
    scal = ops.schedule(torch.zeros(4, 1, device="cuda"), torch.zeros(4, 1, device="cuda"), 0)
    g = torch.empty(B, N, device="cuda")
    ws = ops.kkt_resgrad_ws(B, n, m, "cuda")

    def call():
        ops.kkt_resgrad(Q, A0, p, x, y, z, xv, 6e-6, scal, mi, g=g, ws=ws)

    call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    byts = B * (2.0 * (n * n + m * n) * 4 + 10.0 * N * 4)
    del Q, A0
    torch.cuda.empty_cache()
    return ms, byts / ms / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="*", default=["1,1000,500,500", "16,1000,500,500", "128,1000,500,500",
                                                    "256,1000,500,500", "1024,1000,500,500",
                                                    "512,5000,2500,2500"])
    a = ap.parse_args()
    for sh in a.shapes:
        B, n, mi, me = (int(v) for v in sh.split(","))
        ms, gbs = run(B, n, mi, me)
        print(json.dumps({"B": B, "n": n, "m": mi + me, "ms": ms, "GBps": gbs, "frac_of_8TBps": gbs / HBM_PEAK_GBS}),
              flush=True)


if __name__ == "__main__":
    main()
