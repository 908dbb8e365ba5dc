"""Instance loader/writer throughput (iadmm/dataset.py) on the host: write
and read B reference-layout gz-pickle files of the bench shape with 1 and with W worker threads.

  python tools/loaderbench.py [--batch 32] [--workers 8] [--dir /tmp/loaderbench]

Prints one JSON line per (operation, workers): seconds, instances/s, decompressed MB/s."""
import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))
import torch  # noqa: E402
from iadmm import data, dataset  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--num_var", type=int, default=1000)
    ap.add_argument("--num_ineq", type=int, default=500)
    ap.add_argument("--num_eq", type=int, default=500)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--dir", default="/tmp/loaderbench")
    a = ap.parse_args()
    B, n, mi, me = a.batch, a.num_var, a.num_ineq, a.num_eq
    d = data.make_qp_batch(n, mi, me, B, first_index=0, device="cpu")
    # decompressed fp64 bytes per instance: Q, A0, G+A (= A0 again), p, zl, zu, c, b
    mb = (n * n + 2 * (mi + me) * n + n + 4 * (mi + me)) * 8 / 1e6
    ref = None
    for w in (1, a.workers):
        out = os.path.join(a.dir, f"w{w}")
        shutil.rmtree(out, ignore_errors=True)
        t0 = time.perf_counter()
        dataset.write_qp(out, d, mi, workers=w)
        tw = time.perf_counter() - t0
        t0 = time.perf_counter()
        r = dataset.read_qp(out, list(range(B)), "cpu", workers=w)
        tr = time.perf_counter() - t0
        if ref is None:
            ref = r
        same = all(torch.equal(r[k], ref[k]) for k in ref)
        for op, t in (("write", tw), ("read", tr)):
            print(json.dumps({"op": op, "workers": w, "batch": B, "n": n, "m": mi + me, "s": round(t, 3),
                              "instances_per_s": round(B / t, 2), "MB_per_s": round(B * mb / t, 1),
                              "equal_to_workers_1": same}), flush=True)
        shutil.rmtree(out, ignore_errors=True)


if __name__ == "__main__":
    main()
