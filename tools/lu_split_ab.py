"""Experiment (r05): the batched LU at B = 1024, N = 2000 as one call on one stream against the batch split
into k equal parts factored concurrently on k streams (no data is shared between instances).  Prints the
best of a few reps for each, and whether the factors are bitwise the same.
Parts 0 is the library's own split (iadmm_lu_factor_ex with a context, r05).
    python tools/lu_split_ab.py [--parts 2 4] [--reps 4]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "i-admm-lstm_amd"))
import torch  # noqa: E402
from iadmm import data, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--N", type=int, default=2000)
ap.add_argument("--parts", type=int, nargs="+", default=[2, 4])
ap.add_argument("--reps", type=int, default=4)
a = ap.parse_args()
B, N = a.batch, a.N
n = N // 2
mi = me = n // 2
d = data.make_qp_batch(n, mi, me, B, device="cuda")
rho = torch.full((B, mi + me), 0.5, device="cuda")
rho[:, mi:] = 500.0
K0 = ops.kkt_assemble(d["Q"], d["A0"], 6e-6, None, 0, rho_rows=rho)
del d
K = torch.empty_like(K0)


def run(parts):
    K.copy_(K0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream()
    e0.record()
    if parts in (0, 1):  # 1: one stream (no context); 0: the library's own split (context, B >= 512)
        LU, piv, info = ops.lu_factor(K, ws=ws[1][0], lookahead=parts == 0)
        outs = [(piv, info)]
    else:
        outs = []
        step = B // parts
        for i in range(parts):
            s = streams[i]
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                outs.append(ops.lu_factor(K[i * step:(i + 1) * step], ws=ws[parts][i], lookahead=False)[1:])
        for s in streams[:parts]:
            cur.wait_stream(s)
    e1.record()
    torch.cuda.synchronize()
    piv = torch.cat([o[0] for o in outs])
    fp = int(torch.sum(K.view(torch.int32).flatten(1), dim=1, dtype=torch.int64).sum())
    return e0.elapsed_time(e1), fp, int(piv.sum(dtype=torch.int64))


streams = [torch.cuda.Stream() for _ in range(max(a.parts))]
ws = {p: [ops.lu_factor_ws(B // p, N, "cuda") for _ in range(p)] for p in [1] + a.parts}
res = {}
for p in [1, 0] + a.parts:
    run(p)
    ts = []
    for _ in range(a.reps):
        t, fp, ps = run(p)
        ts.append(t)
    res[p] = (min(ts), fp, ps)
    print(f"parts {p}: best {min(ts):.2f} ms (reps {', '.join(f'{t:.2f}' for t in ts)}), fingerprint {fp} piv {ps}", flush=True)
print("bitwise equal to one call:", {p: res[p][1:] == res[1][1:] for p in [0] + a.parts}, "(parts 0 = the library's split)")
