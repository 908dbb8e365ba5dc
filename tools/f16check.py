"""Diagnostic: NaN / agreement of the optional f16x3 cell against the fp32 path on the bench
instance shape (n=1000, m=500+500, h=800) for a few batch sizes and iteration counts."""
import sys
import torch
sys.path.insert(0, "i-admm-lstm_amd")
sys.path.insert(0, ".")
from iadmm import data, solver  # noqa: E402

n, mi, me, h = 1000, 500, 500, 800
params = data.init_lstm_params(h, 100, device="cuda")
d = data.make_qp_batch(n, mi, me, 1024, device="cuda")
for B, T in ((4, 30), (4, 60), (4, 100), (1024, 100)):
    with torch.no_grad():
        o32 = solver.solve(params, d["Q"][:B], d["p"][:B], d["A0"][:B], d["zl"][:B], d["zu"][:B], mi, me, T, 6e-6,
                           history=True)
    x = o32["x"]
    hist = o32.get("history")
    print(f"B={B} T={T}: nan x32[:4] {int(torch.isnan(x[:4]).sum())} nan all {int(torch.isnan(x).sum())} "
          f"primal[:4] {o32['primal'][:4].flatten().tolist()}", flush=True)
    if hist is not None and B == 4:
        pr = hist["primal"] if isinstance(hist, dict) else None
        if pr is not None:
            print("  primal history (inst 0):", [float(v) for v in pr[::10, 0]], flush=True)
