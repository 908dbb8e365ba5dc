"""Train an I-ADMM-LSTM checkpoint for the bench shape with this repo's own HIP training path.

The random-init weights diverge at the bench shape (n=1000, 500+500, h=800, K=100: the primal
residual grows to ~1e4), so the residual half of the BASELINE metric needs trained weights.  The
parameters do not depend on n (models/lstm.py:21-41), but the reference trains on the test shape
(scripts/Synthetic.sh: QP_1000_500_500, outer_T = truncated_length = 100, h = 800), and so does
this script: Ruiz-scaled synthetic instances from a pool disjoint from the bench's (seeds
17 + 100000 + i; the bench uses 17 + 0..B-1), one TBPTT window per step through the HIP
forward/backward kernels (iadmm/train.py, the main.py:336-358 loop), Adam.  Every ``--val_every``
steps a no-grad solve of held-out instances reports the final unscaled primal/dual residual;
the best one (lowest primal + dual) is saved in the reference's .pth format (a state_dict).

  python tools/train_checkpoint.py --minutes 8 --out checkpoints/QP_1000_500_500_100_800.pth
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-admm-lstm_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num_var", type=int, default=1000)
    ap.add_argument("--num_ineq", type=int, default=500)
    ap.add_argument("--num_eq", type=int, default=500)
    ap.add_argument("--hidden_dim", type=int, default=800)
    ap.add_argument("--outer_T", type=int, default=100)
    ap.add_argument("--truncated_length", type=int, default=100)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--pool", type=int, default=128, help="training instances (cycled)")
    ap.add_argument("--val", type=int, default=8)
    ap.add_argument("--val_every", type=int, default=25)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--steps", type=int, default=100000)
    ap.add_argument("--minutes", type=float, default=8.0)
    ap.add_argument("--sigma", type=float, default=6e-6)
    ap.add_argument("--seed", type=int, default=17)
    ap.add_argument("--init", type=str, default="", help="start from this .pth")
    ap.add_argument("--out", type=str, default="checkpoints/QP_1000_500_500_100_800.pth")
    a = ap.parse_args()
    from iadmm import data, ops, solver, train
    from models.lstm import LSTM

    n, mi, me, h, T = a.num_var, a.num_ineq, a.num_eq, a.hidden_dim, a.outer_T
    dev = "cuda"
    t_start = time.time()
    pool = data.make_qp_batch(n, mi, me, a.pool, first_index=100000, seed=a.seed, device=dev)
    Qs, ps, As, zls, zus, _, _, _ = ops.ruiz_scale(pool["Q"], pool["p"], pool["A0"], pool["zl"], pool["zu"], 10)
    del pool
    val = data.make_qp_batch(n, mi, me, a.val, first_index=200000, seed=a.seed, device=dev)
    torch.manual_seed(a.seed)
    model = LSTM(mi + me, 2, h, T, dev)
    if a.init:
        model.load_state_dict(torch.load(a.init, map_location=dev, weights_only=True))
    opt = torch.optim.Adam(model.parameters(), lr=a.lr)
    packed = solver.PackedWeights()

    def validate():
        with torch.no_grad():
            out = solver.solve(model, val["Q"], val["p"], val["A0"], val["zl"], val["zu"], mi, me, T, a.sigma,
                               packed=packed)
            return float(out["primal"].mean()), float(out["dual"].mean())

    pr, du = validate()
    best = pr + du
    print(f"[train] step 0 val primal {pr:.4g} dual {du:.4g} (random init)", flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    torch.save(model.state_dict(), a.out)
    step = 0
    while step < a.steps and time.time() - t_start < 60 * a.minutes:
        s = (step * a.batch) % a.pool
        idx = torch.arange(s, s + a.batch, device=dev) % a.pool
        d = dict(Q=Qs[idx], p=ps[idx], A0=As[idx], zl=zls[idx], zu=zus[idx])
        loss = train.tbptt_batch(model, d, mi, me, T, a.truncated_length, a.sigma, opt)
        step += 1
        if step % 5 == 0:
            print(f"[train] step {step} loss {loss:.5g} ({time.time() - t_start:.0f} s)", flush=True)
        if step % a.val_every == 0:
            pr, du = validate()
            tag = ""
            if pr + du < best and pr == pr and du == du:
                best = pr + du
                torch.save(model.state_dict(), a.out)
                tag = " saved"
            print(f"[train] step {step} val primal {pr:.4g} dual {du:.4g}{tag}", flush=True)
    print(f"[train] done: {step} steps, best val primal+dual {best:.4g} -> {a.out}", flush=True)


if __name__ == "__main__":
    main()
