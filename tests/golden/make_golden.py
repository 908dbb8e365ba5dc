"""Golden-vector generator for the I-ADMM-LSTM solve loop (run in the survey container only).

Imports the *reference* modules read-only from /root/reference and records their outputs on
small seeded QPs as ``.npz`` fixtures next to this file.  Nothing under /root/reference is copied:
the fixtures are data (inputs + outputs).  Bytecode writing is disabled (the
reference tree must not gain ``.pyc`` files), so run it as::

    PYTHONDONTWRITEBYTECODE=1 python -B tests/golden/make_golden.py

What is restated here (not importable from the reference):
  * the QP branch of the instance generator ``generate_data.py:67-76`` without the OSQP filter
    (OSQP is not installed), with ``pinv(A)`` as in the reference;
  * the Q*2 load quirk ``main.py:718``;
  * the test loop ``main.py:818-1031`` (scale -> K x model(t,...) -> unscale, per-iteration
    metrics on unscaled data ``main.py:892-988``);
  * Stage II ``main.py:1035-1066``;
  * one TBPTT loss/backward ``main.py:336-350`` for parameter-gradient fixtures.
The imported reference pieces are ``models/lstm.py:LSTM``, ``models/lu.py:LU``,
``methods/scaling.py:Scaling`` and ``utils.py:{primal_dual_loss,obj_fn}``.
"""
import os
import sys

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path = [p for p in sys.path if os.path.abspath(p or ".") not in (REPO, HERE)]
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from models.lstm import LSTM  # noqa: E402  (reference)
from models.lu import LU  # noqa: E402  (reference)
from methods.scaling import Scaling  # noqa: E402  (reference)
from utils import primal_dual_loss, obj_fn  # noqa: E402  (reference)

assert os.path.abspath(sys.modules["models.lstm"].__file__).startswith(REF)

# single-threaded: the multi-threaded MKL getrf in this torch build hangs on KKT matrices
# (SLASWP "parameter 6" error at N=400), see DESIGN.md
torch.set_num_threads(1)


def make_qp(seed, n, mi, me, B):
    """generate_data.py:67-76 (QP branch), restated; returns fp64 numpy like the pickles."""
    g = torch.Generator().manual_seed(seed)
    Q0 = 0.5 * torch.diag_embed(torch.rand((B, n), generator=g)).numpy()
    p0 = torch.rand((B, n), generator=g).unsqueeze(-1).numpy()
    A = torch.normal(0.0, 1.0, (B, me, n), generator=g).numpy()
    b = (2 * torch.rand((B, me), generator=g).unsqueeze(-1) - 1).numpy()
    G = torch.normal(0.0, 1.0, (B, mi, n), generator=g).numpy()
    if me > 0:
        c = torch.sum(torch.abs(torch.bmm(torch.tensor(G), torch.pinverse(torch.tensor(A)))), dim=2)
        c = c.unsqueeze(-1).numpy()
    else:  # no equality block: any positive bound works as test data
        c = 0.5 * np.abs(G).sum(axis=2, keepdims=True)
    A0 = np.concatenate([G, A], axis=1)
    zl = np.concatenate([-np.inf * np.ones((B, mi, 1)), b], axis=1)
    zu = np.concatenate([c, b], axis=1)
    # main.py:718-722: fp32 tensors, Q*2
    t = lambda a: torch.tensor(np.array(a), dtype=torch.float32)  # noqa: E731
    return dict(Q=t(Q0) * 2, p=t(p0), A0=t(A0), zl=t(zl), zu=t(zu), G=t(G), c=t(c), A=t(A), b=t(b))


def run_case(name, seed, n, mi, me, h, T, B, wscale=1.0, scaling=True, stage2=0, keep_iters=3,
             keep_state_every=False, grads=False):
    torch.manual_seed(17)
    model = LSTM(mi + me, 2, h, T, "cpu")
    if wscale != 1.0:
        with torch.no_grad():
            for k in ("W_i", "U_i", "W_f", "U_f", "W_o", "U_o", "W_u", "U_u", "W_h"):
                getattr(model, k).mul_(wscale)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    d = make_qp(seed, n, mi, me, B)
    m = mi + me
    sigma = 6e-6
    out = {"meta": np.array([n, mi, me, h, T, B, int(scaling), stage2], dtype=np.int64),
           "sigma": np.float32(sigma), "wscale": np.float32(wscale)}
    for k in ("Q", "p", "A0", "zl", "zu"):
        out["in_" + k] = d[k].numpy()
    for k, v in sd.items():
        out["param_" + k] = v.numpy()

    Q, p, A0, zl, zu = d["Q"], d["p"], d["A0"], d["zl"], d["zu"]
    Qu, pu, A0u, zlu, zuu = Q, p, A0, zl, zu
    if scaling:  # main.py:818-834
        sc = Scaling(n, m, 10, "cpu")
        Q, p, A0, zl, zu = sc.scale_data(Q, p, A0, zl, zu)
        out.update(sc_Q=Q.numpy(), sc_p=p.numpy(), sc_A0=A0.numpy(), sc_zl=zl.numpy(),
                   sc_zu=zu.numpy(), sc_D=torch.diagonal(sc.D, dim1=1, dim2=2).numpy(),
                   sc_E=torch.diagonal(sc.E, dim1=1, dim2=2).numpy(), sc_c=sc.c.reshape(B).numpy())

    with torch.no_grad():
        x = torch.zeros(B, n, 1)
        y = torch.zeros(B, m, 1)
        z = torch.zeros(B, m, 1)
        xv = torch.zeros(B, n + m, 1)
        H = torch.zeros(B, n + m, h)
        C = torch.zeros(B, n + m, h)
        hist = {k: [] for k in ("obj", "ls_res", "primal", "dual")}
        for t in range(T):  # main.py:874-988
            xv_prev = xv
            x, y, z, xv, H, C, Kt, bt, rho_vec = model(t, mi, me, x, y, z, xv, sigma, H, C,
                                                         Q=Q, p=p, A0=A0, lb=None, ub=None, zl=zl, zu=zu)
            if t < keep_iters or keep_state_every:
                g = torch.bmm(Kt.permute(0, 2, 1), torch.bmm(Kt, xv_prev) - bt)  # lstm.py:72
                for k, v in (("x", x), ("y", y), ("z", z), ("xv", xv), ("H", H), ("C", C),
                             ("btild", bt), ("rhovec", rho_vec), ("g", g)):
                    out[f"it{t}_{k}"] = v.numpy().copy()
            # metrics on unscaled data (main.py:892-978)
            if scaling:
                xs, ys, zs = torch.bmm(sc.D, x), torch.bmm(sc.cinv * sc.E, y), torch.bmm(sc.Einv, z)
            else:
                xs, ys, zs = x, y, z
            hist["obj"].append(obj_fn(xs, Q=Qu, p=pu).reshape(B).numpy())
            hist["ls_res"].append(torch.linalg.vector_norm(torch.bmm(Kt, xv) - bt, dim=(1, 2)).numpy())
            pr, dr, _ = primal_dual_loss(xs, ys, zs, Qu, pu, A0u)
            hist["primal"].append(pr.reshape(B).numpy())
            hist["dual"].append(dr.reshape(B).numpy())
        for k, v in hist.items():
            out["hist_" + k] = np.stack(v, 0).astype(np.float32)  # [T, B]
        out.update(fin_x_scaled=x.numpy(), fin_y_scaled=y.numpy(), fin_z_scaled=z.numpy(),
                   fin_xv=xv.numpy(), fin_H=H.numpy(), fin_C=C.numpy(), fin_rhovec=rho_vec.numpy())
        if scaling:  # final unscale main.py:1017-1027
            x, y, z = torch.bmm(sc.D, x), torch.bmm(sc.cinv * sc.E, y), torch.bmm(sc.Einv, z)
        out.update(fin_x=x.numpy(), fin_y=y.numpy(), fin_z=z.numpy())

        if stage2:  # main.py:1035-1066 (Stage II on unscaled data, last scaled rho_vec)
            lu_m = LU("cpu")
            Kt2, lu, piv = None, None, None
            s2 = {k: [] for k in ("x", "y", "z", "xv")}
            for t in range(stage2):
                x, y, z, xv, Kt2, bt2, lu, piv = lu_m(rho_vec, x, y, z, xv, sigma, Kt2, lu, piv,
                                                      Q=Qu, p=pu, A0=A0u, lb=None, ub=None, zl=zlu, zu=zuu)
                for k, v in (("x", x), ("y", y), ("z", z), ("xv", xv)):
                    s2[k].append(v.numpy().copy())
            for k, v in s2.items():
                out["s2_" + k] = np.stack(v, 0)
            pr, dr, _ = primal_dual_loss(x, y, z, Qu, pu, A0u)
            out.update(s2_primal=pr.reshape(B).numpy(), s2_dual=dr.reshape(B).numpy())

    if grads:  # main.py:336-350, one truncation window over the whole unroll, scaled data
        model.zero_grad()
        x = torch.zeros(B, n, 1)
        y = torch.zeros(B, m, 1)
        z = torch.zeros(B, m, 1)
        xv = torch.zeros(B, n + m, 1)
        H = torch.zeros(B, n + m, h)
        C = torch.zeros(B, n + m, h)
        loss_tot = 0.0
        for t in range(T):
            x, y, z, xv, H, C, _, _, _ = model(t, mi, me, x, y, z, xv, sigma, H, C,
                                               Q=Q, p=p, A0=A0, lb=None, ub=None, zl=zl, zu=zu)
            _, _, loss = primal_dual_loss(x, y, z, Q, p, A0)
            loss_tot = loss_tot + loss.mean() / T
        loss_tot.backward()
        out["train_loss"] = np.float32(loss_tot.item())
        for k, prm in model.named_parameters():
            out["grad_" + k] = prm.grad.numpy().copy()

    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {os.path.getsize(path)/1e3:.1f} kB  final primal {out['hist_primal'][-1]} "
          f"dual {out['hist_dual'][-1]}")


if __name__ == "__main__":
    # small full-history case, Stage II and grads
    run_case("qp_n32_m16x16_h16", seed=1, n=32, mi=16, me=16, h=16, T=10, B=3, stage2=5,
             keep_state_every=True, grads=True)
    # mid-size case at a reference-like hidden size ratio
    run_case("qp_n200_m100x100_h64", seed=2, n=200, mi=100, me=100, h=64, T=20, B=2, keep_iters=2,
             stage2=3)
    # sharper learned dynamics (weights x10)
    run_case("qp_n64_m32x32_h32_w10", seed=3, n=64, mi=32, me=32, h=32, T=20, B=2, wscale=10.0,
             keep_iters=2, grads=True)
    # ragged / one-sided constraint blocks, no scaling
    run_case("qp_n24_m12x0_h8_noscale", seed=4, n=24, mi=12, me=0, h=8, T=6, B=2, scaling=False,
             keep_iters=6)
    run_case("qp_n24_m0x12_h8", seed=5, n=24, mi=0, me=12, h=8, T=6, B=2, keep_iters=6, stage2=2)
    # odd sizes that are not multiples of any tile (n=37, m=23, h=40)
    run_case("qp_n37_m15x8_h40", seed=6, n=37, mi=15, me=8, h=40, T=8, B=5, keep_iters=8, grads=True)
