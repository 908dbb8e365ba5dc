"""Drop-in check: the reference's test loop (main.py:818-1031, restated exactly as the golden
generator does, with torch.bmm on the dense scaling matrices and on A_tild) runs unchanged with
this repo's modules imported in place of the reference's, on the GPU, and reproduces the
reference's per-iteration report (tests/golden).  Tolerances as in test_parity_gpu.py."""
import numpy as np
import pytest
import torch

import iadmm_path  # noqa: F401

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(b.norm(), 1e-30))


def test_reference_test_loop_with_dropin_modules(golden):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    # the reference's import lines (main.py:14-18), resolved to this repo
    from methods.scaling import Scaling
    from models.lstm import LSTM
    from models.lu import LU
    from utils import primal_dual_loss, obj_fn
    name, g = golden
    n, mi, me, h, T, B, scaling, stage2 = (int(v) for v in g["meta"])
    m = mi + me
    dev = "cuda:0"
    model = LSTM(m, 2, h, T, dev)
    model.load_state_dict({k[len("param_"):]: torch.from_numpy(g[k]) for k in g if k.startswith("param_")})
    model.eval()
    Q, p, A0, zl, zu = (torch.from_numpy(g["in_" + k]).to(dev) for k in ("Q", "p", "A0", "zl", "zu"))
    sigma = float(g["sigma"])
    hist = {k: [] for k in ("obj", "ls_res", "primal", "dual")}
    with torch.no_grad():
        Qp, pp, A0p, zlp, zup = Q, p, A0, zl, zu
        if scaling:
            sc = Scaling(n, m, 10, dev)
            Q, p, A0, zl, zu = sc.scale_data(Q, p, A0, zl, zu)
        x = torch.zeros((B, n, 1), device=dev)
        y = torch.zeros((B, m, 1), device=dev)
        z = torch.zeros((B, m, 1), device=dev)
        xv = torch.zeros((B, n + m, 1), device=dev)
        H = torch.zeros((B, n + m, h), device=dev)
        C = torch.zeros((B, n + m, h), device=dev)
        for t in range(T):
            x, y, z, xv, H, C, A_tild, b_tild, rho_vec = model(t, mi, me, x, y, z, xv, sigma, H, C, Q=Q, p=p,
                                                               A0=A0, lb=None, ub=None, zl=zl, zu=zu)
            if scaling:
                xs = torch.bmm(sc.D, x)
                zs = torch.bmm(sc.Einv, z)
                ys = torch.bmm(sc.cinv * sc.E, y)
            else:
                xs, ys, zs = x, y, z
            hist["obj"].append(obj_fn(xs, Q=Qp, p=pp).reshape(B))
            hist["ls_res"].append(torch.linalg.vector_norm(torch.bmm(A_tild, xv) - b_tild, dim=(1, 2)))
            pr, du, _ = primal_dual_loss(xs, ys, zs, Qp, pp, A0p)
            hist["primal"].append(pr.reshape(B))
            hist["dual"].append(du.reshape(B))
        if stage2:
            exact = LU(dev)
            lu = piv = At = None
            for t in range(stage2):
                xs, ys, zs, xv, At, bt, lu, piv = exact(rho_vec, xs, ys, zs, xv, sigma, At, lu, piv, Q=Qp, p=pp,
                                                        A0=A0p, lb=None, ub=None, zl=zlp, zu=zup)
            assert rel_l2(xs, g["s2_x"][-1]) < 1e-3
    tol = 1e-2 if float(g["wscale"]) > 1 else 1e-4
    for k in hist:
        got = torch.stack(hist[k]).cpu().numpy()
        np.testing.assert_allclose(got, g["hist_" + k], rtol=max(tol, 1e-3 if k == "ls_res" else tol), atol=1e-4)
