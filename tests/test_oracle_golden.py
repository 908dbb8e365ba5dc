"""Pin the CPU oracle (oracle/iadmm_oracle.py) against the golden vectors the reference itself
produced (tests/golden/make_golden.py).  Same torch, same op structure -> expected bit-exact;
the stated tolerance only absorbs BLAS threading differences (rel 1e-5)."""
import numpy as np
import pytest
import torch

from oracle import iadmm_oracle as orc

torch.set_num_threads(1)  # see tests/golden/make_golden.py (MKL getrf threading)


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def close(a, b, rtol=1e-5, atol=1e-6):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol * max(1.0, float(np.abs(b).max(initial=0))))


def meta(g):
    n, mi, me, h, T, B, scaling, stage2 = (int(v) for v in g["meta"])
    return n, mi, me, h, T, B, bool(scaling), stage2


def test_ruiz_matches_reference(golden):
    name, g = golden
    n, mi, me, h, T, B, scaling, _ = meta(g)
    if not scaling:
        pytest.skip("fixture runs without scaling")
    sc = orc.ruiz(t(g["in_Q"]), t(g["in_p"]), t(g["in_A0"]), t(g["in_zl"]), t(g["in_zu"]), 10)
    for k in ("Q", "p", "A0", "zu"):
        close(sc[k].numpy(), g["sc_" + k], rtol=1e-6, atol=0)
    np.testing.assert_array_equal(np.isneginf(sc["zl"].numpy()), np.isneginf(g["sc_zl"]))
    fin = np.isfinite(g["sc_zl"])
    close(sc["zl"].numpy()[fin], g["sc_zl"][fin], rtol=1e-6, atol=0)
    close(torch.diagonal(sc["D"], dim1=1, dim2=2).numpy(), g["sc_D"], rtol=1e-6, atol=0)
    close(torch.diagonal(sc["E"], dim1=1, dim2=2).numpy(), g["sc_E"], rtol=1e-6, atol=0)
    close(sc["c"].reshape(B).numpy(), g["sc_c"], rtol=1e-6, atol=0)


def test_iterations_match_reference(golden):
    name, g = golden
    n, mi, me, h, T, B, scaling, _ = meta(g)
    params = orc.params_from_npz(g)
    pre = "sc_" if scaling else "in_"
    Q, p, A0, zl, zu = (t(g[pre + k]) for k in ("Q", "p", "A0", "zl", "zu"))
    m = mi + me
    x, y, z = torch.zeros(B, n, 1), torch.zeros(B, m, 1), torch.zeros(B, m, 1)
    xv = torch.zeros(B, n + m, 1)
    H, C = torch.zeros(B, n + m, h), torch.zeros(B, n + m, h)
    sigma = float(g["sigma"])
    with torch.no_grad():
        for it in range(T):
            xv_prev = xv
            x, y, z, xv, H, C, K, b, rv = orc.lstm_iteration(params, it, mi, me, x, y, z, xv, sigma,
                                                             H, C, Q, p, A0, zl, zu)
            if f"it{it}_x" in g:
                close(orc.kkt_resgrad(K, b, xv_prev).numpy(), g[f"it{it}_g"])
                close(b.numpy(), g[f"it{it}_btild"])
                close(rv.numpy(), g[f"it{it}_rhovec"], rtol=0, atol=0)
                for k, v in (("x", x), ("y", y), ("z", z), ("xv", xv), ("H", H), ("C", C)):
                    close(v.numpy(), g[f"it{it}_{k}"])
    for k, v in (("xv", xv), ("H", H), ("C", C)):
        close(v.numpy(), g["fin_" + k], rtol=1e-4, atol=1e-6)


def test_solve_matches_reference(golden):
    name, g = golden
    n, mi, me, h, T, B, scaling, _ = meta(g)
    params = orc.params_from_npz(g)
    with torch.no_grad():
        out = orc.solve(params, t(g["in_Q"]), t(g["in_p"]), t(g["in_A0"]), t(g["in_zl"]),
                        t(g["in_zu"]), mi, me, T, float(g["sigma"]), h, scaling=scaling, history=True)
    close(out["x"].numpy(), g["fin_x"], rtol=1e-4, atol=1e-6)
    close(out["hist_primal"].numpy(), g["hist_primal"], rtol=1e-4, atol=1e-6)
    close(out["hist_dual"].numpy(), g["hist_dual"], rtol=1e-4, atol=1e-6)


def test_stage2_matches_reference(golden):
    name, g = golden
    n, mi, me, h, T, B, scaling, stage2 = meta(g)
    if not stage2:
        pytest.skip("no Stage II in this fixture")
    x, y, z = t(g["fin_x"]), t(g["fin_y"]), t(g["fin_z"])
    xv, rv = t(g["fin_xv"]), t(g["fin_rhovec"])
    Q, p, A0, zl, zu = (t(g["in_" + k]) for k in ("Q", "p", "A0", "zl", "zu"))
    K = lu = piv = None
    with torch.no_grad():
        for it in range(stage2):
            x, y, z, xv, K, b, lu, piv = orc.lu_iteration(rv, x, y, z, xv, float(g["sigma"]), K, lu, piv,
                                                          Q, p, A0, zl, zu)
            close(x.numpy(), g["s2_x"][it], rtol=1e-4, atol=1e-5)
            close(z.numpy(), g["s2_z"][it], rtol=1e-4, atol=1e-5)
        pr, du, _ = orc.primal_dual(x, y, z, Q, p, A0)
    close(pr.reshape(-1).numpy(), g["s2_primal"], rtol=1e-3, atol=1e-5)
    close(du.reshape(-1).numpy(), g["s2_dual"], rtol=1e-3, atol=1e-5)


def test_grads_match_reference(golden):
    name, g = golden
    if "train_loss" not in g:
        pytest.skip("no gradient fixture")
    n, mi, me, h, T, B, scaling, _ = meta(g)
    params = {k: v.clone().requires_grad_(True) for k, v in orc.params_from_npz(g).items()}
    Q, p, A0, zl, zu = (t(g["sc_" + k]) for k in ("Q", "p", "A0", "zl", "zu"))
    m = mi + me
    x, y, z = torch.zeros(B, n, 1), torch.zeros(B, m, 1), torch.zeros(B, m, 1)
    xv = torch.zeros(B, n + m, 1)
    H, C = torch.zeros(B, n + m, h), torch.zeros(B, n + m, h)
    loss_tot = 0.0
    for it in range(T):
        x, y, z, xv, H, C, _, _, _ = orc.lstm_iteration(params, it, mi, me, x, y, z, xv,
                                                        float(g["sigma"]), H, C, Q, p, A0, zl, zu)
        loss_tot = loss_tot + orc.primal_dual(x, y, z, Q, p, A0)[2].mean() / T
    loss_tot.backward()
    close(loss_tot.item(), g["train_loss"], rtol=1e-5)
    for k, v in params.items():
        close(v.grad.numpy(), g["grad_" + k], rtol=1e-3, atol=1e-5)
