"""GPU parity: the HIP path (through the C-ABI) against the reference's golden vectors and the
CPU oracle on identical inputs.

Tolerances (fp32 throughout; the reference and the oracle sum in MKL order, the kernels in
their own fixed order, so results agree to rounding, amplified by the learned dynamics):
  * Ruiz-scaled data, D, E, c                  rel 2e-6 elementwise (one-ulp cost-scale drift)
  * one KKT residual-gradient evaluation       rel-L2 1e-5
  * one full Stage-I iteration from a given state  rel-L2 1e-5 on every state tensor
  * T-iteration solve (non-divergent fixtures) rel-L2 1e-4 on x^K, rel 1e-4 on residuals
    (the contract proposed in SURVEY.md §8(c)); divergent fixtures (weights x10) 1e-2.
"""
import numpy as np
import pytest
import torch

import iadmm_path  # noqa: F401
from oracle import iadmm_oracle as orc

pytestmark = pytest.mark.gpu

DEV = "cuda"


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def rel_l2(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(b.norm(), 1e-30))


def meta(g):
    n, mi, me, h, T, B, scaling, stage2 = (int(v) for v in g["meta"])
    return n, mi, me, h, T, B, bool(scaling), stage2


def divergent(g):
    return float(g["wscale"]) > 1.0


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from iadmm import _abi
    _abi.lib()


def test_ruiz_golden(golden):
    from iadmm import ops
    name, g = golden
    n, mi, me, h, T, B, scaling, _ = meta(g)
    if not scaling:
        pytest.skip("fixture without scaling")
    Qs, ps, As, zls, zus, D, E, c = ops.ruiz_scale(dev(g["in_Q"]), dev(g["in_p"]), dev(g["in_A0"]),
                                                   dev(g["in_zl"]), dev(g["in_zu"]), 10)
    for k, v in (("Q", Qs), ("p", ps), ("A0", As), ("zu", zus)):
        np.testing.assert_allclose(v.cpu().numpy(), g["sc_" + k], rtol=2e-6, atol=0)
    zl = zls.cpu().numpy()
    assert (np.isneginf(zl) == np.isneginf(g["sc_zl"])).all()
    fin = np.isfinite(g["sc_zl"])
    np.testing.assert_allclose(zl[fin], g["sc_zl"][fin], rtol=2e-6)
    np.testing.assert_allclose(D.cpu().numpy(), g["sc_D"], rtol=2e-6)
    np.testing.assert_allclose(E.cpu().numpy(), g["sc_E"], rtol=2e-6)
    np.testing.assert_allclose(c.cpu().numpy(), g["sc_c"], rtol=2e-6)


def _scaled(g):
    pre = "sc_" if bool(g["meta"][6]) else "in_"
    return [dev(g[pre + k]) for k in ("Q", "p", "A0", "zl", "zu")]


def _state(g, it, B, n, m, h):
    if it < 0:
        z = lambda *s: torch.zeros(*s, device=DEV)  # noqa: E731
        return z(B, n, 1), z(B, m, 1), z(B, m, 1), z(B, n + m, 1), z(B, n + m, h), z(B, n + m, h)
    return tuple(dev(g[f"it{it}_{k}"]) for k in ("x", "y", "z", "xv", "H", "C"))


def _model(g, n, m, h, T):
    from models.lstm import LSTM
    model = LSTM(m, 2, h, T, DEV)
    sd = {k[len("param_"):]: torch.from_numpy(g[k]) for k in g if k.startswith("param_")}
    model.load_state_dict(sd)
    return model


def test_kkt_resgrad_golden(golden):
    from iadmm import ops
    name, g = golden
    n, mi, me, h, T, B, scaling, _ = meta(g)
    m = mi + me
    Q, p, A0, zl, zu = _scaled(g)
    model = _model(g, n, m, h, T)
    its = [it for it in range(T) if f"it{it}_g" in g]
    assert its
    for it in its:
        x, y, z, xv, _, _ = _state(g, it - 1, B, n, m, h)
        scal = ops.schedule(model.rho.detach(), model.alpha.detach(), it)
        bt = ops.empty(B, n + m, like=Q)
        rv = ops.empty(B, m, like=Q)
        gk = ops.kkt_resgrad(Q, A0, p.reshape(B, n), x.reshape(B, n), y.reshape(B, m), z.reshape(B, m),
                             xv.reshape(B, n + m), float(g["sigma"]), scal, mi, btild=bt, rho_vec=rv)
        assert rel_l2(gk, g[f"it{it}_g"].reshape(B, -1)) < 1e-5, (name, it)
        assert rel_l2(bt, g[f"it{it}_btild"].reshape(B, -1)) < 1e-6
        np.testing.assert_allclose(rv.cpu().numpy(), g[f"it{it}_rhovec"].reshape(B, m), rtol=1e-6)


def test_one_iteration_golden(golden):
    """models.lstm.LSTM.forward from the golden state at it-1 reproduces the state at it."""
    name, g = golden
    n, mi, me, h, T, B, scaling, _ = meta(g)
    m = mi + me
    Q, p, A0, zl, zu = _scaled(g)
    model = _model(g, n, m, h, T)
    its = [it for it in range(T) if f"it{it}_H" in g]
    with torch.no_grad():
        for it in its:
            x, y, z, xv, H, C = _state(g, it - 1, B, n, m, h)
            out = model(it, mi, me, x, y, z, xv, float(g["sigma"]), H, C, Q=Q, p=p, A0=A0, lb=None,
                        ub=None, zl=zl, zu=zu)
            for k, v in zip(("x", "y", "z", "xv", "H", "C"), out[:6]):
                err = rel_l2(v, g[f"it{it}_{k}"])
                assert err < 1e-5, (name, it, k, err)
            assert rel_l2(out[7], g[f"it{it}_btild"]) < 1e-6
            # the lazy A_tild behaves like the dense K under torch.bmm (main.py:952)
            K = torch.from_numpy(orc.kkt_matrix(torch.from_numpy(g[("sc_" if scaling else "in_") + "Q"]),
                                                torch.from_numpy(g[("sc_" if scaling else "in_") + "A0"]),
                                                float(g["sigma"]), out[8].cpu()).numpy())
            kv = torch.bmm(out[6], out[3]).cpu()
            assert rel_l2(kv, torch.bmm(K, out[3].cpu())) < 1e-5
            assert rel_l2(out[6].dense().cpu(), K) < 1e-7


def test_solve_golden(golden):
    from iadmm import solver
    name, g = golden
    n, mi, me, h, T, B, scaling, _ = meta(g)
    params = {k[len("param_"):]: dev(g[k]) for k in g if k.startswith("param_")}
    with torch.no_grad():
        out = solver.solve(params, dev(g["in_Q"]), dev(g["in_p"]), dev(g["in_A0"]), dev(g["in_zl"]),
                           dev(g["in_zu"]), mi, me, T, float(g["sigma"]), scaling=scaling, history=True)
    tol = 1e-2 if divergent(g) else 1e-4
    assert rel_l2(out["x"], g["fin_x"]) < tol, name
    np.testing.assert_allclose(out["hist_primal"].cpu().numpy(), g["hist_primal"], rtol=tol, atol=1e-6)
    np.testing.assert_allclose(out["hist_dual"].cpu().numpy(), g["hist_dual"], rtol=tol, atol=1e-6)
    np.testing.assert_allclose(out["hist_obj"].cpu().numpy(), g["hist_obj"], rtol=tol, atol=1e-4)
    np.testing.assert_allclose(out["hist_ls_res"].cpu().numpy(), g["hist_ls_res"], rtol=max(tol, 1e-3),
                               atol=1e-5)
    np.testing.assert_allclose(out["primal"].cpu().numpy(), g["hist_primal"][-1], rtol=tol, atol=1e-6)
    np.testing.assert_allclose(out["dual"].cpu().numpy(), g["hist_dual"][-1], rtol=tol, atol=1e-6)


def test_solve_scaled_identity_metrics(golden):
    """keep_unscaled=False (in-place scaling, memory-saving bench mode) reports the same residuals."""
    from iadmm import solver
    name, g = golden
    n, mi, me, h, T, B, scaling, _ = meta(g)
    if not scaling:
        pytest.skip("needs scaling")
    params = {k[len("param_"):]: dev(g[k]) for k in g if k.startswith("param_")}
    with torch.no_grad():
        out = solver.solve(params, dev(g["in_Q"]), dev(g["in_p"]), dev(g["in_A0"]), dev(g["in_zl"]),
                           dev(g["in_zu"]), mi, me, T, float(g["sigma"]), scaling=True, keep_unscaled=False)
    tol = 1e-2 if divergent(g) else 1e-4
    np.testing.assert_allclose(out["primal"].cpu().numpy(), g["hist_primal"][-1], rtol=tol, atol=1e-5)
    np.testing.assert_allclose(out["dual"].cpu().numpy(), g["hist_dual"][-1], rtol=tol, atol=1e-5)
    np.testing.assert_allclose(out["obj"].cpu().numpy(), g["hist_obj"][-1], rtol=tol, atol=1e-4)


def test_metric_utils_match_oracle(golden):
    import utils
    name, g = golden
    n, mi, me, h, T, B, scaling, _ = meta(g)
    Q, p, A0 = dev(g["in_Q"]), dev(g["in_p"]), dev(g["in_A0"])
    x, y, z = dev(g["fin_x"]), dev(g["fin_y"]), dev(g["fin_z"])
    with torch.no_grad():
        pr, du, tot = utils.primal_dual_loss(x, y, z, Q, p, A0)
        ob = utils.obj_fn(x, Q, p)
    opr, odu, _ = orc.primal_dual(*(torch.from_numpy(g[k]) for k in ("fin_x", "fin_y", "fin_z", "in_Q", "in_p", "in_A0")))
    oob = orc.objective(torch.from_numpy(g["fin_x"]), torch.from_numpy(g["in_Q"]), torch.from_numpy(g["in_p"]))
    np.testing.assert_allclose(pr.cpu().numpy(), opr.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(du.cpu().numpy(), odu.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ob.cpu().numpy(), oob.numpy(), rtol=1e-5, atol=1e-5)
    if mi > 0 and me > 0:
        G, Aeq = A0[:, :mi], A0[:, mi:]
        c, b = dev(g["in_zu"])[:, :mi], dev(g["in_zu"])[:, mi:]
        with torch.no_grad():
            idist = utils.ineq_dist(x, G.contiguous(), c.contiguous())
            edist = utils.eq_dist(x, Aeq.contiguous(), b.contiguous())
        xc = torch.from_numpy(g["fin_x"])
        Gc, Ac = torch.from_numpy(g["in_A0"][:, :mi]), torch.from_numpy(g["in_A0"][:, mi:])
        cc, bc = torch.from_numpy(g["in_zu"][:, :mi]), torch.from_numpy(g["in_zu"][:, mi:])
        np.testing.assert_allclose(idist.cpu().numpy(), torch.clamp(torch.bmm(Gc, xc) - cc, 0).numpy(),
                                   rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(edist.cpu().numpy(), torch.abs(bc - torch.bmm(Ac, xc)).numpy(),
                                   rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("B,n,mi,me", [(3, 2100, 200, 100),     # 2 column panels, 256 threads
                                       (2, 2101, 150, 99),      # 2 panels, scalar (n % 4 != 0) loads
                                       (2, 4100, 2000, 2000)])  # 3 panels, 512 threads (81 KB LDS)
def test_kkt_resgrad_panels(B, n, mi, me):
    """Large-n path of iadmm_kkt_resgrad (column panels; csrc/kkt.hip) against the oracle's dense
    K^T (K xv - b~) in fp64 on the same fp32 inputs (non-symmetric Q exercises the transpose)."""
    from iadmm import ops
    m = mi + me
    gen = torch.Generator().manual_seed(n)
    r = lambda *s: torch.randn(*s, generator=gen)  # noqa: E731
    Q, A0 = r(B, n, n) / n ** 0.5, r(B, m, n) / n ** 0.5
    p, x, y, z, xv = r(B, n, 1), r(B, n, 1), r(B, m, 1), r(B, m, 1), r(B, n + m, 1)
    sigma = 6e-6
    params = {"rho": torch.full((2, 1), 0.3), "alpha": torch.zeros(2, 1)}
    rv, _ = orc.schedule(params, 1, y, mi, me)
    K = orc.kkt_matrix(Q.double(), A0.double(), sigma, rv.double())
    bt = orc.kkt_rhs(x.double(), z.double(), y.double(), p.double(), sigma, rv.double())
    ref = orc.kkt_resgrad(K, bt, xv.double()).reshape(B, -1)
    del K
    d = lambda t: t.reshape(B, -1).contiguous().to(DEV) if t.dim() == 3 and t.shape[-1] == 1 else t.to(DEV)  # noqa: E731
    scal = ops.schedule(params["rho"].to(DEV), params["alpha"].to(DEV), 1)
    g = ops.kkt_resgrad(Q.to(DEV), A0.to(DEV), d(p), d(x), d(y), d(z), d(xv), sigma, scal, mi)
    assert rel_l2(g, ref) < 1e-5
    g2 = ops.kkt_resgrad(Q.to(DEV), A0.to(DEV), d(p), d(x), d(y), d(z), d(xv), sigma, scal, mi)
    assert torch.equal(g, g2)  # deterministic


@pytest.mark.parametrize("n,mi,me", [(1000, 500, 500), (300, 130, 0), (77, 0, 50)])
def test_kkt_resgrad_batch_invariant(n, mi, me):
    """iadmm_kkt_resgrad splits each instance over B-dependent numbers of workgroups (1 or 128
    instances: every 256-row block apart at n = m = 1000; 2048: whole instances),
    but sums the per-block column partials in block order: g is bitwise the same whatever the batch
    (and so whatever the shard), and matches the fp64 oracle at B = 1 and B = 128."""
    from iadmm import ops
    m = mi + me
    B = 128
    gen = torch.Generator().manual_seed(n + m)
    r = lambda *s: torch.randn(*s, generator=gen)  # noqa: E731
    Q, A0 = (r(B, n, n) / n ** 0.5).to(DEV), (r(B, m, n) / n ** 0.5).to(DEV)
    p, x, y, z, xv = (r(B, k).to(DEV) for k in (n, n, m, m, n + m))
    params = {"rho": torch.full((2, 1), 0.3, device=DEV), "alpha": torch.zeros(2, 1, device=DEV)}
    scal = ops.schedule(params["rho"], params["alpha"], 0)
    full = ops.kkt_resgrad(Q, A0, p, x, y, z, xv, 6e-6, scal, mi)
    for i in (0, 77, B - 1):
        one = ops.kkt_resgrad(*(t[i:i + 1].contiguous() for t in (Q, A0, p, x, y, z, xv)), 6e-6, scal, mi)
        assert torch.equal(one[0], full[i]), i
    big = 2048  # the same instances tiled: one workgroup per instance
    rep = lambda t: t.repeat(big // B, *([1] * (t.dim() - 1))).contiguous()  # noqa: E731
    if n * n + m * n <= 2_000_000:
        tiled = ops.kkt_resgrad(*(rep(t) for t in (Q, A0, p, x, y, z, xv)), 6e-6, scal, mi)
        assert torch.equal(tiled[:B], full) and torch.equal(tiled[-B:], full)
    rv, _ = orc.schedule({k: v.cpu() for k, v in params.items()}, 0, y.cpu().unsqueeze(-1), mi, me)
    K = orc.kkt_matrix(Q[:4].cpu().double(), A0[:4].cpu().double(), 6e-6, rv[:4].double())
    bt = orc.kkt_rhs(x[:4].cpu().double().unsqueeze(-1), z[:4].cpu().double().unsqueeze(-1),
                     y[:4].cpu().double().unsqueeze(-1), p[:4].cpu().double().unsqueeze(-1), 6e-6, rv[:4].double())
    ref = orc.kkt_resgrad(K, bt, xv[:4].cpu().double().unsqueeze(-1)).reshape(4, -1)
    assert rel_l2(full[:4], ref) < 1e-5
