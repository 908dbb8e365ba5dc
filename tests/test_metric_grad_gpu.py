"""Gradients of the reporting metrics (utils.py:53-78: obj_fn, ineq_dist, eq_dist,
primal_dual_loss, aug_lagr) through the drop-in utils on the GPU (iadmm.autograd ObjFn /
IneqDistFn / EqDistFn / LossFn / BmvFn: iadmm_bmv, iadmm_bmv_t, iadmm_bger) against torch
autograd of the oracle's restatement of the reference expressions, in fp64 and fp32.

Tolerance: rel-L2 <= 1e-5 per gradient against fp64 (the fp32 oracle sits at ~1e-7 .. 1e-6 from
fp64 at these sizes); the forward values match the fp32 oracle to 1e-6."""
import pytest
import torch

import iadmm_path  # noqa: F401
from oracle import iadmm_oracle as orc

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _data(B, n, mi, me, seed):
    g = torch.Generator().manual_seed(seed)
    d = dict(x=torch.randn(B, n, 1, generator=g), Q=torch.randn(B, n, n, generator=g) / n ** 0.5,
             p=torch.rand(B, n, 1, generator=g), G=torch.randn(B, mi, n, generator=g),
             c=torch.rand(B, mi, 1, generator=g) * 3, A=torch.randn(B, me, n, generator=g),
             b=torch.randn(B, me, 1, generator=g), y=torch.randn(B, mi + me, 1, generator=g),
             z=torch.randn(B, mi + me, 1, generator=g), rho=torch.rand(B, mi + me, 1, generator=g) + 0.1)
    d["A0"] = torch.cat([d["G"], d["A"]], 1)
    return d


def _leaves(d, keys, dev, dtype):
    return {k: d[k].detach().to(dev, dtype).clone().requires_grad_(k in keys) for k in d}


# n % 4 != 0 exercises the scalar column path of iadmm_bmv_t and the unvectorised iadmm_bger
@pytest.mark.parametrize("B,n,mi,me", [(3, 64, 20, 12), (2, 37, 9, 5), (2, 1000, 500, 500)])
def test_metric_gradients_match_reference_autograd(B, n, mi, me):
    import utils
    d = _data(B, n, mi, me, seed=n)
    wgen = torch.Generator().manual_seed(1)
    w_obj = torch.randn(B, 1, 1, generator=wgen)
    w_in = torch.randn(B, mi, 1, generator=wgen)
    w_eq = torch.randn(B, me, 1, generator=wgen)
    w_pd = torch.randn(2, generator=wgen)
    keys = ("x", "Q", "p", "G", "c", "A", "b", "y", "z", "A0", "rho")

    def total(m, t):
        pr, du, _ = m.primal_dual(t["x"], t["y"], t["z"], t["Q"], t["p"], t["A0"]) if m is orc else \
            m.primal_dual_loss(t["x"], t["y"], t["z"], t["Q"], t["p"], t["A0"])
        obj = m.objective(t["x"], t["Q"], t["p"]) if m is orc else m.obj_fn(t["x"], t["Q"], t["p"])
        al = m.aug_lagr(t["x"], t["z"], t["y"], t["Q"], t["p"], t["A0"], t["rho"])
        return ((w_obj.to(obj) * obj).sum() + (w_in.to(obj) * m.ineq_dist(t["x"], t["G"], t["c"])).sum()
                + (w_eq.to(obj) * m.eq_dist(t["x"], t["A"], t["b"])).sum()
                + w_pd[0].item() * pr.sum() + w_pd[1].item() * du.sum() + 1e-3 * al.sum())

    ref = {}
    for dtype in (torch.float64, torch.float32):
        t = _leaves(d, keys, "cpu", dtype)
        total(orc, t).backward()
        ref[dtype] = {k: t[k].grad for k in keys}
    t = _leaves(d, keys, "cuda", torch.float32)
    total(utils, t).backward()
    for k in keys:
        e_gpu, e_f32 = rel(t[k].grad, ref[torch.float64][k]), rel(ref[torch.float32][k], ref[torch.float64][k])
        assert e_gpu <= max(1e-5, 4 * e_f32), (k, e_gpu, e_f32)
    # forward values equal the grad-free path (same kernels)
    with torch.no_grad():
        tn = _leaves(d, (), "cuda", torch.float32)
        assert torch.equal(utils.ineq_dist(tn["x"], tn["G"], tn["c"]),
                           utils.ineq_dist(t["x"], t["G"], t["c"]).detach())
