"""Row-block split of the training's KKT backward and loss gradient (csrc/kkt.hip
iadmm_kkt_bwd_split / iadmm_loss_grad_split): against an fp64 torch
statement of the same formulas, against the one-workgroup-per-instance kernels, and bitwise
batch invariance (slices of a 512-batch equal the same instances run alone).

Formulas: models/lstm.py:67-72 (K, b~, g = K^T (K xv - b~)) differentiated as in
autograd.KktFn.backward; utils.py:68-71 (primal/dual loss).  Tolerance rel-L2 <= 1e-5 (fp32 sums
of <= 2000 terms against fp64)."""
import pytest
import torch

import iadmm_path  # noqa: F401

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-5

SHAPES = [(128, 1000, 500, 500),   # the config-5 micro-batch: 8 workgroups per instance
          (3, 300, 130, 0),         # no equality rows, 2 Q blocks
          (2, 77, 0, 50),           # n % 4 != 0 (scalar loads), equality rows only
          (2, 2101, 150, 99),       # two column panels, scalar loads
          (1, 40, 12, 12)]


def rel_l2(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _data(B, n, mi, me, seed):
    from iadmm import ops
    m = mi + me
    gen = torch.Generator().manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=gen)  # noqa: E731
    d = dict(Q=r(B, n, n) / n ** 0.5, A0=r(B, m, n) / n ** 0.5, p=r(B, n), x=r(B, n), y=r(B, m), z=r(B, m),
             xv=r(B, n + m), rf=r(B, n + m), dg=r(B, n + m), dxv=r(B, n + m), dx=r(B, n), dy=r(B, m), dz=r(B, m),
             cp=r(B).abs(), cd=r(B).abs())
    d = {k: v.to(DEV) for k, v in d.items()}
    scal = ops.schedule(torch.tensor([[0.3], [-0.2]], device=DEV), torch.zeros(2, 1, device=DEV), 0)
    return d, scal


def _rho(scal, mi, me):
    from iadmm import ops
    s = scal.double().cpu()
    rho = torch.cat([s[ops.S_RHO_IN].repeat(mi), s[ops.S_RHO_EQ].repeat(me)])
    kappa = torch.cat([torch.ones(mi), torch.full((me,), 1e3)]).double()
    return rho, 1.0 / rho, kappa


def _kkt_bwd_ref(d, scal, sigma, n, mi, me):
    """fp64: dr = K dg, dxv += K^T dr, dx -= sigma dr1, dz -= dr2, dy += dr2 / rho,
    ds = sum_j kappa_j (dg2_j r2_j - dr2_j (y_j - v_j)) / rho_j^2."""
    D = {k: v.double().cpu() for k, v in d.items()}
    rho, irho, kappa = _rho(scal, mi, me)
    Q, A0, dg = D["Q"], D["A0"], D["dg"]
    dg1, dg2 = dg[:, :n], dg[:, n:]
    Kv = lambda M, v1, v2: (torch.einsum("bij,bj->bi", M, v1) + sigma * v1 + torch.einsum("bji,bj->bi", A0, v2),  # noqa: E731
                            torch.einsum("bij,bj->bi", A0, v1) - irho * v2)
    dr1, dr2 = Kv(Q, dg1, dg2)
    t1, t2 = Kv(Q.transpose(1, 2), dr1, dr2)
    diota = -dg2 * D["rf"][:, n:] + dr2 * (D["y"] - D["xv"][:, n:])
    return dict(dxv=D["dxv"] + torch.cat([t1, t2], 1), dx=D["dx"] - sigma * dr1, dy=D["dy"] + irho * dr2,
                dz=D["dz"] - dr2, ds=(kappa * (-diota / rho ** 2)).sum(1))


def _run_kkt_bwd(d, scal, sigma, mi, split):
    from iadmm import ops
    out = {k: d[k].clone() for k in ("dxv", "dx", "dy", "dz")}
    ds = ops.kkt_bwd(d["Q"], d["A0"], d["xv"], d["y"], d["rf"], d["dg"], sigma, scal, mi, out["dxv"], out["dx"],
                     out["dy"], out["dz"], split=split)
    out["ds"] = ds
    return out


@pytest.mark.parametrize("B,n,mi,me", SHAPES)
def test_kkt_bwd_split(B, n, mi, me):
    d, scal = _data(B, n, mi, me, n + mi)
    sigma = 6e-6
    ref = _kkt_bwd_ref(d, scal, sigma, n, mi, me)
    got = _run_kkt_bwd(d, scal, sigma, mi, split=True)
    one = _run_kkt_bwd(d, scal, sigma, mi, split=False)
    for k in ("dxv", "dx", "dy", "dz", "ds"):
        if ref[k].numel() == 0:
            continue
        assert rel_l2(got[k], ref[k]) < TOL, (k, rel_l2(got[k], ref[k]))
        assert rel_l2(one[k], ref[k]) < TOL, (k, rel_l2(one[k], ref[k]))
    again = _run_kkt_bwd(d, scal, sigma, mi, split=True)
    assert all(torch.equal(got[k], again[k]) for k in got)  # deterministic


def _loss_ref(d, n):
    D = {k: v.double().cpu() for k, v in d.items()}
    x = D["x"].clone().requires_grad_(True)
    y = D["y"].clone().requires_grad_(True)
    z = D["z"].clone().requires_grad_(True)
    ep = torch.einsum("bij,bj->bi", D["A0"], x) - z
    ed = torch.einsum("bij,bj->bi", D["Q"], x) + D["p"] + torch.einsum("bji,bj->bi", D["A0"], y)
    pr, du = ep.norm(dim=1), ed.norm(dim=1)
    (D["cp"] * pr + D["cd"] * du).sum().backward()
    return pr.detach(), du.detach(), x.grad, y.grad, z.grad


@pytest.mark.parametrize("B,n,mi,me", SHAPES)
def test_loss_grad_split(B, n, mi, me):
    from iadmm import ops
    d, _ = _data(B, n, mi, me, 7 * n + me)
    ref = _loss_ref(d, n)
    args = (d["Q"], d["p"], d["A0"], d["x"], d["y"], d["z"], d["cp"], d["cd"])
    got = ops.loss_grad(*args, split=True)
    one = ops.loss_grad(*args, split=False)
    names = ("primal", "dual", "dx", "dy", "dz")
    for k, g, o, r in zip(names, got, one, ref):
        if r.numel() == 0:
            continue
        assert rel_l2(g, r) < TOL, (k, rel_l2(g, r))
        assert rel_l2(o, r) < TOL, (k, rel_l2(o, r))
    pr, du, dx, dy, dz = ops.loss_grad(*args, want_grad=False, split=True)  # first sweep only
    assert torch.equal(pr, got[0]) and torch.equal(du, got[1]) and dx is None


def test_split_batch_invariant():
    """A slice of the batch gives bitwise the outputs its instances get inside the 512-batch
    (2 workgroups per instance at B = 512, 8 at B <= 128): the block-order sums depend on the
    256-row block structure only, never on how many workgroups share an instance."""
    from iadmm import ops
    B, n, mi, me = 512, 1000, 500, 500
    d, scal = _data(B, n, mi, me, 11)
    sigma = 6e-6
    full = _run_kkt_bwd(d, scal, sigma, mi, split=True)
    lfull = ops.loss_grad(d["Q"], d["p"], d["A0"], d["x"], d["y"], d["z"], d["cp"], d["cd"])
    for lo, hi in ((0, 1), (77, 205), (B - 1, B)):
        part = {k: v[lo:hi].contiguous() for k, v in d.items()}
        sub = _run_kkt_bwd(part, scal, sigma, mi, split=True)
        for k in sub:
            assert torch.equal(sub[k], full[k][lo:hi]), (k, lo, hi)
        lsub = ops.loss_grad(part["Q"], part["p"], part["A0"], part["x"], part["y"], part["z"], part["cp"],
                             part["cd"])
        for a, b in zip(lsub, lfull):
            assert torch.equal(a, b[lo:hi])
