"""r06: the window's parameter gradients are summed inside the IterationFn chain (iadmm/autograd.py
WindowGrads) instead of by autograd's input buffers.  Same sums in the same order, so the result must
be bit for bit what autograd produced from per-iteration parameter gradients: that path is still
reachable -- an H passed through .clone() between iterations starts a new chain at every iteration, so
every node returns its own gradients and autograd adds them (in execution order, t = T-1 .. 0)."""
import pytest
import torch

import iadmm_path  # noqa: F401

pytestmark = pytest.mark.gpu


def _grads(model, d, T, mi, me, chain, scale_loss=1.0):
    import utils
    B, n = d["Q"].shape[0], d["Q"].shape[1]
    m = mi + me
    h = model.hidden_dim
    model.zero_grad(set_to_none=True)
    x, y, z = (torch.zeros(B, r, 1, device="cuda") for r in (n, m, m))
    xv = torch.zeros(B, n + m, 1, device="cuda")
    H, C = torch.zeros(B, n + m, h, device="cuda"), torch.zeros(B, n + m, h, device="cuda")
    loss = 0.0
    for t in range(T):
        if not chain:
            H = H.clone()
        x, y, z, xv, H, C, _, _, _ = model(t, mi, me, x, y, z, xv, 6e-6, H, C, lb=None, ub=None, **d)
        _, _, l = utils.primal_dual_loss(x, y, z, d["Q"], d["p"], d["A0"])
        loss = loss + l.mean() / T
    (scale_loss * loss).backward()
    return {k: v.grad.clone() for k, v in model.named_parameters()}


@pytest.mark.parametrize("B,T", [(3, 12), (2, 1)])
def test_window_sums_equal_autograd_sums(B, T):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from iadmm import data, ops
    from models.lstm import LSTM
    n, mi, me, h = 60, 20, 12, 64
    raw = data.make_qp_batch(n, mi, me, B, first_index=5, device="cuda")
    Qs, ps, As, zls, zus, _, _, _ = ops.ruiz_scale(raw["Q"], raw["p"], raw["A0"], raw["zl"], raw["zu"], 10)
    d = dict(Q=Qs, p=ps, A0=As, zl=zls, zu=zus)
    torch.manual_seed(3)
    model = LSTM(mi + me, 2, h, max(T, 4), "cuda")
    with torch.no_grad():
        for q in model.parameters():
            q.mul_(5.0)
            q.add_(0.01)  # nonzero biases: every gradient path carries data
    chained = _grads(model, d, T, mi, me, chain=True)
    per_iter = _grads(model, d, T, mi, me, chain=False)
    assert chained.keys() == per_iter.keys()
    for k in chained:
        assert bool(torch.isfinite(chained[k]).all()), k
        assert torch.equal(chained[k], per_iter[k]), (k, float((chained[k] - per_iter[k]).abs().max()))
    # and a second backward pass over a new graph (buffers released by the owner) gives the same again
    again = _grads(model, d, T, mi, me, chain=True)
    for k in chained:
        assert torch.equal(chained[k], again[k]), k
