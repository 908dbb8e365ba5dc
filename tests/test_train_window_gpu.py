"""Training gradient over a full TBPTT window: outer_T = truncated_length = 100,
the reference's training shape of the loop (main.py:336-358, scripts/Synthetic.sh:3), at a small
instance shape (n = 200, m = 100 + 100, h = 64, B = 2; Ruiz-scaled as with --scaling).

The HIP forward + backward (the models/lstm.py drop-in under autograd, utils.primal_dual_loss, the
loss sum(loss.mean() / outer_T) over the window, one backward) against torch autograd through the
oracle's restatement of the same 100 iterations (oracle.lstm_iteration / oracle.primal_dual) in
fp32 AND fp64.  A 100-step window compounds every rounding difference through the recurrence, so
no fixed tolerance is meaningful; the bound is the fp64 envelope of tests/k100_envelope.py, per
parameter (stated before measuring):

    rel-L2(grad_HIP - grad_fp64) <= 2 x rel-L2(grad_fp32 oracle - grad_fp64) + 1e-7.

Three weight sets: the reference's initialisation (models/lstm.py:21-41, seed 17), the same weights
x 6 (gates away from their linear regime, larger rho / alpha excursions) and x 20.

x 20 drives the solve into a chaotic regime (loss ~5e3): in r05 the HIP gradients
of every U_* were 2.2-3.0x the fp32 oracle's fp64 distance.  Whether that is chaos or a kernel bias is
measured here, per parameter, instead of asserted:

    pert64 = rel-L2(grad_fp64(inputs and parameters each moved by one fp32 ulp, seeded signs) - grad_fp64)
    pert32 = rel-L2(grad_fp32 oracle(same perturbed inputs) - grad_fp64)
    chaos  = max(fp32 oracle vs fp64, pert64, pert32)

and the x 20 bound is rel-L2(grad_HIP - grad_fp64) <= 2 x chaos + 1e-7 (the rule VERDICT r05 states);
x 1 and x 6 keep the r05 bound against the fp32 oracle alone.  pert64 is the fp64 algorithm's own
sensitivity to the representation error of its fp32 inputs: an fp32 implementation in any order
cannot be expected closer to fp64 than the dynamics amplify one rounding.  (On the CPU generator's
instances at x 20, pert64 is 40-150, i.e. one ulp decorrelates the gradient completely;
`profiles/r06_train_window_chaos.txt` holds the GPU box's numbers.)
"""
import os

import pytest
import torch

import iadmm_path  # noqa: F401
from oracle import iadmm_oracle as orc

pytestmark = pytest.mark.gpu

N_VAR, MI, ME, H, T, B, SIGMA = 200, 100, 100, 64, 100, 2, 6e-6
FACTOR, FLOOR = 2.0, 1e-7


def rel_l2(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def perturb_ulp(t, seed):
    """Each finite element moved one fp32 ulp up or down (seeded sign); infinities kept."""
    t = t.detach().cpu().float()
    g = torch.Generator().manual_seed(seed)
    up = torch.randint(0, 2, t.shape, generator=g).bool()
    moved = torch.where(up, torch.nextafter(t, torch.full_like(t, float("inf"))),
                        torch.nextafter(t, torch.full_like(t, -float("inf"))))
    return torch.where(torch.isfinite(t), moved, t)


def oracle_grads(params, d, dtype):
    prm = {k: v.detach().cpu().to(dtype).requires_grad_(True) for k, v in params.items()}
    Q, p, A0, zl, zu = (d[k].cpu().to(dtype) for k in ("Q", "p", "A0", "zl", "zu"))
    n, m = Q.shape[1], A0.shape[1]
    x, y, z = (torch.zeros(B, r, 1, dtype=dtype) for r in (n, m, m))
    xv = torch.zeros(B, n + m, 1, dtype=dtype)
    Hs, Cs = torch.zeros(B, n + m, H, dtype=dtype), torch.zeros(B, n + m, H, dtype=dtype)
    loss = 0.0
    for t in range(T):
        x, y, z, xv, Hs, Cs, _, _, _ = orc.lstm_iteration(prm, t, MI, ME, x, y, z, xv, SIGMA, Hs, Cs, Q, p, A0,
                                                          zl, zu)
        _, _, l = orc.primal_dual(x, y, z, Q, p, A0)
        loss = loss + l.mean() / T
    loss.backward()
    return float(loss), {k: v.grad for k, v in prm.items()}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("scale", [1.0, 6.0, 20.0])
def test_full_window_grads_fp64_envelope(scale):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from iadmm import data, ops
    from models.lstm import LSTM
    import utils
    raw = data.make_qp_batch(N_VAR, MI, ME, B, first_index=3, device="cuda")
    Qs, ps, As, zls, zus, _, _, _ = ops.ruiz_scale(raw["Q"], raw["p"], raw["A0"], raw["zl"], raw["zu"], 10)
    d = dict(Q=Qs, p=ps, A0=As, zl=zls, zu=zus)
    torch.manual_seed(17)
    model = LSTM(MI + ME, 2, H, T, "cuda")
    with torch.no_grad():
        for prm in model.parameters():
            prm.mul_(scale)
    model.train()
    m = MI + ME
    x, y, z = (torch.zeros(B, r, 1, device="cuda") for r in (N_VAR, m, m))
    xv = torch.zeros(B, N_VAR + m, 1, device="cuda")
    Hs, Cs = torch.zeros(B, N_VAR + m, H, device="cuda"), torch.zeros(B, N_VAR + m, H, device="cuda")
    loss = 0.0
    for t in range(T):  # main.py:337-346: one window of truncated_length = outer_T steps
        x, y, z, xv, Hs, Cs, _, _, _ = model(t, MI, ME, x, y, z, xv, SIGMA, Hs, Cs, lb=None, ub=None, **d)
        _, _, l = utils.primal_dual_loss(x, y, z, d["Q"], d["p"], d["A0"])
        loss = loss + l.mean() / T
    loss.backward()
    params = {k: v.detach() for k, v in model.named_parameters()}
    threads = torch.get_num_threads()
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    try:
        l32, g32 = oracle_grads(params, d, torch.float32)
        l64, g64 = oracle_grads(params, d, torch.float64)
        pparams = {k: perturb_ulp(v, i) for i, (k, v) in enumerate(params.items())}
        pd = {k: perturb_ulp(v, 100 + i) for i, (k, v) in enumerate(d.items())}
        lp64, gp64 = oracle_grads(pparams, pd, torch.float64)
        lp32, gp32 = oracle_grads(pparams, pd, torch.float32)
    finally:
        torch.set_num_threads(threads)
    chaotic = scale >= 20.0
    lerr, lerr32 = abs(float(loss) - l64), abs(l32 - l64)
    lchaos = max(lerr32, abs(lp64 - l64), abs(lp32 - l64)) if chaotic else lerr32
    report, bad = {}, {}
    for k, prm in model.named_parameters():
        assert prm.grad is not None and bool(torch.isfinite(prm.grad).all()), k
        e64 = rel_l2(prm.grad, g64[k])
        o64 = rel_l2(g32[k], g64[k])
        p64 = rel_l2(gp64[k], g64[k])
        p32 = rel_l2(gp32[k], g64[k])
        e32 = rel_l2(prm.grad, g32[k])
        bound = FACTOR * (max(o64, p64, p32) if chaotic else o64) + FLOOR
        report[k] = (e64, o64, p64, p32, e32, e64 / bound)
        if e64 > bound:
            bad[k] = report[k]
    print(f"[T=100 window grads x{scale:g}] loss {l64:.6e} (|HIP - fp64| {lerr:.1e}, |fp32 - fp64| {lerr32:.1e}, "
          f"|fp64(1 ulp) - fp64| {abs(lp64 - l64):.1e}, |fp32(1 ulp) - fp64| {abs(lp32 - l64):.1e}); per parameter "
          "(HIP vs fp64, fp32 oracle vs fp64, fp64(1 ulp) vs fp64, fp32(1 ulp) vs fp64, HIP vs fp32 oracle, "
          f"HIP / bound; bound = {FACTOR:g} x {'max of the three' if chaotic else 'fp32 oracle'}):",
          {k: tuple(f"{v:.1e}" for v in r) for k, r in report.items()})
    assert lerr <= FACTOR * lchaos + FLOOR * abs(l64), (lerr, lchaos)
    assert not bad, bad
