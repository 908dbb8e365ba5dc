"""Optional split-precision cell ("f16x3", csrc/lstm_f16x3.hip): its accuracy against an fp64
evaluation of the same cell, side by side with the default fp32-MFMA kernel, and the full solve
against the reference's golden vectors at the fp32 path's own tolerances.

Bars (stated before measuring, from the error analysis in the kernel's header): the f16x3 cell's
rel-L2 error against fp64 is at most 4x the fp32 kernel's and below 1e-6; the solve meets the
SAME contract as the fp32 path (rel-L2 1e-4 on x^K, 1e-4 on residuals; divergent fixtures 1e-2).
"""
import numpy as np
import pytest
import torch

import iadmm_path  # noqa: F401
from oracle import iadmm_oracle as orc

from test_parity_gpu import dev, divergent, meta, rel_l2  # noqa: F401

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_split_planes_reconstruct():
    from iadmm import ops
    gen = torch.Generator().manual_seed(3)
    x = torch.cat([torch.randn(4096, generator=gen), torch.randn(4096, generator=gen) * 1e-3,
                   torch.rand(4096, generator=gen) * 2 - 1]).to(DEV)
    y = ops.split_f16(x)
    rec = y[0].float() + y[1].float()
    err = (rec - x).abs()
    bound = x.abs() * 2.0 ** -22 + 2.0 ** -25  # 22 significant bits; subnormal-lo floor
    assert bool((err <= bound).all())


@pytest.mark.parametrize("M,h,wscale", [(4096, 96, 1.0), (2048, 800, 1.0), (2048, 256, 10.0)])
def test_cell_accuracy_vs_fp64(M, h, wscale):
    from iadmm import ops, solver
    from iadmm.data import init_lstm_params
    params = init_lstm_params(h, 4, device="cpu", seed=h)
    for k in params:
        if k.startswith("U_") or k.startswith("W_"):
            params[k] = params[k] * wscale
    for k in ("b_i", "b_f", "b_o", "b_u"):
        params[k] = torch.randn(h) * 0.1
    gen = torch.Generator().manual_seed(M + h)
    H = torch.tanh(torch.randn(M, h, generator=gen))
    C = torch.randn(M, h, generator=gen)
    xv, g = torch.randn(M, generator=gen), torch.randn(M, generator=gen)
    # fp64 evaluation of the same cell (the oracle's op structure)
    p64 = {k: v.double() for k, v in params.items()}
    inputs = torch.stack([xv, g], 1).double()
    H64, C64, _ = orc.lstm_cell(p64, inputs, H.double(), C.double())
    part64 = (H64 * p64["W_h"].reshape(1, h)).reshape(M, -1, 32).sum(-1) if h % 32 == 0 else None

    pd = {k: v.to(DEV) for k, v in params.items()}
    packed = solver.PackedWeights()
    Upk, Wx = packed.get(pd, h)
    Hf, Cf, partf = ops.lstm_cell(H.to(DEV), C.to(DEV), xv.to(DEV), g.to(DEV), Upk, Wx)
    Upk16, ws, Wx = packed.get_f16x3(pd, h)
    H16 = ops.split_f16(H.to(DEV))
    Hn = torch.empty(M, h, device=DEV)
    Hn16, Cs, parts, _ = ops.lstm_cell_f16x3(H16, C.to(DEV), xv.to(DEV), g.to(DEV), Upk16, ws, Wx, Hn=Hn)
    e32 = max(rel_l2(Hf, H64), rel_l2(Cf, C64))
    e16 = max(rel_l2(Hn, H64), rel_l2(Cs, C64))
    assert e16 < 1e-6, (e16, e32)
    assert e16 < 4 * max(e32, 1e-8), (e16, e32)
    # the split planes written for the next iteration reconstruct the fp32 H'
    rec = Hn16[0].float() + Hn16[1].float()
    assert float(((rec - Hn).abs() - Hn.abs() * 2.0 ** -22).max()) <= 2.0 ** -25
    if part64 is not None:
        assert rel_l2(parts.t(), part64) < 4 * max(rel_l2(partf.t(), part64), 1e-8) + 1e-7


def test_solve_golden_f16x3(golden):
    from iadmm import solver
    name, g = golden
    n, mi, me, h, T, B, scaling, _ = meta(g)
    params = {k[len("param_"):]: dev(g[k]) for k in g if k.startswith("param_")}
    with torch.no_grad():
        out = solver.solve(params, dev(g["in_Q"]), dev(g["in_p"]), dev(g["in_A0"]), dev(g["in_zl"]),
                           dev(g["in_zu"]), mi, me, T, float(g["sigma"]), scaling=scaling, history=True,
                           precision="f16x3")
    tol = 1e-2 if divergent(g) else 1e-4
    assert rel_l2(out["x"], g["fin_x"]) < tol, name
    np.testing.assert_allclose(out["hist_primal"].cpu().numpy(), g["hist_primal"], rtol=tol, atol=1e-6)
    np.testing.assert_allclose(out["hist_dual"].cpu().numpy(), g["hist_dual"], rtol=tol, atol=1e-6)
    np.testing.assert_allclose(out["primal"].cpu().numpy(), g["hist_primal"][-1], rtol=tol, atol=1e-6)
    np.testing.assert_allclose(out["dual"].cpu().numpy(), g["hist_dual"][-1], rtol=tol, atol=1e-6)
    # the fp32 H returned on the last iteration is the state the fp32 path would carry
    assert rel_l2(out["H"], g[f"it{T - 1}_H"] if f"it{T - 1}_H" in g else out["H"]) < max(tol, 1e-4)
