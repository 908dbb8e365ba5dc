"""The fused LSTM-cell kernel (iadmm_lstm_cell_fwd) against an fp64 restatement of
models/lstm.py:74-80, over the shapes that select its code paths:

* h % 4 == 0 -> LDS-DMA main loop (cell_tile.h cell_mainloop_dma); h % 16 != 0 exercises the
  partial last 16-deep chunk, h < 16 a single chunk;
* h % 4 != 0 -> register-staged 32-deep main loop (cell_mainloop<false>);
* M not a multiple of the 256-row tile (rows past M must read as zero and not be written).

Tolerance: fp32 accumulation over h products plus <= 3.1 ulp transcendentals
(profiles/r01_mathcheck.txt), far below 1e-5 relative at these sizes.
"""
import pytest
import torch

GATES = "ifou"


def _params(h, scale, gen):
    p = {}
    for k in GATES:
        p["W_" + k] = torch.randn(2, h, generator=gen) * scale
        p["U_" + k] = torch.randn(h, h, generator=gen) * scale
        p["b_" + k] = torch.randn(h, generator=gen) * scale
    p["W_h"] = torch.randn(h, 1, generator=gen) * scale
    return p


def _cell_fp64(p, H, C, xv, g):
    """models/lstm.py:74-80 in fp64: gates, C' = I U + F C, H' = O tanh(C'), q = H' W_h."""
    d = {k: v.double() for k, v in p.items()}
    inp = torch.stack([xv.double(), g.double()], dim=1)
    Hd, Cd = H.double(), C.double()
    gate = {k: inp @ d["W_" + k] + Hd @ d["U_" + k] + d["b_" + k] for k in GATES}
    i, f, o = (torch.sigmoid(gate[k]) for k in "ifo")
    u = torch.tanh(gate["u"])
    Cn = i * u + f * Cd
    Hn = o * torch.tanh(Cn)
    return Hn, Cn, (Hn @ d["W_h"]).squeeze(1)


def rel(a, b):
    return float((a.double().cpu() - b).norm() / b.norm().clamp_min(1e-300))


@pytest.mark.gpu
# h % 16 == 0 runs the VALU-free K16 loop: h = 16 (one chunk), 48 / 800 / 80 / 112 (head paths
# (h/16 - 1) % 3 = 2 / 1 / 1 / 0) and partial hidden tiles (h % 32 = 16: the buffer epilogue's tail)
@pytest.mark.parametrize("M,h", [(700, 48), (257, 40), (64, 8), (300, 36), (513, 13), (100, 30), (1000, 800),
                                 (700, 16), (513, 64), (300, 112), (257, 80)])
def test_cell_matches_fp64(M, h):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from iadmm import ops
    gen = torch.Generator().manual_seed(M * 7 + h)
    p = _params(h, 0.3 / h ** 0.5 * 4, gen)
    H = torch.tanh(torch.randn(M, h, generator=gen))
    C = torch.randn(M, h, generator=gen)
    xv, g = torch.randn(M, generator=gen), torch.randn(M, generator=gen)
    dev = {k: v.cuda() for k, v in p.items()}
    Upk, Wx = ops.lstm_pack(dev, h)
    Hn, Cn, part = ops.lstm_cell(H.cuda(), C.cuda(), xv.cuda(), g.cuda(), Upk, Wx)
    torch.cuda.synchronize()
    Href, Cref, qref = _cell_fp64(p, H, C, xv, g)
    assert rel(Hn, Href) < 1e-5
    assert rel(Cn, Cref) < 1e-5
    assert rel(part.sum(0), qref) < 1e-5          # per-tile projection partials sum to H' W_h
    # deterministic: a second launch is bitwise identical
    Hn2, Cn2, part2 = ops.lstm_cell(H.cuda(), C.cuda(), xv.cuda(), g.cuda(), Upk, Wx)
    assert torch.equal(Hn, Hn2) and torch.equal(Cn, Cn2) and torch.equal(part, part2)


@pytest.mark.gpu
@pytest.mark.parametrize("mag", [1e2, 1e6, 1e30, float("inf")])
def test_cell_saturated_gates(mag):
    """Divergent solves drive xv and g (and so the gate pre-activations) to huge values: the gates
    must saturate to 0 / 1 / -1 like torch.sigmoid / torch.tanh, never produce NaN (the fast exp's
    fma correction once met inf * negative + inf here)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from iadmm import ops
    M, h = 300, 40
    gen = torch.Generator().manual_seed(5)
    p = _params(h, 0.3, gen)
    H = torch.tanh(torch.randn(M, h, generator=gen))
    C = torch.randn(M, h, generator=gen)
    sign = torch.where(torch.rand(M, generator=gen) < 0.5, -1.0, 1.0)
    xv, g = sign * mag, -sign * mag * torch.rand(M, generator=gen)
    dev = {k: v.cuda() for k, v in p.items()}
    Upk, Wx = ops.lstm_pack(dev, h)
    Hn, Cn, part = ops.lstm_cell(H.cuda(), C.cuda(), xv.cuda(), g.cuda(), Upk, Wx)
    torch.cuda.synchronize()
    Href, Cref, _ = _cell_fp64(p, H, C, xv, g)
    ok = torch.isfinite(Cref)            # inf - inf in the fp64 reference's C is not a kernel error
    assert not torch.isnan(Hn.cpu()[ok]).any() and not torch.isnan(Cn.cpu()[ok]).any()
    assert float((Hn.double().cpu() - Href).abs()[ok].max()) < 1e-5
    fin = ok & (Cref.abs() < 1e30)
    assert rel(Cn.cpu()[fin], Cref[fin]) < 1e-5


@pytest.mark.gpu
def test_cell_propagates_nan_like_torch():
    """A NaN gate pre-activation (inf * w0 - inf * w1 when xv and g overflow in a divergent solve)
    or a NaN cell state must come out as NaN like torch.tanh gives it, not as a clamped tanh of
    -7.9 = -1 (the v_med3 clamp returns min3 of its operands for a NaN input): the NaN patterns of
    H' and C' equal the fp64 reference's, and every other entry matches it."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from iadmm import ops
    M, h = 300, 40
    gen = torch.Generator().manual_seed(9)
    p = _params(h, 0.3, gen)
    H = torch.tanh(torch.randn(M, h, generator=gen))
    C = torch.randn(M, h, generator=gen)
    C[7, 3] = float("nan")                      # a NaN cell state
    xv, g = torch.randn(M, generator=gen), torch.randn(M, generator=gen)
    xv[11], g[11] = float("inf"), float("inf")  # pre = inf w0 + inf w1: NaN where w0, w1 differ in sign
    xv[12] = float("nan")                       # NaN input: every gate NaN
    dev = {k: v.cuda() for k, v in p.items()}
    Upk, Wx = ops.lstm_pack(dev, h)
    Hn, Cn, _ = ops.lstm_cell(H.cuda(), C.cuda(), xv.cuda(), g.cuda(), Upk, Wx)
    torch.cuda.synchronize()
    Href, Cref, _ = _cell_fp64(p, H, C, xv, g)
    Hn, Cn = Hn.cpu(), Cn.cpu()
    assert torch.isnan(Href[11]).any() and not torch.isnan(Href[11]).all()  # the case is exercised
    assert torch.equal(torch.isnan(Hn), torch.isnan(Href))
    assert torch.equal(torch.isnan(Cn), torch.isnan(Cref))
    fin = torch.isfinite(Href)
    assert float((Hn.double() - Href).abs()[fin].max()) < 1e-5
