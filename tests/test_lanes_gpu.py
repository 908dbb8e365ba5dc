"""Multi-lane solve (solver.solve(lanes=L): the batch split into L instance groups iterated on L HIP
streams at once) against the single-lane solve.

Every kernel of the iteration is batch-invariant (the residual matvec sums its column partials in
a fixed 256-row-block order, the cell and the update are per row / per instance), so the lanes
must give BITWISE the single-lane result, for the fp32 path and the optional f16x3 path, with
even and uneven lane sizes.
"""
import pytest
import torch

import iadmm_path  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def batch():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from iadmm import data
    d = data.make_qp_batch(300, 100, 60, 7, first_index=11, device="cuda")
    params = data.init_lstm_params(64, 8, device="cuda", seed=5)
    return d, params


def _solve(d, params, lanes, precision="f32"):
    from iadmm import solver
    with torch.no_grad():
        out = solver.solve(params, d["Q"], d["p"], d["A0"], d["zl"], d["zu"], 100, 60, 8, 6e-6, lanes=lanes,
                           precision=precision)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("precision", ["f32", "f16x3"])
@pytest.mark.parametrize("lanes", [2, 3, 7])
def test_lanes_bitwise_equal_single_lane(batch, lanes, precision):
    d, params = batch
    ref = _solve(d, params, 1, precision)
    out = _solve(d, params, lanes, precision)
    for k in ("x", "y", "z", "xv", "H", "C", "primal", "dual", "obj"):
        assert torch.equal(out[k], ref[k]), f"{k} differs with {lanes} lanes ({precision})"


def test_lanes_timer_spans(batch):
    """One cell / KKT span per lane and iteration; busy time <= summed time."""
    from iadmm import solver
    d, params = batch
    tm = solver.Timer(True)
    with torch.no_grad():
        solver.solve(params, d["Q"], d["p"], d["A0"], d["zl"], d["zu"], 100, 60, 8, 6e-6, lanes=2, timer=tm)
    n, mean = tm.stats_ms("k:lstm_cell")
    assert n == 16
    busy = tm.busy_ms("k:lstm_cell")
    # busy_ms works on ref-relative event times, stats_ms on direct span times: each may round
    # differently at the events' microsecond resolution
    assert 0 < busy <= n * mean + n * 2e-3
