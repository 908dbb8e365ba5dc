"""The C-ABI's stated contract (include/iadmm.h "Conventions"):
stream-ordered calls that are safe to capture in a hipGraph and to call from several threads on
distinct streams, and run-to-run determinism of the kernels whose stores go through LDS stages.

* Stage II (models/lu.py:26-35): ``ops.lu_factor`` + ``ops.lu_solve`` captured with
  ``torch.cuda.graph`` and replayed -- factors, pivots and solutions bitwise those of eager runs (N = 2000
  paired blocks; N = 2500 rank-128 blocks with the look-ahead's side stream forked from the capturing
  stream; N = 2000 at B = 512, the batch split's two streams; r06: captured graphs keep the eager
  schedule's concurrency, tools/capture_probe.hip);
* two Python threads factoring different batches on two streams at the same time, each with its own
  look-ahead context -- bitwise the serial results;
* the look-ahead (context) path bitwise equal to the single-stream path (NULL context), for the
  paired-block default and for IADMM_LU_RANK128, and the batch split over the context's two streams
  (B >= 512) bitwise equal to one stream;
* repeat runs bitwise equal: the LU at N = 2000, B = 4 (look-ahead + LDS-staged panels), and the
  cell backward (its dP stores staged through LDS, csrc/train.hip) at the config-5 width.
"""
import threading

import pytest
import torch

import iadmm_path  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _kkt_like(B, N, seed):
    """Random dense matrices with a zero (1,1) entry and a weak diagonal: real interchanges in every
    block."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    K = torch.randn(B, N, N, generator=g, device="cuda")
    K[:, 0, 0] = 0.0
    return K, torch.randn(B, N, generator=g, device="cuda")


def _factor_solve(K, b, lookahead=True, flags=0):
    from iadmm import ops
    LU, piv, info = ops.lu_factor(K.clone(), lookahead=lookahead, flags=flags)
    x = ops.lu_solve(LU, piv, b)
    return LU, piv, info, x


def _same(a, b):
    return all(torch.equal(u, v) for u, v in zip(a, b))


def _diff(a, b):
    """Which of (LU, piv, info, x) differ, and by how much (for the failure message)."""
    out = {}
    for name, u, v in zip(("LU", "piv", "info", "x"), a, b):
        if not torch.equal(u, v):
            ne = (u != v)
            out[name] = (int(ne.sum()), float((u.double() - v.double()).abs().max()),
                         tuple(int(i) for i in ne.nonzero()[0].tolist()))
    return out


@pytest.mark.timeout(300)
@pytest.mark.parametrize("rank128", [False, True])
def test_lu_repeat_and_lookahead_bitwise(rank128):
    """N = 2000: the paired-block default (one stream) and the rank-128 blocks (look-ahead on the
    context's streams)."""
    from iadmm import ops
    fl = ops.LU_RANK128 if rank128 else 0
    K, b = _kkt_like(4, 2000, 11)
    r0 = _factor_solve(K, b, flags=fl)
    r1 = _factor_solve(K, b, flags=fl)
    r2 = _factor_solve(K, b, lookahead=False, flags=fl)
    torch.cuda.synchronize()
    assert int(r0[2].abs().max()) == 0
    assert _same(r0, r1), ("LU not deterministic across runs", _diff(r0, r1))
    assert _same(r0, r2), ("look-ahead path differs from the single-stream path", _diff(r0, r2))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("N,B", [(2000, 4), (2500, 4), (2000, 512)])
def test_lu_graph_capture_replay_bitwise(N, B):
    """N = 2000: paired blocks; N = 2500: rank-128 blocks with the look-ahead (its side stream forked
    from the capturing stream); B = 512: the batch split over the context's two streams."""
    from iadmm import ops
    K, b = _kkt_like(B, N, 12)
    eager = _factor_solve(K, b)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    Ks, bs = K.clone(), b.clone()
    ws = ops.lu_factor_ws(B, N, K.device)
    with torch.cuda.stream(s):  # warm-up on the capture stream (makes its look-ahead context)
        A = Ks.clone()
        ops.lu_factor(A, ws=ws)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        A = Ks.clone()
        LU, piv, info = ops.lu_factor(A, ws=ws)
        x = ops.lu_solve(LU, piv, bs)
    Ks.zero_()  # replay must read the current inputs
    bs.zero_()
    torch.cuda.synchronize()
    for _ in range(2):
        Ks.copy_(K)
        bs.copy_(b)
        g.replay()
        torch.cuda.synchronize()
        assert _same((LU, piv, info, x), eager), ("graph replay differs from eager", _diff((LU, piv, info, x), eager))
    # a second input through the same graph
    K2, b2 = _kkt_like(B, N, 13)
    ref2 = _factor_solve(K2, b2)
    Ks.copy_(K2)
    bs.copy_(b2)
    g.replay()
    torch.cuda.synchronize()
    assert _same((LU, piv, info, x), ref2), _diff((LU, piv, info, x), ref2)


@pytest.mark.timeout(300)
def test_lu_batch_split_bitwise():
    """B >= 512 at N <= 2048 with a context: the two halves (256 + 257 here) are factored on the
    context's two streams (csrc/lu.hip iadmm_lu_factor_ex) -- bitwise the one-stream factorization."""
    K, b = _kkt_like(513, 2000, 31)
    split = _factor_solve(K, b)
    one = _factor_solve(K, b, lookahead=False)
    torch.cuda.synchronize()
    assert int(split[2].abs().max()) == 0
    assert _same(split, one), ("batch-split factorization differs from one stream", _diff(split, one))


@pytest.mark.timeout(300)
def test_lu_two_threads_two_streams_bitwise():
    ins = [_kkt_like(8, 2500, 20 + i) for i in range(2)]  # (N > 2048: rank-128 blocks, look-ahead contexts)
    serial = [_factor_solve(K, b) for K, b in ins]
    torch.cuda.synchronize()
    out = [None, None]
    errs = []
    start = threading.Barrier(2)

    def work(i):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                start.wait()
                res = [_factor_solve(*ins[i]) for _ in range(3)]
            s.synchronize()
            out[i] = res
        except Exception as e:  # reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    assert not errs, errs
    for i in range(2):
        for r in out[i]:
            assert _same(r, serial[i]), f"thread {i} differs from the serial run"


@pytest.mark.timeout(300)
def test_cell_backward_repeat_bitwise():
    """iadmm_lstm_cell_bwd twice on the same inputs (config-5 micro-batch width: M = 128 x 2000 rows,
    h = 800): dC, dP (stored through LDS), the W_h slab and the input partials bitwise equal."""
    from iadmm import data, ops
    h, M = 800, 128 * 2000
    p = data.init_lstm_params(h, 100, device="cuda")
    p = {k: v * 20 for k, v in p.items()}  # larger gates than the 0.01 init: every branch active
    Upk, Wx = ops.lstm_pack(p, h)
    g = torch.Generator(device="cuda").manual_seed(5)
    H = torch.randn(M, h, device="cuda", generator=g)
    C = torch.randn(M, h, device="cuda", generator=g)
    xv = torch.randn(M, device="cuda", generator=g)
    gr = torch.randn(M, device="cuda", generator=g)
    dq = torch.randn(M, device="cuda", generator=g)
    dHn = torch.randn(M, h, device="cuda", generator=g)
    dCn = torch.randn(M, h, device="cuda", generator=g)
    r0 = ops.lstm_cell_bwd(H, C, xv, gr, Upk, Wx, dq, dHn, dCn)
    r1 = ops.lstm_cell_bwd(H, C, xv, gr, Upk, Wx, dq, dHn, dCn)
    torch.cuda.synchronize()
    assert all(bool(torch.isfinite(t).all()) for t in r0)
    assert _same(r0, r1), "cell backward not deterministic across runs"


@pytest.mark.timeout(300)
def test_lu_bench_shape_repeat_bitwise():
    """the bench's Stage-II shape (B = 1024, N = 2000: paired rank-256 blocks, the
    batch split over the context's two streams, every CU holding two co-resident workgroups of each
    LDS-staged kernel) factored twice in one process -- factors, pivots and info bitwise equal; and
    once more on one stream (NULL context), bitwise equal too."""
    from iadmm import ops
    B, N = 1024, 2000
    g = torch.Generator(device="cuda").manual_seed(21)
    K = torch.randn(B, N, N, generator=g, device="cuda")
    K[:, 0, 0] = 0.0
    ws = ops.lu_factor_ws(B, N, K.device)
    outs = []
    for lookahead in (True, True, False):
        A = K.clone()
        LU, piv, info = ops.lu_factor(A, ws=ws, lookahead=lookahead)
        torch.cuda.synchronize()
        outs.append((LU, piv.clone(), info.clone()))
        del A
    assert int(outs[0][2].abs().max()) == 0
    for i in (1, 2):
        if not _same(outs[0], outs[i]):
            bad = (outs[0][0] != outs[i][0]).flatten(1).any(1).nonzero().flatten().tolist()
            pytest.fail(f"run {i} differs from run 0 on {len(bad)} instances (first {bad[:8]}): "
                        f"{_diff(outs[0], outs[i])}")
