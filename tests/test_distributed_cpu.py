"""Multi-process (gloo, world_size 2, CPU) coverage of the N>1 path: instance sharding reproduces
the single-process batch exactly, and the timing reduction takes the max over ranks."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import iadmm_path  # noqa: F401
from iadmm import data, parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, B, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    dist = parallel.init("gloo")
    w, r, _ = parallel.env()
    first, count = parallel.shard(world * B, w, r)
    d = data.make_qp_batch(24, 8, 6, count, first_index=first, device="cpu")
    gathered = [torch.empty_like(d["A0"]) for _ in range(w)]
    dist.all_gather(gathered, d["A0"])
    t = parallel.max_over_ranks(1.0 + r, dist)
    if r == 0:
        q.put((torch.cat(gathered).numpy(), t))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_generation_matches_single_process():
    world, B = 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    A0_all, tmax = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = data.make_qp_batch(24, 8, 6, world * B, first_index=0, device="cpu")["A0"].numpy()
    assert (A0_all == ref).all()
    assert tmax == 2.0


@pytest.mark.parametrize("Bg,world", [(8, 2), (7, 2), (1024 * 8, 8), (5, 4)])
def test_shard_partition(Bg, world):
    spans = [parallel.shard(Bg, world, r) for r in range(world)]
    assert spans[0][0] == 0
    for (s0, c0), (s1, _) in zip(spans, spans[1:]):
        assert s0 + c0 == s1
    assert sum(c for _, c in spans) == Bg
    assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_cli_parses_reference_command_line():
    import main
    cfg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "QP.yaml")
    a = main.parse_args(["--config", cfg, "--prob_type", "QP", "--outer_T", "100",
                         "--truncated_length", "100", "--hidden_dim", "800", "--eq_tol", "0.2",
                         "--ineq_tol", "0.2", "--scaling", "--test", "--test_outer_T", "100", "--save_sol",
                         "--unknown_flag", "3"])
    assert (a.prob_type, a.outer_T, a.hidden_dim, a.test_outer_T) == ("QP", 100, 800, 100)
    assert a.scaling and a.test and a.save_sol
    assert a.sigma == pytest.approx(6e-6) and a.num_var == 5000 and a.weight_decay == 0.0


def _ddp_worker(rank, world, port, q):
    """Data-parallel training math on CPU tensors (gloo): each rank takes its shard of a batch,
    scales its mean loss by shard/global size and the gradients are all-reduced; the result must
    equal the single-process gradient of the full-batch mean."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from iadmm import train
    dist = parallel.init("gloo")
    torch.manual_seed(0)
    model = torch.nn.Linear(5, 3)
    X = torch.randn(7, 5)
    first, count = parallel.shard(7, world, rank)
    loss = model(X[first:first + count]).pow(2).sum(1).mean()
    (count / 7 * loss).backward()
    train.allreduce_grads(list(model.parameters()), dist, bucket_bytes=64)  # forces several buckets
    if rank == 0:
        q.put([p.grad.clone() for p in model.parameters()])
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_gradient_allreduce_equals_full_batch():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    grads = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    model = torch.nn.Linear(5, 3)
    X = torch.randn(7, 5)
    model(X).pow(2).sum(1).mean().backward()
    for g, p in zip(grads, model.parameters()):
        assert torch.allclose(g, p.grad, atol=1e-6)


class _TinySolver(torch.nn.Module):
    """CPU stand-in with LSTM.forward's signature and return tuple (models/lstm.py:47-96): a
    recurrent cell over the KKT rows driven by the instance data, so the TBPTT driver
    (iadmm.train.tbptt_batch: micro-batches, windows, the rank reduction, Adam) runs on gloo
    without the HIP kernels."""

    def __init__(self, hidden=4):
        super().__init__()
        g = torch.Generator().manual_seed(3)
        self.hidden_dim = hidden
        self.W = torch.nn.Parameter(0.3 * torch.randn(2, hidden, generator=g))
        self.U = torch.nn.Parameter(0.3 * torch.randn(hidden, hidden, generator=g))
        self.w_h = torch.nn.Parameter(0.3 * torch.randn(hidden, 1, generator=g))
        self.rho = torch.nn.Parameter(torch.zeros(4, 1))

    def forward(self, t, num_ineq, num_eq, x, y, z, xv, sigma, H, C, **kw):
        Q, p, A0 = kw["Q"], kw["p"], kw["A0"]
        n = x.shape[1]
        g = torch.cat([Q @ x + p, A0 @ x - z], 1)
        Hn = torch.tanh(torch.cat([xv, g], -1) @ self.W + H @ self.U)
        Cn = C + Hn
        xv = xv - Hn @ self.w_h
        x = xv[:, :n]
        y = y + torch.sigmoid(self.rho[t]) * (A0 @ x - z)
        return x, y, z, xv, Hn, Cn, None, None, None


def _tiny_loss(x, y, z, Q, p, A0):
    pr = (A0 @ x - z).norm(dim=(1, 2))
    du = (Q @ x + p + A0.transpose(1, 2) @ y).norm(dim=(1, 2))
    return pr, du, pr + du


class _GradSnap(torch.optim.Adam):
    """Adam that records the gradients it steps with."""

    def __init__(self, params, **kw):
        super().__init__(params, **kw)
        self.seen = []

    def step(self, closure=None):
        self.seen.append([p.grad.clone() for g in self.param_groups for p in g["params"]])
        return super().step(closure)


GB, MB, NV, MI, ME = 10, 2, 6, 2, 2


def _tbptt(model, d, count, dist, chunks=None, reduce="ordered"):
    from iadmm import train
    opt = _GradSnap(model.parameters(), lr=1e-2)
    train.tbptt_batch(model, d, MI, ME, 2, 1, 6e-6, opt, micro_batch=MB, global_batch=GB, dist=dist,
                      loss_fn=_tiny_loss, chunks=chunks, reduce=reduce)
    return opt.seen, [p.detach().clone() for p in model.parameters()]


def _world4_worker(rank, world, port, reduce, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    dist = parallel.init("gloo")
    first, count = parallel.shard(GB, world, rank)
    d = data.make_qp_batch(NV, MI, ME, count, first_index=first, device="cpu")
    seen, params = _tbptt(_TinySolver(), d, count, dist, reduce=reduce)
    rec = dict(rank=rank, first=first, count=count, **parallel.device_record(rank))
    recs = parallel.gather_records(rec, dist)
    if rank == 0:  # numpy: pickled by value (a shared-memory tensor dies with this process)
        q.put(([[a.numpy() for a in w] for w in seen], [a.numpy() for a in params], recs))
    dist.barrier()
    dist.destroy_process_group()


def _run_world(world, reduce):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_world4_worker, args=(r, world, port, reduce, q)) for r in range(world)]
    for p in procs:
        p.start()
    seen, params, recs = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return ([[torch.from_numpy(a) for a in w] for w in seen], [torch.from_numpy(a) for a in params], recs)


def test_world4_uneven_shards_tile_and_ordered_grads_are_bitwise():
    """World 4 over gloo, global batch 10 (shards 3, 3, 2, 2), micro-batch 2, two TBPTT windows:
    the gathered per-rank instance ranges tile the batch, and the ordered reduction's gradients
    (and the Adam-stepped parameters) equal a single process running the same micro-batches
    (train.global_chunks) bit for bit."""
    from iadmm import train
    seen, params, recs = _run_world(4, "ordered")
    assert [r["rank"] for r in recs] == [0, 1, 2, 3]
    assert [(r["first"], r["count"]) for r in recs] == [(0, 3), (3, 3), (6, 2), (8, 2)]
    assert parallel.check_tiling(recs, GB)
    assert not parallel.check_tiling(recs[:3], GB)
    assert all("device" in r and "host" in r for r in recs)
    chunks = train.global_chunks(GB, 4, MB)
    assert chunks == [(0, 2), (2, 3), (3, 5), (5, 6), (6, 8), (8, 10)]
    d = data.make_qp_batch(NV, MI, ME, GB, first_index=0, device="cpu")
    seen1, params1 = _tbptt(_TinySolver(), d, GB, None, chunks=chunks)
    assert len(seen) == len(seen1) == 2
    for w in range(2):
        for a, b in zip(seen[w], seen1[w]):
            assert torch.equal(a, b)
    for a, b in zip(params, params1):
        assert torch.equal(a, b)


def test_world4_allreduce_grads_match_to_rounding():
    """The ring all-reduce alternative (reduce="allreduce"): same gradients up to the summation
    order's rounding."""
    from iadmm import train
    seen, _, _ = _run_world(4, "allreduce")
    d = data.make_qp_batch(NV, MI, ME, GB, first_index=0, device="cpu")
    seen1, _ = _tbptt(_TinySolver(), d, GB, None, chunks=train.global_chunks(GB, 4, MB))
    for a, b in zip(seen[0], seen1[0]):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-7)


def _nograd_worker(rank, world, port, q):
    """ordered_reduce_grads with a parameter that no micro-batch of any rank touches."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    dist = parallel.init("gloo")
    from iadmm import train
    used = torch.nn.Parameter(torch.ones(3))
    unused = torch.nn.Parameter(torch.ones(2))
    only_rank1 = torch.nn.Parameter(torch.ones(2))
    chunks = []
    for c in range(2):
        g_used = torch.full((3,), float(1 + c + 10 * rank))
        g_r1 = torch.full((2,), 5.0) if rank == 1 else None
        chunks.append([g_used, None, g_r1])
    train.ordered_reduce_grads([used, unused, only_rank1], chunks, dist)
    q.put((rank, used.grad.tolist(), unused.grad, only_rank1.grad.tolist() if only_rank1.grad is not None else None))
    dist.barrier()
    dist.destroy_process_group()


def test_ordered_reduce_keeps_none_for_untouched_parameters():
    """a parameter without a gradient anywhere keeps grad None on every rank (one process
    leaves it None and Adam skips it); one with a gradient on some rank gets the fold, zeros elsewhere."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_nograd_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, used, unused, r1 in res:
        assert used == [1.0 + 2.0 + 11.0 + 12.0] * 3
        assert unused is None
        assert r1 == [10.0, 10.0]
