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
