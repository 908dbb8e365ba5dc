"""Training-step benchmark (BASELINE config 5 shape per GPU): one TBPTT window of the reference's
training loop (main.py:336-358) = outer_T forward iterations + loss + backward through all of them
+ gradient all-reduce + Adam step, on synthetic QPs.  Reports instances/s of optimizer-step work
and the per-kernel time split from rocprof-compatible hipEvents.  Not the headline metric
(bench.py is); this measures row a12.

  python bench_train.py --batch 32 --micro_batch 32 --outer_T 100      # per GPU
  python bench_train.py --gpus 8 --batch 512 --micro_batch 128      # starts 8 ranks itself
  python -m torch.distributed.run --nproc-per-node 8 bench_train.py --gpus 8 --batch 512 --micro_batch 128
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def launch_ranks(args):
    """N > 1 ranks without a launcher: torch.distributed.run child (iadmm/launch.py, loaded by
    path before anything touches the GPU), exit with its status; see bench.launch_ranks."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "iadmm_launch", os.path.join(ROOT, "i-admm-lstm_amd", "iadmm", "launch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.relaunch(os.path.abspath(sys.argv[0]), sys.argv[1:], args.gpus)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); started here when no launcher did")
    ap.add_argument("--batch", type=int, default=32, help="instances per GPU")
    ap.add_argument("--micro_batch", type=int, default=32)
    ap.add_argument("--num_var", type=int, default=1000)
    ap.add_argument("--num_ineq", type=int, default=500)
    ap.add_argument("--num_eq", type=int, default=500)
    ap.add_argument("--hidden_dim", type=int, default=800)
    ap.add_argument("--outer_T", type=int, default=100)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reduce", choices=("ordered", "allreduce"), default="ordered",
                    help="gradient reduction over ranks (iadmm/train.py): the ordered fold (bitwise "
                         "world-size invariant) or the ring all-reduce")
    args = ap.parse_args()
    launch_ranks(args)
    from iadmm import data, ops, parallel, train
    from models.lstm import LSTM
    world, rank, local = parallel.env()
    local, backend = parallel.device_and_backend(local)
    torch.cuda.set_device(local)
    dist = parallel.init(backend, local) if parallel.want_dist(world) else None
    n, mi, me, h, T, B = args.num_var, args.num_ineq, args.num_eq, args.hidden_dim, args.outer_T, args.batch
    first, count = parallel.shard(world * B, world, rank)
    d = data.make_qp_batch(n, mi, me, count, first_index=first, device="cuda")
    Qs, ps, As, zls, zus, _, _, _ = ops.ruiz_scale(d["Q"], d["p"], d["A0"], d["zl"], d["zu"], 10)
    d = dict(Q=Qs, p=ps, A0=As, zl=zls, zu=zus)
    torch.manual_seed(17)
    model = LSTM(mi + me, 2, h, T, "cuda")
    opt = torch.optim.Adam(model.parameters(), lr=5e-5)

    def step():
        return train.tbptt_batch(model, d, mi, me, T, T, 6e-6, opt, micro_batch=args.micro_batch,
                                 global_batch=world * B, dist=dist, reduce=args.reduce)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    el = 0.0
    step_s = []
    for _ in range(args.steps):
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loss = step()
        torch.cuda.synchronize()
        step_s.append(time.perf_counter() - t0)
        el += step_s[-1]
    ranks = parallel.gather_records(dict(rank=rank, first=first, count=count, elapsed_s=el, step_s=step_s,
                                         **parallel.device_record(local)), dist)
    el = parallel.max_over_ranks(el, dist, device="cuda")
    if rank == 0:
        N = n + mi + me
        fwd_flop = (8.0 * N * h * h + 18.0 * N * h) * B * T
        print(json.dumps({"metric": "training instances/s (one optimizer step = T-iteration TBPTT window)",
                          "value": world * B * args.steps / el, "ms_per_step": 1e3 * el / args.steps,
                          "n_gpus": world, "batch_per_gpu": B, "micro_batch": args.micro_batch, "outer_T": T,
                          "hidden_dim": h, "loss": loss,
                          "cell_gemm_tflops_equiv": 4 * fwd_flop * args.steps / el / 1e12,
                          "dist_backend": dist.get_backend() if dist else None,
                          "allreduce_calls": train.ALLREDUCE_CALLS, "reduce": args.reduce,
                          "ranks": ranks, "ranks_tile_batch": parallel.check_tiling(ranks, world * B),
                          "note": "cell GEMM work per step = forward + recompute + dH + dU = 4x forward flops"}))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
