"""Training driver: TBPTT over the unrolled solve (main.py:325-358) with microbatching and
data-parallel gradient all-reduce.

The loss of one batch is sum_t mean_b(primal_b + dual_b) / outer_T (main.py:346-347).  Because it
is a batch MEAN of per-instance terms and instances are independent, splitting the batch into
microbatches (memory) and across ranks (one process per GPU) is exact: each piece contributes
(its size / global batch) x its own mean, and the gradients are summed — locally by autograd
accumulation, across ranks by one all-reduce of the flattened gradient buckets (RCCL over xGMI;
2.57 M fp32 = 10.3 MB at h=800, T=100).
"""
from __future__ import annotations

import torch

from .parallel import shard


def flat_grads(params):
    return torch.cat([p.grad.reshape(-1) if p.grad is not None else torch.zeros_like(p).reshape(-1) for p in params])


ALLREDUCE_CALLS = 0  # gradient buckets all-reduced by this process (bench_train.py reports it)


def allreduce_grads(params, dist, bucket_bytes=32 << 20):
    """Sum every parameter gradient over ranks: gradients are packed into contiguous buckets of
    at most ``bucket_bytes`` (one bucket at the reference's parameter count), all-reduced, and
    copied back (fixed order, so every rank ends with bitwise identical gradients).  A world-1
    group runs the collective too when IADMM_FORCE_DIST=1 (parallel.want_dist)."""
    global ALLREDUCE_CALLS
    from . import parallel
    if dist is None or not dist.is_initialized():
        return
    if dist.get_world_size() == 1 and not parallel.want_dist(1):
        return
    params = [p for p in params if p.requires_grad]
    for p in params:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    buckets, cur, size = [], [], 0
    for p in params:
        nb = p.numel() * p.element_size()
        if cur and size + nb > bucket_bytes:
            buckets.append(cur)
            cur, size = [], 0
        cur.append(p)
        size += nb
    if cur:
        buckets.append(cur)
    for bucket in buckets:
        flat = torch.cat([q.grad.reshape(-1) for q in bucket])
        dist.all_reduce(flat)
        ALLREDUCE_CALLS += 1
        off = 0
        for q in bucket:
            q.grad.copy_(flat[off:off + q.numel()].view_as(q.grad))
            off += q.numel()


def tbptt_batch(model, data, num_ineq, num_eq, outer_T, truncated_length, sigma, optimizer,
                micro_batch=None, global_batch=None, dist=None, loss_fn=None, final=None):
    """Train on one (already scaled) batch: ``outer_T // truncated_length`` windows, each ending
    in one optimiser step, like main.py:336-358 (t restarts at 0 in every window, as there).

    ``data`` = dict(Q, p, A0, zl, zu) of this rank's instances; ``global_batch`` = instances over
    all ranks (default: this rank's).  Returns the mean training loss of the last window; a dict
    passed as ``final`` receives this rank's last (scaled) iterate x [B,n,1] (the epoch report's
    Train_Obj / violations, main.py:362-379)."""
    if loss_fn is None:
        import utils
        loss_fn = utils.primal_dual_loss
    Q, p, A0, zl, zu = (data[k] for k in ("Q", "p", "A0", "zl", "zu"))
    B, n = Q.shape[0], Q.shape[1]
    m = A0.shape[1]
    h = model.hidden_dim
    mb = B if not micro_batch else min(micro_batch, B)
    gB = global_batch or B
    dev = Q.device
    chunks = [(s, min(B, s + mb)) for s in range(0, B, mb)]
    states = {}
    for s, e in chunks:
        b = e - s
        states[s] = [torch.zeros(b, n, 1, device=dev), torch.zeros(b, m, 1, device=dev),
                     torch.zeros(b, m, 1, device=dev), torch.zeros(b, n + m, 1, device=dev),
                     torch.zeros(b, n + m, h, device=dev), torch.zeros(b, n + m, h, device=dev)]
    last = 0.0
    params = [q for q in model.parameters() if q.requires_grad]
    for _ in range(int(outer_T / truncated_length)):
        optimizer.zero_grad()
        window_loss = torch.zeros((), device=dev)
        for s, e in chunks:
            x, y, z, xv, H, C = states[s]
            kw = dict(Q=Q[s:e], p=p[s:e], A0=A0[s:e], lb=None, ub=None, zl=zl[s:e], zu=zu[s:e])
            loss = 0.0
            for t in range(truncated_length):
                x, y, z, xv, H, C, _, _, _ = model(t, num_ineq, num_eq, x, y, z, xv, sigma, H, C, **kw)
                _, _, l = loss_fn(x, y, z, kw["Q"], kw["p"], kw["A0"])
                loss = loss + l.mean() / outer_T
            ((e - s) / gB * loss).backward()
            window_loss += (e - s) / gB * loss.detach()
            states[s] = [v.detach() for v in (x, y, z, xv, H, C)]
        allreduce_grads(params, dist)
        if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(window_loss)
        optimizer.step()
        last = float(window_loss)
    if final is not None:
        final["x"] = torch.cat([states[s][0] for s, _ in chunks])
    return last


__all__ = ["allreduce_grads", "tbptt_batch", "flat_grads", "shard"]
