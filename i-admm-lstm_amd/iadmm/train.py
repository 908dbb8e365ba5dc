"""Training driver: TBPTT over the unrolled solve (main.py:325-358) with microbatching and
data-parallel gradient all-reduce.

The loss of one batch is sum_t mean_b(primal_b + dual_b) / outer_T (main.py:346-347).  Because it
is a batch MEAN of per-instance terms and instances are independent, splitting the batch into
microbatches (memory) and across ranks (one process per GPU) is exact: each piece contributes
(its size / global batch) x its own mean, and the gradients are summed.

Summation order (r04).  On one process autograd accumulates the micro-batch gradients G_c as a
left fold ((G_0 + G_1) + G_2) + ... in micro-batch order.  Across ranks the default reduction
(``reduce="ordered"``) continues that same fold over the global micro-batch order: rank r receives
the prefix sum of ranks < r from rank r-1, adds its own G_c one by one, sends the new prefix to
rank r+1, and the last rank broadcasts the total (per <= 32 MB bucket, point-to-point RCCL over
xGMI: W-1 hops of 10.3 MB at h=800, T=100 -- about a millisecond per optimiser step against a
16-s window).  The gradients are therefore bitwise those of a single process running the same
micro-batches, for any world size.  ``reduce="allreduce"`` is the ring all-reduce of the
flattened buckets (its summation order depends on the world size and the backend's algorithm).
"""
from __future__ import annotations

import torch

from .parallel import shard


def flat_grads(params):
    return torch.cat([p.grad.reshape(-1) if p.grad is not None else torch.zeros_like(p).reshape(-1) for p in params])


ALLREDUCE_CALLS = 0  # gradient buckets reduced over ranks by this process (bench_train.py reports it)


def _buckets(params, bucket_bytes):
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
    return buckets


def _dist_active(dist):
    from . import parallel
    if dist is None or not dist.is_initialized():
        return False
    return dist.get_world_size() > 1 or parallel.want_dist(1)


def ordered_reduce_grads(params, chunk_grads, dist, bucket_bytes=32 << 20):
    """Sum the per-micro-batch gradients of every rank as ONE left fold in global micro-batch order
    (module docstring) and write the total into ``p.grad`` of every rank.

    ``chunk_grads``: this rank's micro-batch gradients in its order, each a list of per-parameter
    tensors (None = no gradient) aligned with ``params``.  Rank r's micro-batches follow rank r-1's
    in the global order (contiguous shards, parallel.shard).  A parameter that got no gradient in
    any micro-batch of any rank keeps ``grad = None``, as in one process (so Adam skips it instead
    of applying weight decay and moment updates to a zero gradient): a per-parameter count of the
    micro-batches that produced a gradient rides at the end of the last bucket's fold (ADVICE r05:
    no collective of its own)."""
    global ALLREDUCE_CALLS
    world, rank = dist.get_world_size(), dist.get_rank()
    params = list(params)
    if not params:
        return
    index = {id(p): i for i, p in enumerate(params)}
    P = len(params)
    ref0 = params[0]
    mask = torch.tensor([float(sum(g[i] is not None for g in chunk_grads)) for i in range(P)],
                        dtype=ref0.dtype, device=ref0.device)
    buckets = _buckets(params, bucket_bytes)
    totals = []
    for bi, bucket in enumerate(buckets):
        last = bi == len(buckets) - 1
        ids = [index[id(q)] for q in bucket]
        numel = sum(q.numel() for q in bucket)
        extra = P if last else 0
        ref = bucket[0]
        acc = None
        if rank > 0:
            acc = torch.empty(numel + extra, dtype=ref.dtype, device=ref.device)
            dist.recv(acc, src=rank - 1)
        for g in chunk_grads:
            flat = torch.cat([(g[i] if g[i] is not None else torch.zeros_like(params[i])).reshape(-1) for i in ids])
            if acc is None:
                acc = torch.cat([flat, torch.zeros(extra, dtype=ref.dtype, device=ref.device)]) if extra else flat
            else:
                acc[:numel] = acc[:numel] + flat
        if acc is None:  # rank 0 without instances (global batch < world)
            acc = torch.zeros(numel + extra, dtype=ref.dtype, device=ref.device)
        if extra:
            acc[numel:] += mask
        if rank < world - 1:
            dist.send(acc, dst=rank + 1)
        dist.broadcast(acc, src=world - 1)
        ALLREDUCE_CALLS += 1
        totals.append((bucket, acc))
    got = totals[-1][1][-P:].cpu().tolist()  # (one D2H; the window's loss read syncs anyway)
    for bucket, acc in totals:
        off = 0
        for q in bucket:
            if not got[index[id(q)]]:
                q.grad = None
            else:
                if q.grad is None:
                    q.grad = torch.empty_like(q)
                q.grad.copy_(acc[off:off + q.numel()].view_as(q))
            off += q.numel()


def allreduce_grads(params, dist, bucket_bytes=32 << 20):
    """Sum every parameter gradient over ranks: gradients are packed into contiguous buckets of
    at most ``bucket_bytes`` (one bucket at the reference's parameter count), all-reduced, and
    copied back (fixed order, so every rank ends with bitwise identical gradients).  A world-1
    group runs the collective too when IADMM_FORCE_DIST=1 (parallel.want_dist)."""
    global ALLREDUCE_CALLS
    if not _dist_active(dist):
        return
    params = [p for p in params if p.requires_grad]
    for p in params:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    for bucket in _buckets(params, bucket_bytes):
        flat = torch.cat([q.grad.reshape(-1) for q in bucket])
        dist.all_reduce(flat)
        ALLREDUCE_CALLS += 1
        off = 0
        for q in bucket:
            q.grad.copy_(flat[off:off + q.numel()].view_as(q.grad))
            off += q.numel()


def global_chunks(global_batch, world, micro_batch=None):
    """The micro-batches of a global batch as the ranks run them: each rank's contiguous shard
    (parallel.shard) cut into ``micro_batch``-sized pieces, as global [(s, e)] in global order.  A
    single process given these boundaries (``tbptt_batch(chunks=...)``) computes bitwise the
    gradients of the ``world``-rank run under the ordered reduction."""
    out = []
    for r in range(world):
        first, count = shard(global_batch, world, r)
        mb = count if not micro_batch else min(micro_batch, count)
        out += [(first + s, first + min(count, s + mb)) for s in range(0, count, max(mb, 1))]
    return out


def tbptt_batch(model, data, num_ineq, num_eq, outer_T, truncated_length, sigma, optimizer,
                micro_batch=None, global_batch=None, dist=None, loss_fn=None, final=None, chunks=None,
                reduce="ordered"):
    """Train on one (already scaled) batch: ``outer_T // truncated_length`` windows, each ending
    in one optimiser step, like main.py:336-358 (t restarts at 0 in every window, as there).

    ``data`` = dict(Q, p, A0, zl, zu) of this rank's instances; ``global_batch`` = instances over
    all ranks (default: this rank's).  Returns the mean training loss of the last window; a dict
    passed as ``final`` receives this rank's last (scaled) iterate x [B,n,1] (the epoch report's
    Train_Obj / violations, main.py:362-379).  ``chunks``: explicit micro-batch boundaries [(s, e)]
    over this rank's instances (default: consecutive ``micro_batch``-sized pieces); ``reduce``:
    "ordered" (bitwise world-size invariant, default) or "allreduce" across ranks."""
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
    if chunks is None:
        chunks = [(s, min(B, s + mb)) for s in range(0, B, mb)]
    chunks = [(int(s), int(e)) for s, e in chunks]
    if reduce not in ("ordered", "allreduce"):
        raise ValueError(f"reduce must be 'ordered' or 'allreduce', got {reduce!r}")
    ordered = reduce == "ordered" and _dist_active(dist)
    states = {}
    for s, e in chunks:
        b = e - s
        states[s] = [torch.zeros(b, n, 1, device=dev), torch.zeros(b, m, 1, device=dev),
                     torch.zeros(b, m, 1, device=dev), torch.zeros(b, n + m, 1, device=dev),
                     torch.zeros(b, n + m, h, device=dev), torch.zeros(b, n + m, h, device=dev)]
    last = 0.0
    params = [q for q in model.parameters() if q.requires_grad]
    for _ in range(int(outer_T / truncated_length)):
        optimizer.zero_grad(set_to_none=True)  # the first micro-batch's gradient is then taken as is
        window_loss = torch.zeros((), device=dev)
        chunk_grads = []
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
            if ordered:  # keep each micro-batch's gradient apart for the global-order fold
                chunk_grads.append([q.grad for q in params])
                for q in params:
                    q.grad = None
        if ordered:
            ordered_reduce_grads(params, chunk_grads, dist)
        else:
            allreduce_grads(params, dist)
        if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(window_loss)
        optimizer.step()
        last = float(window_loss)
    if final is not None:
        final["x"] = torch.cat([states[s][0] for s, _ in chunks])
    return last


__all__ = ["allreduce_grads", "ordered_reduce_grads", "tbptt_batch", "flat_grads", "shard", "global_chunks"]
