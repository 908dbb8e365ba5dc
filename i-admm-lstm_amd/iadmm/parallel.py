"""Multi-GPU plumbing: one process per GPU, instance-batch sharding, no data-path collective.

QP instances are independent and the LSTM weights are read-only at inference,
so rank r solves the contiguous instance range ``shard(B_global, world, r)``; instance seeds are
global indices, so a shard reproduces exactly the instances a single GPU would solve.  The only
collectives are measurement (barrier, max-over-ranks time) and, for training, the gradient
all-reduce.
"""
from __future__ import annotations

import os

import torch


def env():
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


SHARED_GPU_ENV = "IADMM_SHARED_GPU"


def device_and_backend(local_rank):
    """(cuda device index, backend) of this rank: one GPU per rank over RCCL ("nccl").  With
    IADMM_SHARED_GPU=1 every rank uses cuda:0 over gloo -- a rehearsal of the N>1 code path
    (sharding, barriers, max-over-ranks, gradient all-reduce) on a one-GPU machine; RCCL refuses
    two ranks on one device."""
    if os.environ.get(SHARED_GPU_ENV) == "1":
        return 0, "gloo"
    return int(local_rank), "nccl"


FORCE_DIST_ENV = "IADMM_FORCE_DIST"


def want_dist(world):
    """Initialise a process group: always for world > 1; at world 1 only with IADMM_FORCE_DIST=1
    (exercises the RCCL branch and the gradient all-reduce on a one-GPU box)."""
    return world > 1 or os.environ.get(FORCE_DIST_ENV) == "1"


def shard(global_batch, world, rank):
    """Contiguous [start, start+count) of ``global_batch`` instances for ``rank`` (sizes differ by
    at most one when the batch does not divide)."""
    base, extra = divmod(int(global_batch), int(world))
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def init(backend, local_rank=0):
    import torch.distributed as dist
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend)
    return dist


def max_over_ranks(value, dist=None, device="cpu"):
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t)


def gather_records(rec, dist=None):
    """Every rank's ``rec`` (a small JSON-able dict) in rank order, on every rank
    (all_gather_object; measurement only).  Without a process group: ``[rec]``."""
    if dist is None or not dist.is_initialized():
        return [rec]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, rec)
    return out


def device_record(local_rank):
    """Which GPU this rank runs on: name, PCI location and UUID of ``cuda:local_rank``, the
    process's HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES, and the host name."""
    import socket
    rec = {"local_rank": int(local_rank), "host": socket.gethostname()}
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if os.environ.get(k) is not None:
            rec[k] = os.environ[k]
    if torch.cuda.is_available():
        p = torch.cuda.get_device_properties(local_rank)
        rec["device"] = p.name
        rec["pci"] = "{:04x}:{:02x}:{:02x}".format(getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", 0),
                                                   getattr(p, "pci_device_id", 0))
        rec["uuid"] = str(getattr(p, "uuid", ""))
        rec["cus"] = int(p.multi_processor_count)
    else:
        rec["device"] = "cpu"
    return rec


def check_tiling(records, global_batch):
    """The gathered instance ranges (``first``, ``count`` per rank record) tile [0, global_batch)
    in rank order with no gap or overlap."""
    pos = 0
    for r in sorted(records, key=lambda r: r["rank"]):
        if r["first"] != pos or r["count"] < 0:
            return False
        pos += r["count"]
    return pos == global_batch
