"""Data-parallel helpers (one process per GPU, torch.distributed over RCCL).

The reference is single-device; the build adds exactly one strategy (SURVEY.md
8e): every rank computes the same global stream from the same seeds and takes a
contiguous shard of each global batch; the gradient exchange is one all-reduce
of the flat gradient bucket (dense tower grads + dense embedding grads), which
keeps dense-Adam parity with the single-device run.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def shard_range(global_rows: int, world: int, rank: int):
    """[lo, hi) of a global batch owned by `rank` -- the same arithmetic as
    ncf_train_step (per = ceil(gb / world))."""
    per = (global_rows + world - 1) // world
    lo = min(rank * per, global_rows)
    return lo, min(lo + per, global_rows)


def allreduce_flat_grads(flat: torch.Tensor, group=None):
    """Sum the flat gradient bucket over ranks (in place)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    return flat


def init_from_env(backend="nccl"):
    """torchrun-style init (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*); 127.0.0.1 default."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, **kw)
    return world, rank, local
