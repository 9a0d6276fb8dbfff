"""Data-parallel helpers (one process per GPU, torch.distributed over RCCL).

The reference is single-device; the build adds one strategy:
every rank computes the same global stream from the same seeds and takes a
contiguous shard of each global batch.  The gradient exchange forms
(``TrainEngine(dp_mode=...)``; "touched" is engine-side, ncf_touched_pack):

* ``"zero1"`` (default for world > 1): the flat gradient bucket (dense
  embedding tables + tower + predict, zero padded to world x shard floats) is
  reduce-scattered, each rank runs Adam on its own contiguous shard of the
  flat parameters (its moments are shard-sized), and the updated parameters
  are all-gathered in place.  Same bytes on the wire as one all-reduce, 1/W
  of the optimizer's HBM traffic and moment memory per rank.
* ``"allreduce"``: one all-reduce of the flat gradient bucket, replicated Adam.
* ``"owner"``: embedding row id owned by rank id % W; the touched rows' gradients go
  to their owners and the rows each rank's next batch reads come back, two
  fixed-size all-to-alls per step (device kernels ncf_owner_*, engine.py);
  ``owner_gather_rows`` brings every replica up to date at the end of a run.

All keep dense-Adam parity with the single-device run (Adam is elementwise).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

ALIGN = 64  # floats: flat-buffer segments and shards start 256-byte aligned


def shard_range(global_rows: int, world: int, rank: int):
    """[lo, hi) of a global batch owned by `rank` -- the same arithmetic as
    ncf_train_step (per = ceil(gb / world))."""
    per = (global_rows + world - 1) // world
    lo = min(rank * per, global_rows)
    return lo, min(lo + per, global_rows)


def shard_floats(total: int, world: int, align: int = ALIGN) -> int:
    """Floats per rank of the flat buffer under the sharded optimizer: the
    smallest multiple of `align` with world * shard >= total."""
    per = (int(total) + world - 1) // world
    return max(align, (per + align - 1) // align * align)


def shard_ranges(ranges, world: int, rank: int, shard: int):
    """Active [begin, end) float ranges of the flat buffer that fall inside rank's
    shard [rank*shard, (rank+1)*shard), shifted to shard-local offsets."""
    lo, hi = rank * shard, (rank + 1) * shard
    out = []
    for b, e in ranges:
        b2, e2 = max(int(b), lo), min(int(e), hi)
        if e2 > b2:
            out.append([b2 - lo, e2 - lo])
    return out


def _native_ok(t: torch.Tensor, group) -> bool:
    """reduce_scatter_tensor / all_gather_into_tensor straight on the backend:
    always for RCCL ('nccl'); gloo only for host tensors.  gloo with device
    tensors (the single-GPU multi-rank test) goes through exact all-reduce
    forms instead."""
    if os.environ.get("NCF_DP_EMULATE", "0") == "1":
        return False
    return dist.get_backend(group) != "gloo" or t.device.type == "cpu"


def allreduce_flat_grads(flat: torch.Tensor, group=None):
    """Sum the flat gradient bucket over ranks (in place)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    return flat


def reduce_scatter_flat(out: torch.Tensor, inp: torch.Tensor, rank: int, group=None):
    """out[:] = (sum over ranks of inp)[rank*S:(rank+1)*S], S = out.numel()."""
    s = out.numel()
    if _native_ok(inp, group):
        dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group)
    else:
        dist.all_reduce(inp, op=dist.ReduceOp.SUM, group=group)
        out.copy_(inp[rank * s:(rank + 1) * s])
    return out


def all_gather_flat(flat: torch.Tensor, rank: int, shard: int, group=None, scratch=None):
    """In-place all-gather: every rank contributes flat[rank*S:(rank+1)*S]."""
    mine = flat[rank * shard:(rank + 1) * shard]
    if _native_ok(flat, group):
        dist.all_gather_into_tensor(flat, mine, group=group)
    else:
        # exact: every other contribution is +0.0
        tmp = scratch if scratch is not None else torch.empty_like(flat)
        tmp.zero_()
        tmp[rank * shard:(rank + 1) * shard].copy_(mine)
        dist.all_reduce(tmp, op=dist.ReduceOp.SUM, group=group)
        flat.copy_(tmp)
    return flat


def _coll_ok(t, group):
    """Run the collective on `t` where it lives (RCCL: device tensors; gloo: host)."""
    return dist.get_backend(group) != "gloo" or t.device.type == "cpu"


def _all_reduce(t, group):
    if _coll_ok(t, group):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return t
    h = t.cpu()
    dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
    t.copy_(h)
    return t


def capturable(t: torch.Tensor, group) -> bool:
    """Collectives on `t` can sit inside a captured hipGraph: RCCL on device tensors."""
    return group is not None and dist.get_backend(group) != "gloo" and t.device.type == "cuda"


def all_to_all_equal(out: torch.Tensor, inp: torch.Tensor, group=None):
    """out[r-th chunk] = rank r's inp[this rank's chunk], equal chunks (RCCL: one
    all_to_all_single; gloo with device tensors: through host copies)."""
    if _coll_ok(inp, group):
        dist.all_to_all_single(out, inp, group=group)
        return out
    o = torch.empty(out.shape, dtype=out.dtype)
    dist.all_to_all_single(o, inp.cpu(), group=group)
    out.copy_(o)
    return out


def owner_gather_rows(flat: torch.Tensor, tables, world: int, rank: int, group=None):
    """dp_mode "owner": every rank's owned rows (id % world == rank) of each table to
    every rank, in place.  tables: [(flat offset, row width, rows)].  One all-gather of
    the rows this rank owns, padded to ceil(rows / world) per table."""
    dev = flat.device
    pers = [(n + world - 1) // world for _, _, n in tables]
    size = sum(p * w for p, (_, w, _) in zip(pers, tables))
    mine = torch.zeros(size, dtype=flat.dtype, device=dev)
    pos = 0
    for p, (off, w, n) in zip(pers, tables):
        t = flat[off:off + n * w].view(n, w)
        own = t[rank::world]
        mine[pos:pos + own.numel()].copy_(own.reshape(-1))
        pos += p * w
    if _coll_ok(mine, group):
        out = torch.empty(world * size, dtype=flat.dtype, device=dev)
        dist.all_gather_into_tensor(out, mine, group=group)
    else:
        parts = [torch.empty(size, dtype=flat.dtype) for _ in range(world)]
        dist.all_gather(parts, mine.cpu(), group=group)
        out = torch.cat(parts).to(dev)
    out = out.view(world, size)
    pos = 0
    for p, (off, w, n) in zip(pers, tables):
        t = flat[off:off + n * w].view(n, w)
        for o in range(world):
            k = len(range(o, n, world))
            if k:
                t[o::world] = out[o, pos:pos + k * w].view(k, w)
        pos += p * w
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
