"""Data-parallel engine on the GPU: two ranks (gloo, both on cuda:0, spawned
processes) run TrainEngine with world_size=2 -- row shards inside
ncf_train_step, the gradient exchange between the compute and optimizer graphs
(zero1: reduce-scatter, Adam on the rank's shard, in-place all-gather of the
parameters; allreduce: all-reduce, replicated Adam; touched: the rows the global
batch touches packed, all-reduced, replicated deferred Adam) -- and must (a) stay
bitwise identical to each other
and (b) match a single-rank run over the same global batches (per-step loss
rtol 1e-5; parameters rtol 1e-4 / atol 1e-6: the summed shard gradients differ
from the full-batch gradient only in fp32 summation order).

RCCL needs one GPU per rank, which the single-GPU test box does not have; gloo
moves the same device buffers through the host (reduce-scatter / all-gather in
their exact all-reduce forms, ncf_amd.distributed), so everything but the
transport is the bench's N>1 path."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

T, B = 12, 1000
U, I = 300, 400


def _batches():
    rng = np.random.default_rng(5)
    users = rng.integers(0, U, T * B)
    items = rng.integers(0, I, T * B)
    labels = (rng.random(T * B) < 0.2).astype(np.float32)
    return users, items, labels


def _run(world, rank, group, mt, f, nl, use_graph, dp_mode=None):
    from ncf_amd import ops
    from ncf_amd.engine import TrainEngine
    from ncf_amd.models import NCF
    torch.manual_seed(3)
    m = NCF(U, I, f, nl, 0.0, mt).to("cuda:0")
    want = None
    split = dp_mode == "zero1-split"
    if dp_mode == "auto-zero1":  # "auto" whose packed test fails on a model above the all-reduce size
        TrainEngine.ALLREDUCE_MAX_FLOATS = 1
        dp_mode, want = "auto", "zero1"
    if split:
        dp_mode = "zero1"
    eng = TrainEngine(m, lr=1e-3, world_size=world, rank=rank, process_group=group, dp_mode=dp_mode)
    if split:
        # every shard range cut in two (the same elements): a table window no longer
        # sits inside one range, so ncf_adam_step_fact takes its two-launch form
        import ctypes
        rng = [(eng._sranges[2 * k], eng._sranges[2 * k + 1]) for k in range(eng._nsranges)]
        cut = []
        for b, e in rng:
            mid = b + ((e - b) // 2 // 64) * 64
            cut += [(b, mid), (mid, e)] if b < mid < e else [(b, e)]
        assert len(cut) > len(rng)
        eng._sranges = (ctypes.c_int64 * (2 * len(cut)))(*[x for q in cut for x in q])
        eng._nsranges = len(cut)
    u, i, y = _batches()
    rows = torch.as_tensor(ops.pack_rows_host(u, i, y), device="cuda:0")
    eng.set_epoch_stream(rows, B)
    if split:
        assert eng._fact_shard  # the factored shard expansion is what the split ranges exercise
    eng.run(T, use_graph=use_graph)
    torch.cuda.synchronize()
    if want is not None:
        assert eng.dp_mode == want, eng.dp_mode
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
    return flat, eng.epoch_losses()[:T].copy()


def _worker(rank, world, port, mt, f, nl, use_graph, dp_mode, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        flat, losses = _run(world, rank, dist.group.WORLD, mt, f, nl, use_graph, dp_mode)
    except Exception:  # report instead of leaving the other rank waiting in a collective
        import traceback
        q.put((rank, None, traceback.format_exc()))
        os._exit(1)
    q.put((rank, flat, losses))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("mt,f,nl,use_graph,dp_mode", [("NeuMF-end", 16, 3, True, "zero1"),
                                                       ("NeuMF-end", 16, 3, False, "zero1"),
                                                       ("NeuMF-end", 16, 3, True, "allreduce"),
                                                       ("NeuMF-end", 16, 3, True, None),  # default: auto
                                                       ("NeuMF-end", 16, 3, True, "touched"),
                                                       ("NeuMF-end", 16, 3, False, "touched"),
                                                       ("GMF", 16, 3, True, "touched"),
                                                       ("MLP", 8, 2, True, "touched"),
                                                       ("NeuMF-end", 32, 3, True, "touched"),
                                                       ("NeuMF-end", 16, 3, True, "auto"),
                                                       ("NeuMF-end", 16, 3, False, "allreduce"),
                                                       ("NeuMF-end", 32, 3, True, "zero1"),
                                                       ("GMF", 16, 3, True, "zero1"),
                                                       ("NeuMF-end", 16, 3, True, "auto-zero1"),
                                                       ("NeuMF-end", 16, 3, True, "zero1-split"),
                                                       ("NeuMF-end", 16, 3, True, "owner"),
                                                       ("NeuMF-end", 16, 3, False, "owner"),
                                                       ("GMF", 16, 3, True, "owner"),
                                                       ("MLP", 8, 2, True, "owner"),
                                                       ("NeuMF-end", 32, 3, True, "owner")])
def test_two_ranks_match_single_rank(mt, f, nl, use_graph, dp_mode):
    _ranks_match_single_rank(2, mt, f, nl, use_graph, dp_mode)


@pytest.mark.parametrize("dp_mode", ["touched", "owner"])
def test_three_ranks_match_single_rank(dp_mode):
    """World 3 (B = 1000: shards of 334 / 334 / 332 rows; owner: ids % 3)."""
    _ranks_match_single_rank(3, "NeuMF-end", 16, 3, True, dp_mode)


def _ranks_match_single_rank(world, mt, f, nl, use_graph, dp_mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mt, f, nl, use_graph, dp_mode, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, flat, losses = q.get(timeout=300)
        if flat is None:
            for p in procs:
                p.kill()
            raise AssertionError(f"rank {r} failed:\n{losses}")
        res[r] = (flat, losses)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(1, world):
        assert np.array_equal(res[0][0], res[r][0]), "ranks diverged"
    flat1, losses1 = _run(1, 0, None, mt, f, nl, use_graph)
    np.testing.assert_allclose(res[0][1], losses1, rtol=1e-5)
    np.testing.assert_allclose(res[0][0], flat1, rtol=1e-4, atol=1e-6)


def _rccl_worker(port, dp_mode, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["NCF_CAPTURE_ALLREDUCE"] = "1"
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    if dp_mode == "owner-fallback":  # the first capture (the one with the all-to-alls) raises
        from ncf_amd.engine import TrainEngine
        orig, calls = TrainEngine._graph_of, []

        def failing(self, fn):
            calls.append(1)
            if len(calls) == 1:
                raise RuntimeError("simulated capture failure")
            return orig(self, fn)
        TrainEngine._graph_of = failing
        dp_mode = "owner"
    try:
        flat, losses = _run(1, 0, dist.group.WORLD, "NeuMF-end", 16, 3, True, dp_mode)
        q.put((flat, losses))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dp_mode", ["zero1", "allreduce", "touched", "owner", "owner-fallback"])
def test_rccl_collective_captured_in_step_graph(dp_mode):
    """NCF_CAPTURE_ALLREDUCE=1 on backend nccl (RCCL): the gradient exchange is
    captured inside the step graphs.  One GPU holds one RCCL rank, so a one-rank
    group with an explicit dp_mode runs the real RCCL reduce-scatter / all-gather /
    all-reduce kernels through the captured graph; the result must equal the
    single-process engine (no collective) to fp32 summation order.  owner-fallback: the
    capture with the all-to-alls raises; the engine continues with eager collectives."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), dp_mode, q))
    p.start()
    flat, losses = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    flat1, losses1 = _run(1, 0, None, "NeuMF-end", 16, 3, True)
    np.testing.assert_allclose(losses, losses1, rtol=1e-5)
    np.testing.assert_allclose(flat, flat1, rtol=1e-4, atol=1e-6)


def _mismatch_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from ncf_amd import ops
    from ncf_amd.engine import TrainEngine
    from ncf_amd.models import NCF
    torch.manual_seed(3)
    m = NCF(U, I, 16, 3, 0.0, "NeuMF-end").to("cuda:0")
    eng = TrainEngine(m, lr=1e-3, world_size=world, rank=rank, process_group=dist.group.WORLD, dp_mode="allreduce")
    u, i, y = _batches()
    if rank == 1:  # the same rows in another order: a non-canonical grouping would do this
        u, i, y = u[::-1].copy(), i[::-1].copy(), y[::-1].copy()
    rows = torch.as_tensor(ops.pack_rows_host(u, i, y), device="cuda:0")
    try:
        eng.set_epoch_stream(rows, B)
        q.put((rank, "accepted"))
    except RuntimeError as e:
        q.put((rank, str(e)))
    dist.destroy_process_group()


def test_ranks_with_different_streams_are_refused():
    """TrainEngine.set_epoch_stream at world > 1 checks that every rank holds the same
    epoch stream (a device checksum, max / -min over the ranks): a rank with its rows
    in another order makes every rank raise instead of training on shards that give
    some rows to two ranks and others to none."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mismatch_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=120)
    for r in range(2):
        assert "different epoch streams" in res[r], res
