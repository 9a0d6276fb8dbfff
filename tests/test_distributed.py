"""Data-parallel decomposition on CPU with torch.distributed (gloo, world_size 2).

The device engine shards every global batch into contiguous per-rank slices
(rows [r*ceil(gb/W), ...), exactly what ncf_train_step does with world/rank),
scales dlogit by 1/global_batch, and all-reduces the flat gradient bucket.  This
test runs that protocol with the CPU oracle's gradient math on two gloo ranks
and checks the all-reduced gradient equals the single-process mean gradient
(BCEWithLogitsLoss mean, train_neumf.py:86), and that both ranks derive the
same epoch stream from the same seeds."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ncf_amd.distributed import shard_range


def test_shard_ranges_partition_every_batch():
    for gb in (1, 2, 3, 1000, 65536, 55645):
        for W in (1, 2, 3, 4, 8):
            parts = [shard_range(gb, W, r) for r in range(W)]
            assert parts[0][0] == 0 and parts[-1][1] == gb
            for (a0, a1), (b0, b1) in zip(parts, parts[1:]):
                assert a1 == b0 and a0 <= a1


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import ncf_oracle as O
    from ncf_amd.data import NCFData, epoch_permutation
    from ncf_amd.distributed import allreduce_flat_grads, shard_range
    torch.manual_seed(0)
    np.random.seed(0)
    # identical host stream on every rank
    pos = np.stack([np.repeat(np.arange(40), 6), np.random.default_rng(1).integers(0, 60, 240)], 1)
    pos = np.unique(pos, axis=0)
    ds = NCFData(pos, 60, None, 4, True)
    ds.ng_sample()
    u, i, y = ds.arrays()
    perm = epoch_permutation(len(u)).numpy()
    B = 300
    bu, bi, by = u[perm[:B]], i[perm[:B]], y[perm[:B]]
    lo, hi = shard_range(B, world, rank)
    torch.manual_seed(5)
    m = O.OracleNCF(40, 60, 8, 3, 0.0, "NeuMF-end")
    # local shard, loss scaled to the global mean: sum_i bce_i / B
    uu = torch.as_tensor(bu[lo:hi], dtype=torch.int64)
    ii = torch.as_tensor(bi[lo:hi], dtype=torch.int64)
    yy = torch.as_tensor(by[lo:hi], dtype=torch.float32)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(m(uu, ii), yy, reduction="sum") / B
    loss.backward()
    flat = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
    allreduce_flat_grads(flat)
    q.put((rank, flat.numpy(), perm[:20].copy(), bu[:20].copy()))
    dist.destroy_process_group()


def test_gloo_two_ranks_equal_single_process_gradient():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, g0, perm0, bu0), (_, g1, perm1, bu1) = res
    assert np.array_equal(perm0, perm1) and np.array_equal(bu0, bu1)
    np.testing.assert_allclose(g0, g1, rtol=0, atol=0)
    # single-process reference
    from oracle import ncf_oracle as O
    from ncf_amd.data import NCFData, epoch_permutation
    torch.manual_seed(0)
    np.random.seed(0)
    pos = np.stack([np.repeat(np.arange(40), 6), np.random.default_rng(1).integers(0, 60, 240)], 1)
    pos = np.unique(pos, axis=0)
    ds = NCFData(pos, 60, None, 4, True)
    ds.ng_sample()
    u, i, y = ds.arrays()
    perm = epoch_permutation(len(u)).numpy()
    B = 300
    torch.manual_seed(5)
    m = O.OracleNCF(40, 60, 8, 3, 0.0, "NeuMF-end")
    _, _, grads = O.forward_backward(m, u[perm[:B]], i[perm[:B]], y[perm[:B]].astype(np.int64))
    ref = torch.cat([grads[k].reshape(-1) for k, _ in m.named_parameters()]).numpy()
    np.testing.assert_allclose(g0, ref, rtol=1e-5, atol=1e-9)
