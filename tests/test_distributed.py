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


# ---------------------------------------------------------------------------
# zero1: reduce-scatter -> Adam on the own shard -> in-place all-gather
# (ncf_amd.engine.TrainEngine(dp_mode="zero1"), the default for world > 1 above
# TrainEngine.ALLREDUCE_MAX_FLOATS)

def test_shard_floats_and_ranges_cover_active_params():
    from ncf_amd.distributed import shard_floats, shard_ranges
    active = [[0, 640], [1024, 1088], [4096, 9000]]
    for total in (64, 1000, 9001, 790_737):
        for W in (1, 2, 3, 4, 8):
            S = shard_floats(total, W)
            assert S % 64 == 0 and S * W >= total and (S - 64) * W < total
            got = []
            for r in range(W):
                for b, e in shard_ranges(active, W, r, S):
                    assert 0 <= b < e <= S and b % 4 == 0 and e % 4 == 0
                    got.append([b + r * S, e + r * S])
            covered = sorted(x for b, e in got for x in range(b, e))
            want = sorted(x for b, e in active for x in range(b, min(e, S * W)))
            assert covered == want


def _zero1_worker(rank, world, port, emulate, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["NCF_DP_EMULATE"] = "1" if emulate else "0"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import ncf_oracle as O
    from ncf_amd.distributed import all_gather_flat, reduce_scatter_flat, shard_floats, shard_range
    torch.manual_seed(5)
    m = O.OracleNCF(40, 60, 8, 3, 0.0, "NeuMF-end")
    params = list(m.parameters())
    n = sum(p.numel() for p in params)
    S = shard_floats(n, world)
    flat = torch.zeros(S * world)
    flat[:n] = torch.cat([p.detach().reshape(-1) for p in params])
    shard = torch.nn.Parameter(flat[rank * S:(rank + 1) * S].clone())
    opt = torch.optim.Adam([shard], lr=1e-2)
    rng = np.random.default_rng(2)
    B = 257
    for _ in range(3):
        u, i = rng.integers(0, 40, B), rng.integers(0, 60, B)
        y = (rng.random(B) < 0.3).astype(np.float32)
        off = 0  # the gathered flat parameters back into the model
        with torch.no_grad():
            for p in params:
                p.copy_(flat[off:off + p.numel()].view_as(p))
                off += p.numel()
        m.zero_grad()
        lo, hi = shard_range(B, world, rank)
        logit = m(torch.as_tensor(u[lo:hi]), torch.as_tensor(i[lo:hi]))
        loss = torch.nn.functional.binary_cross_entropy_with_logits(logit, torch.as_tensor(y[lo:hi]),
                                                                    reduction="sum") / B
        loss.backward()
        g = torch.zeros(S * world)
        g[:n] = torch.cat([p.grad.reshape(-1) for p in params])
        gs = torch.zeros(S)
        reduce_scatter_flat(gs, g, rank)
        shard.grad = gs
        opt.step()
        with torch.no_grad():
            flat[rank * S:(rank + 1) * S].copy_(shard)
        all_gather_flat(flat, rank, S)
    q.put((rank, flat[:n].numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,emulate", [(2, False), (3, False), (2, True)])
def test_gloo_zero1_matches_single_process_adam(world, emulate):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + (os.getpid() % 1000) + 10 * world + int(emulate)
    procs = [ctx.Process(target=_zero1_worker, args=(r, world, port, emulate, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, f in res[1:]:
        assert np.array_equal(f, res[0][1]), "ranks hold different parameters after the all-gather"
    # single process, full-batch mean gradient, dense Adam over every parameter
    from oracle import ncf_oracle as O
    torch.manual_seed(5)
    m = O.OracleNCF(40, 60, 8, 3, 0.0, "NeuMF-end")
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    rng = np.random.default_rng(2)
    B = 257
    for _ in range(3):
        u, i = rng.integers(0, 40, B), rng.integers(0, 60, B)
        y = (rng.random(B) < 0.3).astype(np.float32)
        opt.zero_grad()
        loss = torch.nn.functional.binary_cross_entropy_with_logits(m(torch.as_tensor(u), torch.as_tensor(i)),
                                                                    torch.as_tensor(y))
        loss.backward()
        opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy()
    np.testing.assert_allclose(res[0][1], ref, rtol=1e-4, atol=1e-6)


# ---------------------------------------------------------------------------
# owner: row id owned by rank id % W; gradient rows to their owners, the next batch's
# rows back to their readers (TrainEngine(dp_mode="owner"), include/ncf_hip.h
# ncf_owner_*).  The protocol on CPU tensors, with the lists of tests/owner_model.py.

def test_owner_lists_partition_each_slice():
    """Model lists: per (batch, slice) the S lists of a rank partition its slice's
    unique ids by owner; R(r) of owner o is S(o) of rank r; chunk starts bracket the
    owned rows."""
    from owner_model import chunk_starts, owner_lists, slice_ids, slices
    rng = np.random.default_rng(0)
    n, B, U, I = 2000, 300, 97, 61
    rows = (rng.integers(0, U, n).astype(np.uint64) | (rng.integers(0, I, n).astype(np.uint64) << np.uint64(32)))
    rows[5] = np.uint64(0xFFFFFFFF) | (np.uint64(0x7FFFFFFF) << np.uint64(32))  # padding row
    for W in (1, 2, 3, 8):
        per_rank = [owner_lists(rows, n, B, W, me)[0] for me in range(W)]
        for b, r, lo, hi in slices(n, B, W):
            uu, ii = slice_ids(rows, lo, hi)
            for o in range(W):
                for s, ids in enumerate((uu, ii)):
                    want = ids[ids % W == o]
                    assert np.array_equal(per_rank[r][b]["S"][o][s], want)
                    assert np.array_equal(per_rank[o][b]["R"][r][s], want)
                    ch = 4
                    st = chunk_starts(want, o, W, ch, (max(U, I) + ch - 1) // ch)
                    local = (want - o) // W
                    for c in range(len(st) - 1):
                        seg = local[st[c]:st[c + 1]]
                        assert ((seg >= c * ch) & (seg < (c + 1) * ch)).all()


def _owner_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle import ncf_oracle as O
    from ncf_amd.distributed import all_to_all_equal, owner_gather_rows
    from owner_model import owner_lists, slices
    U, I, f, dm, B, T = 40, 60, 8, 32, 257, 3
    torch.manual_seed(5)
    m = O.OracleNCF(U, I, f, 3, 0.0, "NeuMF-end")
    params = list(m.parameters())
    n = sum(p.numel() for p in params)
    offs = np.cumsum([0] + [p.numel() for p in params])
    flat = torch.nn.Parameter(torch.cat([p.detach().reshape(-1) for p in params]))
    opt = torch.optim.Adam([flat], lr=1e-2)
    rng = np.random.default_rng(2)
    u = rng.integers(0, U, B * T)
    i = rng.integers(0, I, B * T)
    y = (rng.random(B * T) < 0.3).astype(np.float32)
    rows = u.astype(np.uint64) | (i.astype(np.uint64) << np.uint64(32))
    lists, mx = owner_lists(rows, B * T, B, world, rank)
    Mu, Mi = mx
    tables = [(int(offs[k]), w, nr) for k, (w, nr) in enumerate(((f, U), (f, I), (dm, U), (dm, I)))]
    tail0 = int(offs[4])
    wrow = f + dm

    def rows_of(vec, s, ids):  # [len(ids), f + dm] row records (GMF part, then MLP part)
        g = vec[tables[s][0]:tables[s][0] + tables[s][2] * f].view(-1, f)[ids]
        mm = vec[tables[s + 2][0]:tables[s + 2][0] + tables[s + 2][2] * dm].view(-1, dm)[ids]
        return torch.cat([g, mm], 1)

    def set_rows(vec, s, ids, val):
        vec[tables[s][0]:tables[s][0] + tables[s][2] * f].view(-1, f)[ids] = val[:, :f]
        vec[tables[s + 2][0]:tables[s + 2][0] + tables[s + 2][2] * dm].view(-1, dm)[ids] = val[:, f:]

    M = (Mu, Mi)
    D = (Mu + Mi) * wrow + (n - tail0)
    D2 = (Mu + Mi) * wrow
    sl = {(b, r): (lo, hi) for b, r, lo, hi in slices(B * T, B, world)}
    for b in range(T):
        with torch.no_grad():  # the replica into the model (rows this rank does not read may be stale)
            for p, o0 in zip(params, offs[:-1]):
                p.copy_(flat[o0:o0 + p.numel()].view_as(p))
        m.zero_grad()
        lo, hi = sl[(b, rank)]
        logit = m(torch.as_tensor(u[lo:hi]), torch.as_tensor(i[lo:hi]))
        loss = torch.nn.functional.binary_cross_entropy_with_logits(logit, torch.as_tensor(y[lo:hi]),
                                                                    reduction="sum") / B
        loss.backward()
        g = torch.cat([p.grad.reshape(-1) for p in params])
        send = torch.zeros(world, D)
        for o in range(world):
            for s in range(2):
                ids = torch.as_tensor(lists[b]["S"][o][s])
                base = 0 if s == 0 else Mu * wrow
                send[o, base:base + len(ids) * wrow] = rows_of(g, s, ids).reshape(-1)
            send[o, D2:] = g[tail0:]
        recv = torch.zeros(world, D)
        all_to_all_equal(recv.view(-1), send.view(-1))
        gsum = torch.zeros(n)  # owned rows and the tail, summed in rank order
        for r in range(world):
            gsum[tail0:] += recv[r, D2:]
            for s in range(2):
                ids = torch.as_tensor(lists[b]["R"][r][s])
                base = 0 if s == 0 else Mu * wrow
                got = recv[r, base:base + len(ids) * wrow].view(-1, wrow)
                set_rows(gsum, s, ids, rows_of(gsum, s, ids) + got)
        flat.grad = gsum
        opt.step()
        b1 = (b + 1) % T
        send2 = torch.zeros(world, D2)
        with torch.no_grad():
            for qr in range(world):
                for s in range(2):
                    ids = torch.as_tensor(lists[b1]["R"][qr][s])
                    base = 0 if s == 0 else Mu * wrow
                    send2[qr, base:base + len(ids) * wrow] = rows_of(flat.detach(), s, ids).reshape(-1)
            recv2 = torch.zeros(world, D2)
            all_to_all_equal(recv2.view(-1), send2.view(-1))
            for o in range(world):
                if o == rank:
                    continue
                for s in range(2):
                    ids = torch.as_tensor(lists[b1]["S"][o][s])
                    base = 0 if s == 0 else Mu * wrow
                    set_rows(flat.data, s, ids, recv2[o, base:base + len(ids) * wrow].view(-1, wrow))
    with torch.no_grad():
        owner_gather_rows(flat.data, tables, world, rank)
    q.put((rank, flat.detach().numpy().copy(), M))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_owner_protocol_matches_single_process_adam(world):
    """Three steps of the owner exchange (gradient rows to owners, dense Adam on every
    owned row, the next batch's rows fetched, replicas stale elsewhere) then the
    end-of-run gather: ranks bitwise equal, equal to single-process dense Adam."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33500 + (os.getpid() % 1000) + 10 * world
    procs = [ctx.Process(target=_owner_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, f, M in res[1:]:
        assert M == res[0][2]
        assert np.array_equal(f, res[0][1]), "ranks hold different parameters after the gather"
    from oracle import ncf_oracle as O
    torch.manual_seed(5)
    m = O.OracleNCF(40, 60, 8, 3, 0.0, "NeuMF-end")
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    rng = np.random.default_rng(2)
    B, T = 257, 3
    u = rng.integers(0, 40, B * T)
    i = rng.integers(0, 60, B * T)
    y = (rng.random(B * T) < 0.3).astype(np.float32)
    for b in range(T):
        s = slice(b * B, (b + 1) * B)
        opt.zero_grad()
        loss = torch.nn.functional.binary_cross_entropy_with_logits(m(torch.as_tensor(u[s]), torch.as_tensor(i[s])),
                                                                    torch.as_tensor(y[s]))
        loss.backward()
        opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy()
    np.testing.assert_allclose(res[0][1], ref, rtol=1e-4, atol=1e-6)
