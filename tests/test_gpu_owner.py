"""dp_mode "owner" on the GPU: the bucket lists of ncf_owner_lists against the host
model (tests/owner_model.py) and the exchange kernels in a one-rank engine.

The lists are index work: exact equality, on random streams with padding rows and
on the first batches of a C4 (ml-20m-shaped) epoch stream, at world 1, 2, 3 and 8,
for the first and the last rank.  A one-rank owner engine (the two all-to-alls
are copies) must track the single-process engine: the owner sums one contribution per
row and runs the same dense Adam."""
import ctypes
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from owner_model import chunk_starts, decode_record, owner_lists  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _device_lists(rows, n, B, W, me, U, I, f=16, L=3, mt="NeuMF-end", slots=None):
    import ncf_amd._lib as Lb
    from ncf_amd import ops
    from ncf_amd.models import NCF
    from ncf_amd.engine import _active_ranges
    lay = Lb.layout(U, I, f, L, mt)
    torch.manual_seed(0)
    m = NCF(U, I, f, L, 0.0, mt)
    rng = _active_ranges(m, lay)
    ranges = (ctypes.c_int64 * (2 * len(rng)))(*[x for r in rng for x in r])
    _, mx = owner_lists(rows, n, B, W, me) if slots is None else (None, slots)
    P = Lb.NcfOwnerPlan()
    Lb.check(Lb.hip().ncf_owner_plan_init(ctypes.byref(lay), ranges, len(rng), n, B, W, me, int(mx[0]), int(mx[1]),
                                          ctypes.byref(P)), "plan")
    d_rows = torch.as_tensor(rows.view(np.int64), device=DEV)
    buf = torch.full(((int(P.lists_bytes) + 3) // 4,), -7, dtype=torch.int32, device=DEV)
    mxd = torch.zeros(2, dtype=torch.int32, device=DEV)
    Lb.check(Lb.hip().ncf_owner_lists(ctypes.byref(P), ctypes.byref(lay), d_rows.data_ptr(), buf.data_ptr(),
                                      mxd.data_ptr(), Lb.stream_ptr()), "lists")
    torch.cuda.synchronize()
    del ops
    return P, buf.cpu().numpy(), mxd.cpu().numpy()


def _check(rows, n, B, W, me, U, I):
    model, mx = owner_lists(rows, n, B, W, me)
    P, buf, mxd = _device_lists(rows, n, B, W, me, U, I)
    assert list(mxd) == list(mx), (mxd, mx)
    for b in range(int(P.nb)):
        got = decode_record(buf, P, b)
        for key in ("S", "R"):
            for q in range(W):
                for s in range(2):
                    assert np.array_equal(got[key][q][s], model[b][key][q][s]), (b, key, q, s)
        for r in range(W):
            for s, (ch, nch) in enumerate(((P.chunk_u, P.nchunk_u), (P.chunk_i, P.nchunk_i))):
                want = chunk_starts(model[b]["R"][r][s], me, W, ch, nch)
                assert np.array_equal(got["starts"][r][s], want), (b, r, s)


@pytest.mark.parametrize("W", [1, 2, 3, 8])
def test_owner_lists_random_stream(W):
    rng = np.random.default_rng(W)
    U, I, n, B = 5000, 3000, 40000, 4096
    rows = rng.integers(0, U, n).astype(np.uint64) | (rng.integers(0, I, n).astype(np.uint64) << np.uint64(32))
    rows[rng.integers(0, n, 50)] = np.uint64(0xFFFFFFFF) | (np.uint64(0x7FFFFFFF) << np.uint64(32))
    rows[rng.random(n) < 0.3] |= np.uint64(1) << np.uint64(63)  # labels do not matter
    for me in sorted({0, W - 1}):
        _check(rows, n, B, W, me, U, I)


_C4_HEAD = {}


def _c4_head():
    """The first 12 global batches of a C4 epoch stream (built once per session)."""
    if not _C4_HEAD:
        from ncf_amd import ops, synthetic
        from ncf_amd.data import NCFData, epoch_permutation
        ds = synthetic.make_dataset("ml-20m", seed=0)
        U, I = ds["user_num"], ds["item_num"]
        train = NCFData(np.stack([ds["train_users"], ds["train_items"]], 1), I, None, 4, True)
        np.random.seed(0)
        torch.manual_seed(0)
        train.ng_sample()
        u, i, y = train.arrays()
        B = 65536
        perm = epoch_permutation(len(u)).to(DEV)
        d = torch.from_numpy(ops.pack_rows_host(u, i, y)).to(DEV)
        stream = ops.EpochPrep(torch.device(DEV), canonical=True)(d, perm, B, int(I))
        n = 12 * B
        _C4_HEAD.update(rows=stream[:n].cpu().numpy().view(np.uint64), n=n, B=B, U=U, I=I)
    return _C4_HEAD


@pytest.mark.parametrize("W", [2, 8])
def test_owner_lists_c4_stream(W):
    """The first 12 global batches of a C4 epoch stream (ml-20m ids, grouped by item,
    canonical) -- the bench's multi-GPU stress config."""
    h = _c4_head()
    for me in (0, W - 1):
        _check(h["rows"], h["n"], h["B"], W, me, h["U"], h["I"])


def test_owner_lists_truncate_and_report():
    """Slots below the longest list: lists truncated at the slots, the true maxima
    reported (the engine regrows and rebuilds)."""
    rng = np.random.default_rng(9)
    U, I, n, B, W = 2000, 1000, 8192, 4096, 2
    rows = rng.integers(0, U, n).astype(np.uint64) | (rng.integers(0, I, n).astype(np.uint64) << np.uint64(32))
    _, mx = owner_lists(rows, n, B, W, 0)
    P, buf, mxd = _device_lists(rows, n, B, W, 0, U, I, slots=(mx[0] // 2, mx[1] // 2))
    assert list(mxd) == list(mx)
    got = decode_record(buf, P, 0)
    assert all(len(got["S"][o][0]) == mx[0] // 2 or len(got["S"][o][0]) < mx[0] // 2 for o in range(W))


@pytest.mark.parametrize("mt,f,nl,use_graph", [("NeuMF-end", 16, 3, True), ("NeuMF-end", 16, 3, False),
                                               ("GMF", 16, 3, True), ("MLP", 8, 2, True),
                                               ("NeuMF-end", 32, 3, True)])
def test_one_rank_owner_engine_equals_single(mt, f, nl, use_graph):
    from ncf_amd import ops
    from ncf_amd.engine import TrainEngine
    from ncf_amd.models import NCF
    U, I, B, T = 300, 400, 1000, 12
    rng = np.random.default_rng(5)
    u, i = rng.integers(0, U, T * B), rng.integers(0, I, T * B)
    y = (rng.random(T * B) < 0.2).astype(np.float32)
    rows = torch.as_tensor(ops.pack_rows_host(u, i, y), device=DEV)
    out = []
    for mode in (None, "owner"):
        torch.manual_seed(3)
        m = NCF(U, I, f, nl, 0.0, mt).to(DEV)
        eng = TrainEngine(m, lr=1e-3, dp_mode=mode)
        eng.set_epoch_stream(rows, B)
        eng.run(T, use_graph=use_graph)
        torch.cuda.synchronize()
        out.append((torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy(),
                    eng.epoch_losses()[:T].copy(), eng.dp_mode))
    (p1, l1, m1), (p2, l2, m2) = out
    assert m1 == "single" and m2 == "owner"
    # the same dense Adam on one contribution per row; the single-process engine's
    # factored expansion sums W0's block partials in another order and the
    # step's float atomics vary in the last bits between runs
    np.testing.assert_allclose(l2, l1, rtol=1e-6)
    np.testing.assert_allclose(p2, p1, rtol=1e-4, atol=1e-6)
