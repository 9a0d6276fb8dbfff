"""Deferred ("catch-up") Adam (ncf_lazy_adam_step / ncf_lazy_adam_flush, ABI 14) vs
the dense optimizer launch (ncf_reduce_adam_step: torch.optim.Adam of
train_neumf.py:90,115 over every row every step) -- bitwise, on deterministic
gradients at the C4 id space (138,494 users x 26,745 items), over two epochs of
batches; plus the per-batch A / B / C lists (ncf_batch_touched) vs numpy."""
import os
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

U, I, F, NL = 138_494, 26_745, 16, 3


def _stream(nb, B, seed):
    """An epoch stream of nb batches of B packed rows (Zipf-ish users, uniform
    items), the last batch partial, with a few padding rows."""
    rng = np.random.default_rng(seed)
    n = nb * B - B // 3
    u = (rng.zipf(1.3, n) % (U - 1) + 1).astype(np.int64)
    it = rng.integers(1, I, n).astype(np.int64)
    y = (rng.random(n) < 0.2).astype(np.int64)
    rows = u | (it << 32) | (y << 63)
    pad = rng.choice(n, 7, replace=False)
    rows[pad] = np.int64(-1) ^ (np.int64(1) << 63)  # user ~0, item 0x7FFFFFFF
    return rows, n


SPAN = int(os.environ.get("NCF_LAZY_SPAN", "32"))


def _batch_ids(rows, b, B):
    seg = rows[b * B:(b + 1) * B]
    seg = seg[(seg & 0xFFFFFFFF) != 0xFFFFFFFF]
    return np.unique(seg & 0xFFFFFFFF), np.unique((seg >> 32) & 0x7FFFFFFF)


def _expected_lists(rows, n, B):
    """[b][k] (k = 2 * list + side) per include/ncf_hip.h ncf_batch_touched."""
    nb = -(-n // B)
    R = [_batch_ids(rows, b, B) for b in range(nb)]
    out = []
    for b in range(nb):
        lists = [None] * 6
        for side, N in ((0, U), (1, I)):
            a = R[b][side]
            if b + 1 < nb:
                nx = np.setdiff1d(R[b + 1][side], a)
                sl = b % SPAN
                c = np.arange(sl * N // SPAN, (sl + 1) * N // SPAN)
                c = np.setdiff1d(c, np.union1d(a, R[b + 1][side]))
            else:
                nx = np.setdiff1d(np.arange(N), a)
                c = np.zeros(0, np.int64)
            lists[side], lists[2 + side], lists[4 + side] = a, nx, c
        out.append(lists)
    return out


def test_batch_touched_lists_match_numpy():
    import ncf_amd._lib as L
    from ncf_amd.engine import touched_segments
    lib = L.hip()
    dev = torch.device("cuda", 0)
    for B, nb, seed in ((4096, 9, 0), (65536, 3, 1), (1000, 40, 2)):
        rows, n = _stream(nb, B, seed)
        rd = torch.from_numpy(rows).to(dev)
        nbytes = lib.ncf_touched_bytes(n, B, U, I)
        buf = torch.full(((nbytes + 3) // 4,), -7, dtype=torch.int32, device=dev)
        L.check(lib.ncf_batch_touched(rd.data_ptr(), n, B, U, I, buf.data_ptr(), L.stream_ptr(dev)), "touched")
        got = touched_segments(buf.cpu().numpy(), nb)
        want = _expected_lists(rows, n, B)
        for b in range(nb):
            for k in range(6):
                assert np.array_equal(got[b][k], want[b][k]), f"B={B} batch {b} list {k}"


def _ranges(lay):
    from ncf_amd.engine import _active_ranges
    from ncf_amd.models import NCF
    m = NCF(U, I, F, NL, 0.0, "NeuMF-end")
    rng = _active_ranges(m, lay)
    return (ctypes.c_int64 * (2 * len(rng)))(*[x for r in rng for x in r]), len(rng)


def test_lazy_adam_bitwise_equals_dense_over_two_epochs():
    """60 optimizer steps (two epochs of 30 batches, the epoch's last batch included):
    after every step the rows the next batch reads are bitwise the dense optimizer's;
    after ncf_lazy_adam_flush (mid-run and at the end) every parameter and moment
    is; gradients are cleared in both."""
    import ncf_amd._lib as L
    lib = L.hip()
    dev = torch.device("cuda", 0)
    st = L.stream_ptr(dev)
    B, nb = 4096, 30
    lay = L.layout(U, I, F, NL, "NeuMF-end")
    L.check(lib.ncf_layout_tune(ctypes.byref(lay), B), "tune")
    assert lib.ncf_fact_mode(ctypes.byref(lay)) == 0  # C4: U + I beyond the factored path
    ranges, nr = _ranges(lay)
    rows, n = _stream(nb, B, 3)
    rd = torch.from_numpy(rows).to(dev)
    touched = torch.empty((lib.ncf_touched_bytes(n, B, U, I) + 3) // 4, dtype=torch.int32, device=dev)
    L.check(lib.ncf_batch_touched(rd.data_ptr(), n, B, U, I, touched.data_ptr(), st), "touched")
    from ncf_amd.engine import touched_segments
    lists = touched_segments(touched.cpu().numpy(), nb)
    users_of = [lists[b][0] for b in range(nb)]
    items_of = [lists[b][1] for b in range(nb)]

    total = int(lay.total)
    g = torch.Generator(device="cpu").manual_seed(0)
    p0 = (torch.randn(total, generator=g) * 0.05).to(dev)
    bufs = {}
    for k in ("A", "B"):
        bufs[k] = {"p": p0.clone(), "g": torch.zeros(total, device=dev), "m": torch.zeros(total, device=dev),
                   "v": torch.zeros(total, device=dev), "ctl": torch.zeros(6, dtype=torch.int64, device=dev),
                   "hist": torch.zeros(nb, device=dev)}
    last = torch.zeros(U + I, dtype=torch.int32, device=dev)
    RING = 1 << 10
    ring = torch.zeros(2 * RING, device=dev)
    ws_bytes = lib.ncf_workspace_bytes(ctypes.byref(lay), B)
    ws = torch.zeros((ws_bytes + 3) // 4, device=dev)
    rows_slab = lib.ncf_reduce_rows(ctypes.byref(lay))
    stride = lib.ncf_slab_stride(ctypes.byref(lay))
    f, dm = F, F << (NL - 1)

    def rows_idx(ids, off, w):
        ids = torch.as_tensor(ids.astype(np.int64), device=dev)
        return (off + ids[:, None] * w + torch.arange(w, device=dev)[None, :]).reshape(-1)

    def flush_and_compare(tag):
        L.check(lib.ncf_lazy_adam_flush(ctypes.byref(lay), bufs["B"]["p"].data_ptr(), bufs["B"]["g"].data_ptr(),
                                        bufs["B"]["m"].data_ptr(), bufs["B"]["v"].data_ptr(), ranges, nr,
                                        bufs["B"]["ctl"].data_ptr(), 0.9, 0.999, 1e-8, last.data_ptr(),
                                        ring.data_ptr(), RING, st), "flush")
        for k in ("p", "m", "v", "g"):
            a, b = bufs["A"][k], bufs["B"][k]
            assert torch.equal(a, b), f"{tag}: {k} differs at {int((a != b).sum())} elements"

    for t in range(1, 2 * nb + 1):
        b = (t - 1) % nb
        gs = torch.Generator(device="cpu").manual_seed(1000 + t)
        grad = torch.zeros(total, device=dev)
        for ids, (o1, w1), (o2, w2) in ((users_of[b], (lay.ug, f), (lay.um, dm)),
                                         (items_of[b], (lay.ig, f), (lay.im, dm))):
            keep = ids[np.arange(len(ids)) % 17 != 3]  # some touched rows get an exactly-zero gradient
            for o, w in ((o1, w1), (o2, w2)):
                idx = rows_idx(keep, int(o), w)
                grad[idx] = (torch.randn(idx.numel(), generator=gs) * 0.01).to(dev)
        slab = (torch.randn(rows_slab * stride, generator=gs) * 0.001).to(dev)
        ws[: rows_slab * stride].copy_(slab)
        for k in ("A", "B"):
            bufs[k]["g"].copy_(grad)
            bufs[k]["ctl"][4] = b
            bufs[k]["ctl"][5] = t
        A, Bb = bufs["A"], bufs["B"]
        L.check(lib.ncf_reduce_adam_step(ctypes.byref(lay), ws.data_ptr(), A["p"].data_ptr(), A["g"].data_ptr(),
                                         A["m"].data_ptr(), A["v"].data_ptr(), ranges, nr, A["ctl"].data_ptr(),
                                         1e-3, 0.9, 0.999, 1e-8, A["hist"].data_ptr(), nb, st), "dense")
        L.check(lib.ncf_lazy_adam_step(ctypes.byref(lay), ws.data_ptr(), Bb["p"].data_ptr(), Bb["g"].data_ptr(),
                                       Bb["m"].data_ptr(), Bb["v"].data_ptr(), ranges, nr, Bb["ctl"].data_ptr(),
                                       1e-3, 0.9, 0.999, 1e-8, Bb["hist"].data_ptr(), nb, touched.data_ptr(), n, B,
                                       last.data_ptr(), ring.data_ptr(), RING, st), "lazy")
        torch.cuda.synchronize()
        assert torch.equal(A["ctl"][:2], Bb["ctl"][:2]) and torch.equal(A["hist"], Bb["hist"])
        # the tower (dense in both) and the rows the next batch reads: bitwise now
        tb, te = int(lay.tower_begin), int(lay.tower_begin + lay.tower_len)
        for k in ("p", "m", "v"):
            assert torch.equal(A[k][tb:te], Bb[k][tb:te]), f"tower {k} step {t}"
        nxt = (b + 1) % nb
        if b + 1 < nb:
            for ids, (o1, w1), (o2, w2) in ((users_of[nxt], (lay.ug, f), (lay.um, dm)),
                                             (items_of[nxt], (lay.ig, f), (lay.im, dm))):
                idx = torch.cat([rows_idx(ids, int(o1), w1), rows_idx(ids, int(o2), w2)])
                for k in ("p", "m", "v"):
                    assert torch.equal(A[k][idx], Bb[k][idx]), f"next batch's rows, {k}, step {t}"
        else:  # the epoch's last batch brought every row up
            for k in ("p", "m", "v"):
                assert torch.equal(A[k], Bb[k]), f"epoch end {k} step {t}"
        # rolling catch-up: no row more than SPAN steps behind
        assert int(last.min()) >= t - SPAN, f"step {t}: a row sat out {t - int(last.min())} steps"
        if t in (7, 41):
            flush_and_compare(f"step {t}")
    flush_and_compare("end")
    assert int(last.min()) == int(last.max()) == 2 * nb


def test_step_scalar_cache_follows_its_inputs():
    """The optimizer launches take step t's (-lr/bc1, sqrt(bc2)) from a per-control-
    block cache that step t - 1's launch filled (ncf_ops.hip ScCache).  Steps out of
    order, repeated, and with lr / beta changes between them must give bitwise what a
    fresh control block (no usable entry: the double pows) gives."""
    import ncf_amd._lib as L
    lib = L.hip()
    dev = torch.device("cuda", 0)
    st = L.stream_ptr(dev)
    n = 4096
    g = torch.Generator(device="cpu").manual_seed(5)
    p0 = torch.randn(n, generator=g).to(dev)
    grads = [(torch.randn(n, generator=g) * 0.01).to(dev) for _ in range(12)]
    ranges = (ctypes.c_int64 * 2)(0, n)
    seq = [(1, 1e-3, 0.999), (2, 1e-3, 0.999), (3, 1e-3, 0.999), (4, 2e-3, 0.999), (5, 2e-3, 0.99),
           (6, 2e-3, 0.99), (6, 2e-3, 0.99), (3, 2e-3, 0.99), (4, 2e-3, 0.99), (7, 1e-3, 0.999),
           (8, 1e-3, 0.999), (9, 1e-3, 0.999)]
    bufs = {k: [p0.clone(), torch.zeros(n, device=dev), torch.zeros(n, device=dev)] for k in ("cached", "fresh")}
    ctl = torch.zeros(6, dtype=torch.int64, device=dev)
    fresh = []  # kept alive: every fresh control block a new pointer, so a new cache slot
    for i, (t, lr, b2) in enumerate(seq):
        for k in ("cached", "fresh"):
            if k == "fresh":
                fresh.append(torch.zeros(6, dtype=torch.int64, device=dev))
            c = ctl if k == "cached" else fresh[-1]
            c[1] = t
            gr = grads[i].clone()
            p, m, v = bufs[k]
            L.check(lib.ncf_adam_step(p.data_ptr(), gr.data_ptr(), m.data_ptr(), v.data_ptr(), ranges, 1,
                                      c.data_ptr(), lr, 0.9, b2, 1e-8, -1, None, 0, st), "adam")
            torch.cuda.synchronize()
        for a, b in zip(bufs["cached"], bufs["fresh"]):
            assert torch.equal(a, b), f"step {i} (t={t}, lr={lr}, beta2={b2})"
