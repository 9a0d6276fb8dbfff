"""Host model of the owner-sharded exchange (dp_mode "owner", include/ncf_hip.h
ncf_owner_*), the checker of the device kernels and of the protocol.

Spec restated from the header: embedding row `id` (either side) is owned by rank
id % W; rank r takes rows [r ceil(cnt/W), ...) of each global batch (the slicing of
ncf_train_step, distributed.shard_range); padding rows (user 0xffffffff) touch nothing.
Per batch b, rank `me` keeps
  S_b(o, s)  the sorted unique ids of side s in its own slice with id % W == o
  R_b(r, s)  the sorted unique ids of side s in rank r's slice with id % W == me
and, for R, the start of every chunk of owned rows (chunk c = local rows
[c CH, (c + 1) CH), local row j = id // W).
"""
from __future__ import annotations

import numpy as np


def slices(n, B, W):
    """[(b, r, lo, hi)] absolute row ranges of every rank slice of every batch."""
    out = []
    nb = (n + B - 1) // B
    for b in range(nb):
        r0 = b * B
        cnt = min(B, n - r0)
        per = (cnt + W - 1) // W
        for r in range(W):
            lo = min(r * per, cnt)
            hi = min(lo + per, cnt)
            out.append((b, r, r0 + lo, r0 + hi))
    return out


def slice_ids(rows, lo, hi):
    seg = np.asarray(rows[lo:hi], dtype=np.uint64)
    u = (seg & np.uint64(0xFFFFFFFF)).astype(np.int64)
    keep = u != 0xFFFFFFFF
    it = ((seg >> np.uint64(32)) & np.uint64(0x7FFFFFFF)).astype(np.int64)
    return np.unique(u[keep]), np.unique(it[keep])


def owner_lists(rows, n, B, W, me):
    """{b: {"S": [[users_o, items_o] for o], "R": [[users_r, items_r] for r]}} and the
    longest list over every (b, r, o) per side."""
    out = {}
    mx = [0, 0]
    for b, r, lo, hi in slices(n, B, W):
        ids = slice_ids(rows, lo, hi)
        rec = out.setdefault(b, {"S": [None] * W, "R": [None] * W})
        for o in range(W):
            per_side = [x[x % W == o] for x in ids]
            for s in range(2):
                mx[s] = max(mx[s], len(per_side[s]))
            if r == me:
                rec["S"][o] = per_side
            if o == me:
                rec["R"][r] = per_side
    return out, mx


def chunk_starts(ids, me, W, ch, nchunk):
    """Start index in sorted `ids` (all owned by `me`) of every owned-row chunk."""
    local = (np.asarray(ids, dtype=np.int64) - me) // W
    return np.searchsorted(local, np.arange(nchunk + 1) * ch, side="left").astype(np.int64)


def decode_record(buf, plan, b):
    """One batch record of ncf_owner_lists output (int32 numpy) -> the same dict form
    as owner_lists()[0][b] plus the chunk starts of R."""
    W, mu, mi = plan.world, plan.max_u, plan.max_i
    rec = np.asarray(buf[b * plan.record_ints:(b + 1) * plan.record_ints])
    cnt = rec[:4 * W].reshape(2, W, 2)
    base = 4 * W
    out = {"S": [], "R": [], "starts": []}
    for kind, key in ((0, "S"), (1, "R")):
        k0 = base + kind * W * (mu + mi)
        for q in range(W):
            u0 = k0 + q * mu
            i0 = k0 + W * mu + q * mi
            out[key].append([rec[u0:u0 + cnt[kind, q, 0]].astype(np.int64),
                             rec[i0:i0 + cnt[kind, q, 1]].astype(np.int64)])
    s0 = base + 2 * W * (mu + mi)
    ncu, nci = plan.nchunk_u, plan.nchunk_i
    for q in range(W):
        su = rec[s0 + q * (ncu + 1): s0 + (q + 1) * (ncu + 1)].astype(np.int64)
        si0 = s0 + W * (ncu + 1) + q * (nci + 1)
        out["starts"].append([su, rec[si0:si0 + nci + 1].astype(np.int64)])
    return out
