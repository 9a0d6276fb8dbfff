"""Synthetic MovieLens-shaped interaction data (no network: real MovieLens files
are not available).  Shapes follow SURVEY.md section 8(d):

    ml-100k    943 users x  1,682 items x     100,000 ratings
    ml-1m    6,040 users x  3,706 items x   1,000,209 ratings
    ml-20m 138,493 users x 26,744 items x  20,000,263 ratings

Ids are 1-based like MovieLens, so ``user_num = max id + 1`` (row 0 unused),
exactly as ``load_all`` computes it (reference src/data/datasets.py:16-17).
Users get lognormal activity with at least 20 ratings; items are drawn without
replacement per user from a Zipf(0.8) popularity; timestamps are uniform.  The
split is the reference's temporal leave-one-out (src/data/preprocessing.py:45-90):
each user's last interaction is the test positive, the rest are training rows in
timestamp order; 99 test negatives per user are distinct non-interacted items,
written sorted (preprocessing.py:92-135).
"""
from __future__ import annotations

import os

import numpy as np

SHAPES = {
    "tiny": (60, 400, 1_800),  # test-sized: script-compatibility tests
    "ml-100k": (943, 1682, 100_000),
    "ml-1m": (6040, 3706, 1_000_209),
    "ml-20m": (138_493, 26_744, 20_000_263),
}


def _counts(rng, n_users, n_items, n_ratings, min_per_user=20):
    w = rng.lognormal(0.0, 1.0, n_users)
    extra = n_ratings - min_per_user * n_users
    c = min_per_user + np.floor(w / w.sum() * extra).astype(np.int64)
    cap = max(min_per_user, n_items // 2)
    c = np.minimum(c, cap)
    short = n_ratings - int(c.sum())
    order = np.argsort(-w)
    k = 0
    while short > 0:
        u = order[k % n_users]
        if c[u] < cap:
            c[u] += 1
            short -= 1
        k += 1
    return c


def _first_unique(user, item):
    """Mask (in draw order) of the first draw of each (user, item) pair."""
    k = user.astype(np.int64) * (1 << 32) + item.astype(np.int64)
    order = np.argsort(k, kind="stable")
    ks = k[order]
    first = np.ones(len(ks), dtype=bool)
    first[1:] = ks[1:] != ks[:-1]
    keep = np.zeros(len(ks), dtype=bool)
    keep[order[first]] = True
    return keep


def _make_large(n_users, n_items, n_ratings, seed, zipf_a, test_neg):
    """The same design as make_dataset, vectorised for ml-20m-sized shapes (the
    per-user Gumbel top-k over every item would draw U x I = 3.7G keys): items per
    user drawn from the Zipf popularity with replacement and de-duplicated in draw
    order (more draws until a user has its count; users holding more than a tenth
    of the items take the exact Gumbel top-k), uniform timestamps, the temporal
    leave-one-out split and 99 distinct non-interacted test negatives, sorted."""
    rng = np.random.default_rng(seed)
    counts = _counts(rng, n_users, n_items, n_ratings)
    logp = -zipf_a * np.log(np.arange(1, n_items + 1, dtype=np.float64))
    pop = np.exp(logp - logp.max())
    cdf = np.cumsum(pop / pop.sum())
    item_of_rank = rng.permutation(n_items)
    heavy = counts > n_items // 10
    users, items = [], []
    need = np.where(heavy, 0, counts)
    have = np.zeros(n_users, dtype=np.int64)
    pool_u = np.zeros(0, dtype=np.int32)
    pool_i = np.zeros(0, dtype=np.int32)
    while True:
        short = need - have
        todo = np.nonzero(short > 0)[0]
        if len(todo) == 0:
            break
        draws = (short[todo] * 1.25 + 8).astype(np.int64)
        du = np.repeat(todo.astype(np.int32), draws)
        di = item_of_rank[np.minimum(np.searchsorted(cdf, rng.random(len(du))), n_items - 1)].astype(np.int32)
        pool_u = np.concatenate([pool_u, du])
        pool_i = np.concatenate([pool_i, di])
        keep = _first_unique(pool_u, pool_i)
        pool_u, pool_i = pool_u[keep], pool_i[keep]
        # at most `need` per user, in draw order
        order = np.argsort(pool_u, kind="stable")
        su = pool_u[order]
        start = np.searchsorted(su, np.arange(n_users))
        rank = np.arange(len(su)) - start[su]
        ok = rank < need[su]
        pool_u, pool_i = su[ok], pool_i[order][ok]
        have = np.bincount(pool_u, minlength=n_users)
    users.append(pool_u)
    items.append(pool_i)
    for u in np.nonzero(heavy)[0]:  # exact sampling without replacement for the heaviest users
        keys = logp + rng.gumbel(size=n_items)
        sel = np.argpartition(-keys, counts[u] - 1)[: counts[u]]
        users.append(np.full(counts[u], u, dtype=np.int32))
        items.append(item_of_rank[sel].astype(np.int32))
    u = np.concatenate(users)
    it = np.concatenate(items)
    ts = rng.random(len(u))
    order = np.lexsort((ts, u))  # per user, by timestamp
    u, it = u[order], it[order]
    last = np.ones(len(u), dtype=bool)
    last[:-1] = u[1:] != u[:-1]
    train_users = (u[~last] + 1).astype(np.int32)
    train_items = (it[~last] + 1).astype(np.int32)
    test_users = (u[last] + 1).astype(np.int32)
    test_items = (it[last] + 1).astype(np.int32)
    # test negatives: distinct ids in [1, n_items] the user never rated
    seen = np.sort(u.astype(np.int64) * (n_items + 1) + it + 1)
    negs = np.zeros((n_users, test_neg), dtype=np.int32)
    filled = np.zeros(n_users, dtype=np.int64)
    todo = np.arange(n_users)
    while len(todo):
        m = 2 * test_neg
        cu = np.repeat(todo, m)
        ci = rng.integers(1, n_items + 1, len(cu))
        key = cu.astype(np.int64) * (n_items + 1) + ci
        pos = np.minimum(np.searchsorted(seen, key), len(seen) - 1)
        ok = seen[pos] != key
        cu, ci = cu[ok], ci[ok]
        # drop candidates already chosen for the user, then duplicates, keep draw order
        prev = np.repeat(np.arange(n_users), test_neg).reshape(n_users, test_neg)[todo]
        pu = prev.reshape(-1)
        pi = negs[todo].reshape(-1)
        pk = filled[todo][:, None] > np.arange(test_neg)[None, :]
        allu = np.concatenate([pu[pk.reshape(-1)], cu])
        alli = np.concatenate([pi[pk.reshape(-1)], ci])
        keep = _first_unique(allu, alli)
        n_prev = int(pk.sum())
        cu, ci = cu[keep[n_prev:]], ci[keep[n_prev:]]
        order = np.argsort(cu, kind="stable")
        cu, ci = cu[order], ci[order]
        start = np.searchsorted(cu, np.arange(n_users))
        rank = np.arange(len(cu)) - start[cu] + filled[cu]
        ok = rank < test_neg
        negs[cu[ok], rank[ok]] = ci[ok]
        filled = np.minimum(test_neg, filled + np.bincount(cu[ok], minlength=n_users))
        todo = np.nonzero(filled < test_neg)[0]
    negs.sort(axis=1)
    return {
        "train_users": train_users,
        "train_items": train_items,
        "test_users": test_users,
        "test_items": test_items,
        "test_negatives": negs,
        "user_num": int(train_users.max()) + 1,
        "item_num": int(train_items.max()) + 1,
    }


def make_dataset(shape="ml-1m", seed=0, zipf_a=0.8, test_neg=99):
    """Return a dict of int32 arrays in reference order (see module docstring).
    Shapes above 1G user x item pairs (ml-20m) use the vectorised generator of the
    same design (_make_large)."""
    n_users, n_items, n_ratings = SHAPES[shape] if isinstance(shape, str) else shape
    if n_users * n_items > 1_000_000_000:
        return _make_large(n_users, n_items, n_ratings, seed, zipf_a, test_neg)
    rng = np.random.default_rng(seed)
    counts = _counts(rng, n_users, n_items, n_ratings)
    logp = -zipf_a * np.log(np.arange(1, n_items + 1, dtype=np.float64))
    item_of_rank = rng.permutation(n_items)  # popularity rank -> item index
    tr_u, tr_i, te_u, te_i = [], [], [], []
    negs = np.empty((n_users, test_neg), dtype=np.int32)
    chunk = max(1, int(4_000_000 // n_items))
    for u0 in range(0, n_users, chunk):
        u1 = min(n_users, u0 + chunk)
        keys = logp[None, :] + rng.gumbel(size=(u1 - u0, n_items))     # Gumbel-top-k = sampling w/o replacement
        kmax = int(counts[u0:u1].max())
        top = np.argpartition(-keys, kmax - 1, axis=1)[:, :kmax]
        for r in range(u1 - u0):
            u = u0 + r
            k = int(counts[u])
            sel = top[r]
            sel = sel[np.argsort(-keys[r, sel])][:k]
            items = item_of_rank[sel]
            ts = rng.random(k)                                          # uniform timestamps
            items = items[np.argsort(ts, kind="stable")]
            uid = u + 1
            tr_u.append(np.full(k - 1, uid, dtype=np.int32))
            tr_i.append((items[:-1] + 1).astype(np.int32))
            te_u.append(uid)
            te_i.append(int(items[-1]) + 1)
            seen = np.zeros(n_items + 1, dtype=bool)
            seen[items + 1] = True
            seen[0] = True  # id 0 never occurs in MovieLens; keep it out of the candidates too
            cand = rng.integers(1, n_items + 1, size=4 * test_neg + 64)
            cand = cand[~seen[cand]]
            _, first = np.unique(cand, return_index=True)
            cand = cand[np.sort(first)]
            while len(cand) < test_neg:
                more = rng.integers(1, n_items + 1, size=4 * test_neg)
                more = more[~seen[more]]
                cand = np.concatenate([cand, more])
                _, first = np.unique(cand, return_index=True)
                cand = cand[np.sort(first)]
            negs[u] = np.sort(cand[:test_neg])
    train_users = np.concatenate(tr_u)
    train_items = np.concatenate(tr_i)
    return {
        "train_users": train_users,
        "train_items": train_items,
        "test_users": np.asarray(te_u, dtype=np.int32),
        "test_items": np.asarray(te_i, dtype=np.int32),
        "test_negatives": negs,
        "user_num": int(train_users.max()) + 1,
        "item_num": int(train_items.max()) + 1,
    }


def write_reference_files(ds, out_dir):
    """u.train.rating ('u\\ti' lines) and u.test.negative ('(u,pos)\\tn1\\t...')
    in the formats load_all parses (datasets.py:9-36, preprocessing.py:132)."""
    os.makedirs(out_dir, exist_ok=True)
    tr = os.path.join(out_dir, "u.train.rating")
    np.savetxt(tr, np.stack([ds["train_users"], ds["train_items"]], 1), fmt="%d", delimiter="\t")
    te = os.path.join(out_dir, "u.test.rating")
    np.savetxt(te, np.stack([ds["test_users"], ds["test_items"]], 1), fmt="%d", delimiter="\t")
    neg = os.path.join(out_dir, "u.test.negative")
    with open(neg, "w") as f:
        lines = []
        for u, p, row in zip(ds["test_users"].tolist(), ds["test_items"].tolist(), ds["test_negatives"]):
            lines.append(f"({u},{p})\t" + "\t".join(map(str, row.tolist())))
        f.write("\n".join(lines))
    return tr, neg
