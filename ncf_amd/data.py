"""Data path of the NeuMF hot loop: ``load_all`` / ``NCFData`` (reference
src/data/datasets.py:9-83) with the same signatures and semantics, backed by
numpy arrays and the C++ negative sampler (libncf_sampler.so).

* ``NCFData.ng_sample`` consumes NumPy's *global* legacy RandomState exactly
  like the reference's Python loop (datasets.py:57-63): the sampler reads the
  state with ``np.random.get_state()``, draws in C++, and writes it back with
  ``np.random.set_state()``.  Negatives are bit-identical.
* ``__getitem__`` returns python ints like the reference; ``__getitems__``
  (torch >= 2 batched fetch) returns ``[users, items, labels]`` int64 tensors,
  which the default collate stacks to ``[3, B]`` so ``for user, item, label in
  loader`` still unpacks correctly while avoiding per-sample Python.
* ``load_all`` parses the reference file formats literally (no ``eval``).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.utils.data as data

from . import _lib as L


def _state_arrays():
    st = np.random.get_state(legacy=True)
    if st[0] != "MT19937":
        raise RuntimeError("numpy global generator is not MT19937")
    key = np.ascontiguousarray(st[1], dtype=np.uint32).copy()
    pos = np.array([st[2]], dtype=np.int32)
    return st, key, pos


class HostSampler:
    """Membership index + bit-exact legacy-MT19937 negative draws (C++,
    libncf_sampler.so).  The runs come from the positives in file order
    (datasets.py:57: ``for x in self.features_ps``), membership from
    ``mem_users / mem_items`` (the keys of ``train_mat``, datasets.py:61), which
    default to the positives.  ``threads``: the parallel pass's pool (default
    ``sampler_threads(len(pos_users))``; 1 = the sequential pass)."""

    def __init__(self, pos_users, pos_items, num_users, num_items, mem_users=None, mem_items=None, threads=None):
        self.pos_users = np.ascontiguousarray(pos_users, dtype=np.int32)
        self.pos_items = np.ascontiguousarray(pos_items, dtype=np.int32)
        if mem_users is None:
            mem_users, mem_items = self.pos_users, self.pos_items
        self.mem_users = np.ascontiguousarray(mem_users, dtype=np.int32)
        self.mem_items = np.ascontiguousarray(mem_items, dtype=np.int32)
        self._h = L.sampler_lib().ncf_sampler_create2(self.pos_users.ctypes.data, len(self.pos_users),
                                                      self.mem_users.ctypes.data, self.mem_items.ctypes.data,
                                                      len(self.mem_users), int(num_users), int(num_items))
        if not self._h:
            raise RuntimeError("ncf_sampler_create2 failed")
        self.num_users, self.num_items = int(num_users), int(num_items)
        self.set_threads(sampler_threads(len(pos_users)) if threads is None else threads)

    def set_threads(self, threads):
        if L.sampler_lib().ncf_sampler_set_threads(self._h, int(threads)) != 0:
            raise ValueError(f"sampler threads {threads}")
        self.threads = int(threads)

    def stats(self):
        """(parallel passes, sequential passes, runs walked directly, parallel passes
        redone sequentially, threads, blocks, ns: words / walk / end state / chain,
        window bits) of this sampler."""
        import ctypes
        out = (ctypes.c_int64 * 13)()
        L.sampler_lib().ncf_sampler_stats(self._h, out, 13)
        keys = ("parallel", "sequential", "run_fallbacks", "epoch_fallbacks", "threads", "blocks",
                "words_ns", "walk_ns", "end_ns", "chain_ns", "window_bits", "tab_thread_ns", "fin_thread_ns")
        return dict(zip(keys, list(out)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                L.sampler_lib().ncf_sampler_destroy(h)
            except Exception:
                pass

    def contains(self, u, i):
        return bool(L.sampler_lib().ncf_sampler_contains(self._h, int(u), int(i)))

    def sample(self, num_item, num_ng, key=None, pos=None, out=None):
        """Negatives for every positive (file order) x num_ng.  With key/pos None
        NumPy's global stream is used and advanced (the np.random.seed protocol);
        else the given state arrays (uint32[624], int32[1]) are advanced in place.
        out: optional int32 destination (e.g. pinned staging)."""
        use_global = key is None
        if use_global:
            st, key, pos = _state_arrays()
        n = len(self.pos_users) * int(num_ng)
        if out is None:
            out = np.empty(n, dtype=np.int32)
        elif out.dtype != np.int32 or not out.flags.c_contiguous or len(out) < n:
            raise ValueError("out: contiguous int32 of at least n_pos * num_ng")
        words = L.sampler_lib().ncf_sampler_sample(self._h, int(num_item), int(num_ng), key.ctypes.data,
                                                   pos.ctypes.data, out.ctypes.data)
        if words == -2:
            # the reference's `while (u, j) in train_mat` never ends for a user who owns
            # every item in [0, num_item): refuse instead of hanging
            raise RuntimeError("ng_sample: a user has every item as a positive (the reference loops forever)")
        if words < 0:
            raise RuntimeError("ncf_sampler_sample: bad arguments")
        if use_global:
            np.random.set_state((st[0], key, int(pos[0]), st[3], st[4]))  # the cached Gaussian stays
        return out


def sampler_threads(work=None):
    """Threads of a host sampler pool: NCF_SAMPLER_THREADS, else min(12, half this
    rank's share of the CPUs the process may run on), and, given the pass's size
    `work` in positives, at most one thread per 125,000 of them (at least 4).  A GPU
    box grants 16 CPUs per GPU, and the rest are the training loop's (graph replays,
    the epoch pipeline's staging, the HIP runtime): the pool only has to finish an
    epoch's draws while the previous epoch trains (ml-20m on the box: 42 ms per epoch
    at 8 threads, 27 ms at 12; ml-1m, 994K positives: 1.4 ms at 8 threads against
    1.9 ms at 12, profiles/r03_final/sampler_ml-1m.json and
    profiles/r03_evidence/r03c_sampler_ml1m.jsonl).  The share is the CPUs divided by
    LOCAL_WORLD_SIZE (set by torch.distributed.run and by bench.py's own spawn): the
    pools spin-wait inside a pass, so N local ranks must not each size theirs for
    the whole machine."""
    import os
    v = os.environ.get("NCF_SAMPLER_THREADS")
    if v:
        return max(1, int(v))
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    lws = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
    t = max(1, min(12, (n // lws) // 2))
    if work is not None:
        t = min(t, max(4, -(-int(work) // 125_000)))
    return t


def _membership_from(train_mat, features):
    if train_mat is not None and hasattr(train_mat, "keys") and hasattr(train_mat, "shape"):
        ks = np.array(list(train_mat.keys()), dtype=np.int64).reshape(-1, 2)
        return ks[:, 0].astype(np.int32), ks[:, 1].astype(np.int32), train_mat.shape
    return None


class NCFData(data.Dataset):
    """Reference ``NCFData`` (datasets.py:39-83), array-backed."""

    def __init__(self, features, num_item, train_mat=None, num_ng=0, is_training=None):
        super().__init__()
        f = np.asarray(features, dtype=np.int64).reshape(-1, 2)
        self._ps_u = np.ascontiguousarray(f[:, 0], dtype=np.int32)
        self._ps_i = np.ascontiguousarray(f[:, 1], dtype=np.int32)
        self.num_item = num_item
        self.train_mat = train_mat
        self.num_ng = num_ng
        self.is_training = is_training
        self.labels = np.zeros(len(f), dtype=np.int64)
        self._fill_u = self._fill_i = self._fill_y = None
        self._ng_u = self._ng_i = None
        self._neg_dev = None  # negatives drawn on the device (ncf_amd.pipeline), fetched on use
        self._sampler = None

    # -- compatibility views (lists, like the reference) ---------------------
    @property
    def features_ps(self):
        return np.stack([self._ps_u, self._ps_i], 1).astype(np.int64).tolist()

    @property
    def features_ng(self):
        self._materialize()
        return np.stack([self._ng_u, self._ng_i], 1).astype(np.int64).tolist()

    @property
    def features_fill(self):
        self._materialize()
        return np.stack([self._fill_u, self._fill_i], 1).astype(np.int64).tolist()

    @property
    def labels_fill(self):
        self._materialize()
        return self._fill_y.astype(np.int64).tolist()

    # -- arrays for the device engine ----------------------------------------
    def _set_negatives(self, neg):
        self._ng_u = np.repeat(self._ps_u, self.num_ng)
        self._ng_i = neg
        self._fill_u = np.concatenate([self._ps_u, self._ng_u])
        self._fill_i = np.concatenate([self._ps_i, self._ng_i])
        self._fill_y = np.concatenate([np.ones(len(self._ps_u), dtype=np.int64),
                                       np.zeros(len(self._ng_u), dtype=np.int64)])

    def _set_device_negatives(self, neg_dev):
        """This epoch's negatives live on the device (ng_sample done there); the host
        arrays are rebuilt from them only if something asks for them."""
        self._neg_dev = neg_dev if neg_dev is not None else None
        if neg_dev is None:
            self._set_negatives(np.zeros(0, dtype=np.int32))

    def _materialize(self):
        if self._neg_dev is not None:
            neg = self._neg_dev.cpu().numpy().astype(np.int32)
            self._neg_dev = None
            self._set_negatives(neg)

    def arrays(self):
        """(users int32, items int32, labels float32) in reference fill order."""
        self._materialize()
        if self.is_training:
            return self._fill_u, self._fill_i, self._fill_y.astype(np.float32)
        return self._ps_u, self._ps_i, self.labels.astype(np.float32)

    def _get_sampler(self):
        """The sampler over this data set: runs from the positives (file order),
        membership from ``train_mat``'s keys (``(u, j) in train_mat``,
        datasets.py:61) -- any dok_matrix, duplicates or extra pairs included --
        or from the positives when ``train_mat`` is None."""
        if self._sampler is None:
            mem = _membership_from(self.train_mat, None)
            n_users = int(max(self._ps_u.max(initial=0) + 1, mem[2][0] if mem else 0, 1))
            n_items = int(max(self.num_item, mem[2][1] if mem else 0, 1))
            if mem is None:
                self._sampler = HostSampler(self._ps_u, self._ps_i, n_users, n_items)
            else:
                self._sampler = HostSampler(self._ps_u, self._ps_i, n_users, n_items, mem[0], mem[1])
        return self._sampler

    def ng_sample(self):
        assert self.is_training, "no need to sampling when testing"
        self._neg_dev = None
        self._set_negatives(self._get_sampler().sample(self.num_item, self.num_ng))

    def __len__(self):
        return (self.num_ng + 1) * len(self.labels)

    def __getitem__(self, idx):
        if self._neg_dev is not None:
            self._materialize()
        if self.is_training:
            return int(self._fill_u[idx]), int(self._fill_i[idx]), int(self._fill_y[idx])
        return int(self._ps_u[idx]), int(self._ps_i[idx]), int(self.labels[idx])

    def __getitems__(self, indices):
        self._materialize()
        idx = np.asarray(indices, dtype=np.int64)
        if self.is_training:
            u, i, y = self._fill_u[idx], self._fill_i[idx], self._fill_y[idx]
        else:
            u, i, y = self._ps_u[idx], self._ps_i[idx], self.labels[idx]
        return [torch.from_numpy(u.astype(np.int64)), torch.from_numpy(i.astype(np.int64)),
                torch.from_numpy(np.asarray(y, dtype=np.int64))]


def parse_train_rating(path):
    import pandas as pd
    df = pd.read_csv(path, sep="\t", header=None, names=["user", "item"], usecols=[0, 1],
                     dtype={0: np.int32, 1: np.int32})
    return df["user"].to_numpy(np.int32), df["item"].to_numpy(np.int32)


def parse_test_negative(path):
    """'(u,pos)\\tn1\\t...' lines -> (users, items) int32 in file order, pos first."""
    us, its = [], []
    with open(path, "r") as fd:
        for line in fd:
            line = line.rstrip("\n")
            if not line:
                continue
            arr = line.split("\t")
            head = arr[0].strip()
            if not (head.startswith("(") and head.endswith(")")):
                raise ValueError(f"bad test-negative line head: {head!r}")
            u_s, p_s = head[1:-1].split(",")
            u = int(u_s)
            us.append(u)
            its.append(int(p_s))
            for x in arr[1:]:
                us.append(u)
                its.append(int(x))
    return np.asarray(us, dtype=np.int32), np.asarray(its, dtype=np.int32)


def load_all(test_num=100):
    """Reference ``load_all`` (datasets.py:9-36): same return tuple."""
    import scipy.sparse as sp

    from .config import config
    tu, ti = parse_train_rating(config.train_rating)
    user_num = int(tu.max()) + 1
    item_num = int(ti.max()) + 1
    train_data = np.stack([tu, ti], 1).astype(np.int64).tolist()
    coo = sp.coo_matrix((np.ones(len(tu), dtype=np.float32), (tu, ti)), shape=(user_num, item_num))
    coo.sum_duplicates()
    coo.data[:] = 1.0
    train_mat = coo.todok()
    eu, ei = parse_test_negative(config.test_negative)
    test_data = np.stack([eu, ei], 1).astype(np.int64).tolist()
    return train_data, test_data, user_num, item_num, train_mat


def epoch_permutation_seed(generator=None, peek=False):
    """The two draws a DataLoader(shuffle=True) epoch makes on the torch global (or
    given) generator -- one int64 base_seed by the loader iterator, one int64
    seeding RandomSampler's private generator -- returning the latter
    (scripts/train_neumf.py:55,106; torch/utils/data).  peek: restore the
    generator afterwards (nothing consumed)."""
    if peek:
        state = generator.get_state() if generator is not None else torch.get_rng_state()
    try:
        torch.empty((), dtype=torch.int64).random_(generator=generator)
        return int(torch.empty((), dtype=torch.int64).random_(generator=generator).item())
    finally:
        if peek:
            if generator is not None:
                generator.set_state(state)
            else:
                torch.set_rng_state(state)


def epoch_permutation(n, generator=None):
    """DataLoader(shuffle=True) epoch order: epoch_permutation_seed, then
    randperm(n) on a generator seeded with it."""
    seed = epoch_permutation_seed(generator)
    g = torch.Generator()
    g.manual_seed(seed)
    return torch.randperm(n, generator=g)


def consume_test_pass(generator=None):
    """A metrics() pass over the (unshuffled) test DataLoader draws one base_seed."""
    torch.empty((), dtype=torch.int64).random_(generator=generator)
