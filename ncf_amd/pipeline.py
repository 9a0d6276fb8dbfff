"""Epoch pipeline: the per-epoch data path of the reference loop
(scripts/train_neumf.py:98-106), bit-exact, with the next epoch's host work
done on host threads while the current epoch trains.

Per epoch the reference does
  train_loader.dataset.ng_sample()        datasets.py:53-69, NumPy global MT19937
  for user, item, label in train_loader   DataLoader(shuffle=True): torch global
                                          generator draws base_seed and the
                                          RandomSampler seed, then randperm(n)
and this module produces the same batches as one packed device stream:
  host    the negatives (libncf_sampler.so, blocked C++ sampler: the draws are a
          sequential scan), the torch generator's words for the permutation
          (ncf_mt_words); pinned staging, upload on a copy stream
  device  ncf_build_rows (features_fill / labels_fill), ncf_randperm (Fisher-Yates
          in closed form, three passes), ncf_prepare_epoch (batch membership, grouped by item)
The NumPy global state ends where ng_sample leaves it and the torch generator
has made exactly the DataLoader's two draws, so everything after an epoch sees
the generators the reference would leave behind.

Prefetch: epoch e+1's negatives are drawn from the NumPy state epoch e left, on a
host thread, while epoch e trains; its sampler seed is *peeked* (the torch state
is saved, the metrics() pass's draw and the next two DataLoader draws are made,
the state restored) and its permutation words generated on a second thread; its
rows, permutation and grouping by item are then built on a side stream, under
epoch e's steps, into the other of two output buffers (the step graphs are
captured once per buffer), so the epoch boundary is one stream wait.
When epoch e+1 starts, the real draws are made and compared with what was used;
a mismatch (someone else consumed either generator in between) discards the
prefetch, and the epoch is built synchronously.
"""
from __future__ import annotations

import collections
import os
import threading
import time

import numpy as np
import torch

from . import _lib as L
from . import ops
from .data import epoch_permutation_seed


def _mt_state():
    """(key, pos, (has_gauss, cached_gaussian)) of numpy's global legacy generator."""
    st = np.random.get_state(legacy=True)
    if st[0] != "MT19937":
        raise RuntimeError("numpy global generator is not MT19937")
    return np.ascontiguousarray(st[1], dtype=np.uint32).copy(), int(st[2]), (int(st[3]), float(st[4]))


class WordsGen:
    """Parallel MT19937 word generator (libncf_sampler.so ncf_words_fill: chunks of
    the stream on `threads` host threads, each from the state jumped to its first
    word; same words as the sequential ncf_mt_words)."""

    def __init__(self, threads=None):
        from .data import sampler_threads
        self.threads = sampler_threads() if threads is None else int(threads)
        self._h = L.sampler_lib().ncf_words_create(self.threads)
        if not self._h:
            raise RuntimeError("ncf_words_create failed")

    def fill(self, key, pos, n, out):
        if L.sampler_lib().ncf_words_fill(self._h, key.ctypes.data, pos.ctypes.data, int(n), out.ctypes.data) != 0:
            raise RuntimeError("ncf_words_fill: bad arguments")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                L.sampler_lib().ncf_words_destroy(h)
            except Exception:
                pass


def torch_words(seed, n, out, gen=None):
    """The first n 32-bit words of torch.Generator().manual_seed(seed) (MT19937 on
    the low 32 bits of the seed) into out (uint32); `gen`: a WordsGen (parallel)."""
    key = np.empty(624, dtype=np.uint32)
    pos = np.empty(1, dtype=np.int32)
    lib = L.sampler_lib()
    lib.ncf_mt_seed(int(seed) & 0xFFFFFFFF, key.ctypes.data, pos.ctypes.data)
    if n > 0:
        if gen is not None:
            gen.fill(key, pos, n, out)
        else:
            lib.ncf_mt_words(key.ctypes.data, pos.ctypes.data, int(n), out.ctypes.data)


class _Staged:
    """One epoch's host products (negatives, permutation words), their upload and
    device build."""

    def __init__(self, slot, key, pos, seed):
        self.slot, self.key, self.pos, self.seed = slot, key, pos, seed
        self.end_key = self.end_pos = None  # NumPy state after the epoch's ng_sample
        self.event = None   # uploads done
        self.t0 = None
        self.built = None   # rows + permutation built
        self.ready = None   # grouped epoch stream written
        self.error = None
        self.host_ms = {}
        self.thread = None
        self.sampled = threading.Event()   # end_key / end_pos known (or error)
        self.enqueued = threading.Event()  # device build issued (or error)


class EpochPipeline:
    """depth: epochs staged ahead (host draws, uploads and device build); slots =
    depth + 1 sets of buffers, one being trained from."""

    def __init__(self, dataset, device, batch_size, item_num, user_num=None, prefetch=True, depth=None,
                 canonical=None):
        """canonical: rows of one item inside a batch in (user, label) order
        (ncf_prepare_epoch2 NCF_PREP_CANONICAL) -- every rank of a data-parallel group
        then builds the identical stream; None: on when torch.distributed runs more
        than one rank (ops.default_canonical)."""
        self.ds = dataset
        self.device = torch.device(device)
        self.batch_size = int(batch_size)
        self.item_num = int(item_num)
        pu, pi = dataset._ps_u, dataset._ps_i
        self.P = len(pu)
        self.ng = int(dataset.num_ng)
        self.num_item = int(dataset.num_item)
        if self.P == 0:
            raise ValueError("no training positives")
        user_num = int(user_num) if user_num is not None else int(pu.max()) + 1
        ops.check_ids(pu, pi, user_num, self.item_num)  # once: the negatives are < num_item
        if self.ng > 0 and self.num_item > self.item_num:
            raise IndexError("index out of range in self (sampled item id >= item_num)")
        dev = self.device
        self.pu = torch.as_tensor(pu, dtype=torch.int32).to(dev)
        self.pi = torch.as_tensor(pi, dtype=torch.int32).to(dev)
        self.S = self.P * self.ng
        self.n = self.P + self.S
        if depth is None:
            depth = int(os.environ.get("NCF_PIPE_DEPTH", "2"))
        self.depth = max(1, int(depth)) if prefetch else 0
        self.prefetch = prefetch
        K = self.depth + 1
        # shared by the builds (issued in epoch order on one stream)
        self.rows = torch.empty(self.n, dtype=torch.int64, device=dev)
        self.perm = torch.empty(self.n, dtype=torch.int64, device=dev)
        self.fy_ws = torch.empty(int(L.hip().ncf_randperm_workspace(self.n)), dtype=torch.uint8, device=dev)
        self.prep = ops.EpochPrep(dev, canonical=canonical)
        # per slot
        self._out = [torch.empty(self.n, dtype=torch.int64, device=dev) for _ in range(K)]
        self._neg_host = [torch.empty(max(1, self.S), dtype=torch.int32).pin_memory() for _ in range(K)]
        self._words_host = [torch.empty(max(1, self.n - 1), dtype=torch.int32).pin_memory() for _ in range(K)]
        self._neg_dev = [torch.empty(max(1, self.S), dtype=torch.int32, device=dev) for _ in range(K)]
        self._words_dev = [torch.empty(max(1, self.n - 1), dtype=torch.int32, device=dev) for _ in range(K)]
        self._uploaded = [None] * K  # the uploads last issued from the slot's pinned buffers
        self._free = [None] * K      # main-stream point after which the slot's last epoch is done
        self._next_slot = 0
        self._cur_slot = None
        self._pending = collections.deque()  # staged epochs, in epoch order
        self.copy_stream = torch.cuda.Stream(device=dev)
        self.side_stream = torch.cuda.Stream(device=dev)
        self.stats = {"epochs": 0, "prefetch_hits": 0}
        self._wordgen = WordsGen()
        self.events = None  # (start, rows+perm built, grouped) of the last epoch
        # on_built(rows_out, stream): called after each epoch's build, on the build's
        # stream (the worker thread for a prefetched epoch), e.g. TrainEngine.owner_prebuild
        self.on_built = None

    # ---------------------------------------------------------------- host part
    def _take_slot(self):
        k = self._next_slot
        self._next_slot = (k + 1) % len(self._out)
        return k

    def _stage(self, s):
        """Negatives from NumPy state (s.key, s.pos) and the permutation words of
        s.seed, staged in the slot's pinned buffers and uploaded."""
        slot = s.slot
        t_all = time.perf_counter()
        neg = self._neg_host[slot].numpy()
        words = self._words_host[slot].numpy().view(np.uint32)
        prev, self._uploaded[slot] = self._uploaded[slot], None
        if prev is not None:
            prev.synchronize()  # the slot's pinned buffers are no longer being read
        # the negatives, then the permutation words, each on its own pool of host
        # threads (the next epoch's negatives wait only for the negatives)
        try:
            t0 = time.perf_counter()
            if self.S == 0:
                s.end_key, s.end_pos = s.key.copy(), s.pos
            else:
                k2, p2 = s.key.copy(), np.array([s.pos], dtype=np.int32)
                self.ds._get_sampler().sample(self.num_item, self.ng, k2, p2, out=neg[: self.S])
                s.end_key, s.end_pos = k2, int(p2[0])
            s.host_ms["sample"] = (time.perf_counter() - t0) * 1e3
        finally:
            s.sampled.set()
        t0 = time.perf_counter()
        torch_words(s.seed, self.n - 1, words[: self.n - 1], self._wordgen)
        s.host_ms["words"] = (time.perf_counter() - t0) * 1e3
        with torch.cuda.stream(self.copy_stream):
            if self._free[slot] is not None:
                self.copy_stream.wait_event(self._free[slot])  # the slot's device buffers
            if self.S:
                self._neg_dev[slot][: self.S].copy_(self._neg_host[slot][: self.S], non_blocking=True)
            if self.n > 1:
                self._words_dev[slot][: self.n - 1].copy_(self._words_host[slot][: self.n - 1], non_blocking=True)
            s.event = torch.cuda.Event()
            s.event.record(self.copy_stream)
            self._uploaded[slot] = s.event
        s.host_ms["stage"] = (time.perf_counter() - t_all) * 1e3

    def _device_build(self, staged, stream):
        """On `stream`, after the staged uploads and after the main stream let go of
        the slot: the epoch's packed rows, its permutation and the batch stream
        grouped by item, into the slot's output.  Records staged.built / .ready."""
        lib = L.hip()
        slot = staged.slot
        st = stream.cuda_stream
        stream.wait_event(staged.event)
        if self._free[slot] is not None:
            stream.wait_event(self._free[slot])
        staged.t0 = torch.cuda.Event(enable_timing=True)
        staged.t0.record(stream)
        L.check(lib.ncf_build_rows(self.pu.data_ptr(), self.pi.data_ptr(), self.P,
                                   self._neg_dev[slot].data_ptr() if self.S else None, self.ng,
                                   self.rows.data_ptr(), st), "ncf_build_rows")
        L.check(lib.ncf_randperm(self._words_dev[slot].data_ptr(), self.n, self.perm.data_ptr(),
                                 self.fy_ws.data_ptr(), self.fy_ws.numel(), st), "ncf_randperm")
        staged.built = torch.cuda.Event(enable_timing=True)
        staged.built.record(stream)
        with torch.cuda.stream(stream):
            self.prep(self.rows, self.perm, self.batch_size, self.item_num, out=self._out[slot])
        staged.ready = torch.cuda.Event(enable_timing=True)
        staged.ready.record(stream)
        hook = self.on_built
        if hook is not None:  # per-stream work of the consumer, on the same stream (e.g. owner lists)
            with torch.cuda.stream(stream):
                hook(self._out[slot], stream)

    def _launch(self, seed, prev, key=None, pos=None):
        """Stage the epoch after `prev` (or from (key, pos)) on a worker thread."""
        s = _Staged(self._take_slot(), None if key is None else key.copy(), pos, seed)

        def work():
            try:
                if s.key is None:
                    prev.sampled.wait()
                    if prev.end_key is None:
                        raise RuntimeError("the previous epoch's prefetch failed")
                    s.key, s.pos = prev.end_key.copy(), prev.end_pos
                self._stage(s)
                if prev is not None:
                    prev.enqueued.wait()  # builds are issued to the side stream in epoch order
                self._device_build(s, self.side_stream)
            except Exception as e:  # surfaced when the epoch is consumed
                s.error = e
            finally:
                s.sampled.set()
                s.enqueued.set()
        s.thread = threading.Thread(target=work, daemon=True)
        s.thread.start()
        self._pending.append(s)
        return s

    def _discard_pending(self):
        """Drop every staged epoch (their builds still write shared buffers: wait)."""
        first = None
        while self._pending:
            s = self._pending.popleft()
            s.thread.join()
            if s.ready is not None:
                s.ready.synchronize()
            first = s.slot if first is None else first
        if first is not None:
            self._next_slot = first

    # ---------------------------------------------------------------- API
    def _peek_seeds(self, eval_draw, count):
        """The RandomSampler seeds of the next `count` epochs, each past a metrics()
        draw if `eval_draw` (train_neumf.py:120), consuming nothing."""
        state = torch.get_rng_state()
        out = []
        try:
            for _ in range(count):
                if eval_draw:
                    torch.empty((), dtype=torch.int64).random_()   # the test loader's base_seed
                out.append(epoch_permutation_seed())              # base_seed, sampler seed
        finally:
            torch.set_rng_state(state)
        return out

    def next_epoch(self, peek_eval_draw=True):
        """The epoch's packed stream in batch order (device), consuming the NumPy
        global stream (ng_sample) and the torch global generator (DataLoader)
        exactly like the reference's epoch.  peek_eval_draw: a metrics() pass
        (one torch draw) follows each epoch before the next next_epoch().

        With a prefetch hit the whole stream was built on a side stream while
        earlier epochs trained: the current stream only waits for it.  The result
        is one of depth + 1 rotating buffers, valid for `depth` further calls."""
        t_enter = time.perf_counter()
        key, pos, gauss = _mt_state()
        seed = epoch_permutation_seed()  # the DataLoader's two draws
        staged = self._pending.popleft() if self._pending else None
        if staged is not None:
            staged.thread.join()
        t_joined = time.perf_counter()
        dev = self.device
        cur = torch.cuda.current_stream(dev)
        if (staged is not None and staged.error is None and staged.seed == seed and staged.pos == pos
                and np.array_equal(staged.key, key)):
            self.stats["prefetch_hits"] += 1
        else:
            if staged is not None:
                if staged.ready is not None:
                    staged.ready.synchronize()
                self._pending.appendleft(staged)
            self._discard_pending()
            if staged is not None and staged.error is not None:
                raise staged.error
            staged = _Staged(self._take_slot(), key.copy(), pos, seed)
            try:
                self._stage(staged)
                self._device_build(staged, cur)
            finally:
                staged.sampled.set()
                staged.enqueued.set()
            # the builds share rows / perm / workspaces: later side-stream builds after this one
            self.side_stream.wait_stream(cur)
        # randint draws leave the cached Gaussian of the legacy state alone
        np.random.set_state(("MT19937", staged.end_key, staged.end_pos, gauss[0], gauss[1]))
        cur.wait_event(staged.ready)
        # everything that read the previous epoch's slot (its steps; a build on this
        # stream) is enqueued before this point
        if self._cur_slot is not None:
            free = torch.cuda.Event()
            free.record(cur)
            self._free[self._cur_slot] = free
        self._cur_slot = staged.slot
        self.events = (staged.t0, staged.built, staged.ready)
        self.stats.setdefault("host_ms", []).append(dict(staged.host_ms))
        # the dataset's host view of this epoch's negatives (fetched only if asked for)
        self.ds._set_device_negatives(self._neg_dev[staged.slot][: self.S] if self.S else None)
        self.stats["epochs"] += 1
        if self.depth:
            seeds = self._peek_seeds(peek_eval_draw, self.depth)
            prev = self._pending[-1] if self._pending else staged
            for sd in seeds[len(self._pending):]:
                prev = self._launch(sd, prev)
        t_out = time.perf_counter()
        self.stats.setdefault("boundary_ms", []).append(((t_joined - t_enter) * 1e3, (t_out - t_joined) * 1e3))
        return self._out[staged.slot]

    @property
    def buffers(self):
        """The output buffers next_epoch() rotates through."""
        return list(self._out)

    def device_ms(self):
        """(rows + permutation, grouping) device milliseconds of the last epoch's
        build (on the side stream, under earlier epochs' steps, when the prefetch
        hit)."""
        if self.events is None:
            return None
        t0, built, ready = self.events
        ready.synchronize()
        return t0.elapsed_time(built), built.elapsed_time(ready)

    def close(self):
        self._discard_pending()
