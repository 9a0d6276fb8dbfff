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
rows and permutation are then built on a side stream, under epoch e's steps, so
the epoch boundary is left with the grouping by item only.
When epoch e+1 starts, the real draws are made and compared with what was used;
a mismatch (someone else consumed either generator in between) discards the
prefetch, and the epoch is built synchronously.
"""
from __future__ import annotations

import threading
import time

import numpy as np
import torch

from . import _lib as L
from . import ops
from .data import epoch_permutation_seed


def _mt_state():
    st = np.random.get_state(legacy=True)
    if st[0] != "MT19937":
        raise RuntimeError("numpy global generator is not MT19937")
    return np.ascontiguousarray(st[1], dtype=np.uint32).copy(), int(st[2])


def torch_words(seed, n, out):
    """The first n 32-bit words of torch.Generator().manual_seed(seed) (MT19937 on
    the low 32 bits of the seed) into out (uint32)."""
    key = np.empty(624, dtype=np.uint32)
    pos = np.empty(1, dtype=np.int32)
    lib = L.sampler_lib()
    lib.ncf_mt_seed(int(seed) & 0xFFFFFFFF, key.ctypes.data, pos.ctypes.data)
    if n > 0:
        lib.ncf_mt_words(key.ctypes.data, pos.ctypes.data, int(n), out.ctypes.data)


class _Staged:
    """One epoch's host products (negatives, permutation words) and their upload."""

    def __init__(self, key, pos, seed):
        self.key, self.pos, self.seed = key, pos, seed
        self.end_key = self.end_pos = None  # NumPy state after the epoch's ng_sample
        self.event = None   # uploads done
        self.ready = None   # rows + permutation built
        self.t0 = None
        self.error = None
        self.host_ms = {}


class EpochPipeline:
    def __init__(self, dataset, device, batch_size, item_num, user_num=None, prefetch=True):
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
        self.rows = torch.empty(self.n, dtype=torch.int64, device=dev)
        self.perm = torch.empty(self.n, dtype=torch.int64, device=dev)
        self.fy_ws = torch.empty(int(L.hip().ncf_randperm_workspace(self.n)), dtype=torch.uint8, device=dev)
        self.prep = ops.EpochPrep(dev)
        self.copy_stream = torch.cuda.Stream(device=dev)
        # two slots: one being consumed by the device, one being filled by the host
        self._neg_host = [torch.empty(max(1, self.S), dtype=torch.int32).pin_memory() for _ in range(2)]
        self._words_host = [torch.empty(max(1, self.n - 1), dtype=torch.int32).pin_memory() for _ in range(2)]
        self._neg_dev = [torch.empty(max(1, self.S), dtype=torch.int32, device=dev) for _ in range(2)]
        self._words_dev = [torch.empty(max(1, self.n - 1), dtype=torch.int32, device=dev) for _ in range(2)]
        self._slot = 0
        self.prefetch = prefetch
        self._pending = None
        self._threads = []
        self.side_stream = torch.cuda.Stream(device=dev)
        self.stats = {"epochs": 0, "prefetch_hits": 0}
        self.events = None  # (start, rows+perm ready, grouped) of the last epoch

    # ---------------------------------------------------------------- host part
    def _stage(self, slot, key, pos, seed, before_upload=None):
        """Negatives from NumPy state (key, pos) and the permutation words of
        `seed`, staged in pinned memory and uploaded (runs on worker threads)."""
        s = _Staged(key.copy(), int(pos), seed)
        t_all = time.perf_counter()
        neg = self._neg_host[slot].numpy()
        words = self._words_host[slot].numpy().view(np.uint32)

        def draw_negatives():
            t0 = time.perf_counter()
            if self.S == 0:
                s.end_key, s.end_pos = s.key.copy(), s.pos
                return
            k2, p2 = s.key.copy(), np.array([s.pos], dtype=np.int32)
            self.ds._get_sampler().sample(self.num_item, self.ng, k2, p2, out=neg[: self.S])
            s.end_key, s.end_pos = k2, int(p2[0])
            s.host_ms["sample"] = (time.perf_counter() - t0) * 1e3

        def draw_words():
            t0 = time.perf_counter()
            torch_words(seed, self.n - 1, words[: self.n - 1])
            s.host_ms["words"] = (time.perf_counter() - t0) * 1e3

        try:
            t = threading.Thread(target=draw_words)
            t.start()
            draw_negatives()
            t.join()
            if before_upload is not None:
                before_upload()
            with torch.cuda.stream(self.copy_stream):
                if self.S:
                    self._neg_dev[slot][: self.S].copy_(self._neg_host[slot][: self.S], non_blocking=True)
                if self.n > 1:
                    self._words_dev[slot][: self.n - 1].copy_(self._words_host[slot][: self.n - 1],
                                                              non_blocking=True)
                s.event = torch.cuda.Event()
                s.event.record(self.copy_stream)
        except Exception as e:  # surfaced when the epoch is consumed
            s.error = e
        s.host_ms["stage"] = (time.perf_counter() - t_all) * 1e3
        return s

    # ---------------------------------------------------------------- API
    def _peek_next_seed(self, eval_draw):
        """The next epoch's RandomSampler seed, past this epoch's metrics() draw
        if `eval_draw` (train_neumf.py:120), consuming nothing."""
        state = torch.get_rng_state()
        try:
            if eval_draw:
                torch.empty((), dtype=torch.int64).random_()   # the test loader's base_seed
            return epoch_permutation_seed()                     # base_seed, sampler seed
        finally:
            torch.set_rng_state(state)

    def _join(self):
        for t in self._threads:
            t.join()
        self._threads = []

    def _device_build(self, staged, slot, stream):
        """On `stream` (after the staged uploads): the epoch's packed rows and its
        permutation.  Records staged.ready."""
        lib = L.hip()
        st = stream.cuda_stream
        stream.wait_event(staged.event)
        staged.t0 = torch.cuda.Event(enable_timing=True)
        staged.t0.record(stream)
        L.check(lib.ncf_build_rows(self.pu.data_ptr(), self.pi.data_ptr(), self.P,
                                   self._neg_dev[slot].data_ptr() if self.S else None, self.ng,
                                   self.rows.data_ptr(), st), "ncf_build_rows")
        L.check(lib.ncf_randperm(self._words_dev[slot].data_ptr(), self.n, self.perm.data_ptr(),
                                 self.fy_ws.data_ptr(), self.fy_ws.numel(), st), "ncf_randperm")
        staged.ready = torch.cuda.Event(enable_timing=True)
        staged.ready.record(stream)

    def next_epoch(self, peek_eval_draw=True):
        """The epoch's packed stream in batch order (device), consuming the NumPy
        global stream (ng_sample) and the torch global generator (DataLoader)
        exactly like the reference's epoch.  peek_eval_draw: a metrics() pass
        (one torch draw) follows this epoch before the next next_epoch().

        With a prefetch hit the rows and the permutation were built on a side
        stream while the previous epoch trained; what is left here is the
        grouping by item (ncf_prepare_epoch) on the current stream."""
        self._join()
        key, pos = _mt_state()
        seed = epoch_permutation_seed()  # the DataLoader's two draws
        staged, self._pending = self._pending, None
        if staged is not None and staged.error is not None:
            raise staged.error
        slot = self._slot
        dev = self.device
        cur = torch.cuda.current_stream(dev)
        if (staged is not None and staged.seed == seed and staged.pos == pos
                and np.array_equal(staged.key, key)):
            self.stats["prefetch_hits"] += 1
        else:
            if staged is not None and staged.ready is not None:
                staged.ready.synchronize()  # a discarded prefetch still writes rows / perm: let it finish
            staged = self._stage(slot, key, pos, seed)
            if staged.error is not None:
                raise staged.error
            self._device_build(staged, slot, cur)
        np.random.set_state(("MT19937", staged.end_key, staged.end_pos, 0, 0.0))
        cur.wait_event(staged.ready)
        e1 = torch.cuda.Event(enable_timing=True)
        out = self.prep(self.rows, self.perm, self.batch_size, self.item_num)
        e1.record(cur)
        self.events = (staged.t0, staged.ready, e1)
        self.stats.setdefault("host_ms", []).append(dict(staged.host_ms))
        # the dataset's host view of this epoch's negatives (fetched only if asked for)
        self.ds._set_device_negatives(self._neg_dev[slot][: self.S] if self.S else None)
        self.stats["epochs"] += 1
        if self.prefetch:
            nkey, npos = staged.end_key, staged.end_pos
            nseed = self._peek_next_seed(peek_eval_draw)
            nslot = slot ^ 1

            def work():
                # host draws first; the uploads and the device build wait until this
                # epoch's grouping has read rows / perm (the other slot's buffers were
                # read by the epoch before)
                s = self._stage(nslot, nkey, npos, nseed, before_upload=e1.synchronize)
                if s.error is None:
                    try:
                        self._device_build(s, nslot, self.side_stream)
                    except Exception as e:  # surfaced when the epoch is consumed
                        s.error = e
                self._pending = s
            t = threading.Thread(target=work, daemon=True)
            t.start()
            self._threads.append(t)
            self._slot = nslot
        return out

    def device_ms(self):
        """(rows + permutation, grouping) device milliseconds of the last epoch: the
        first runs on the side stream under the previous epoch's steps when the
        prefetch hit, the second on the current stream at the boundary."""
        if self.events is None:
            return None
        t0, ready, e1 = self.events
        e1.synchronize()
        return t0.elapsed_time(ready), ready.elapsed_time(e1)

    def close(self):
        self._join()
        if self._pending is not None and self._pending.ready is not None:
            self._pending.ready.synchronize()
        self._pending = None
