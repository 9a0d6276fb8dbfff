"""``Trainer.fit()/evaluate()`` -- the training loop of the reference scripts as an API.

The reference has no Trainer: the loop is written inline in
scripts/train_neumf.py:98-144 (and scripts/pretrain.py:61-106).  This class
runs exactly that loop -- same RNG consumption, same batches, same loss,
optimizer, evaluation, printed lines and return dict (train_neumf.py:159-167)
-- with every step on the device engine (ncf_amd.engine.TrainEngine):

  per epoch (train_neumf.py:98-131)
    dataset.ng_sample()                       NumPy global MT19937 stream (C++ sampler)
    DataLoader(shuffle=True) order            torch global generator: base_seed, sampler
                                              seed, randperm (data.epoch_permutation)
    for each batch: zero_grad/fwd/BCE/bwd/step -> one captured hipGraph replay
    metrics(model, test_loader, top_k)        one forward + one HR/NDCG launch; one
                                              base_seed draw, like the test DataLoader
    "Epoch %03d: Loss=%.4f, HR=%.3f, NDCG=%.3f, Time=%.1fs"

Data parallel (world_size > 1): every rank runs the same host stream (same
seeds), processes its contiguous shard of each global batch, and the engine
all-reduces gradients over RCCL; evaluation and checkpoints are rank 0's.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from . import ops
from .data import NCFData, consume_test_pass, epoch_permutation
from .engine import TrainEngine
from .metrics import evaluate_rows_device


class Trainer:
    def __init__(self, model, train_dataset: NCFData, test_loader=None, *, batch_size=256, lr=1e-3,
                 optimizer="adam", top_k=10, device=None, world_size=1, rank=0, process_group=None,
                 use_graph=True, save_path=None, verbose=True, test_batch=None, distill=None):
        """distill: a distillation module (ncf_amd.distill) whose student is `model`:
        every step then trains the student on that module's loss (device plan)."""
        self.model = model
        self.ds = train_dataset
        self.test_loader = test_loader
        self.batch_size = int(batch_size)
        self.top_k = int(top_k)
        self.device = torch.device(device) if device is not None else model.embed_user_GMF.weight.device
        if self.device.type != "cuda":
            raise RuntimeError("Trainer runs the HIP engine: put the model on a HIP device")
        if model.embed_user_GMF.weight.device != self.device:
            model.to(self.device)
        self.world_size, self.rank = int(world_size), int(rank)
        if distill is not None and distill.student_model is not model:
            raise ValueError("distill.student_model must be the model being trained")
        plan = distill.device_plan() if distill is not None else None
        self.engine = TrainEngine(model, lr=lr, optimizer=optimizer, world_size=world_size, rank=rank,
                                  process_group=process_group, distill=plan)
        self.use_graph = use_graph
        self.save_path = save_path
        self.verbose = verbose and self.rank == 0
        self._test = None
        self.test_batch = test_batch
        self.history = []
        self._pipe = None

    # ------------------------------------------------------------------ data
    def _epoch_stream(self):
        """ng_sample + DataLoader order for one epoch -> device stream in batch order.
        Default: the epoch pipeline (ncf_amd.pipeline: the next epoch's negatives and
        permutation words drawn on host threads while this one trains, the
        permutation and rows built on the device); NCF_HOST_EPOCH=1: sampler, torch
        randperm, packing and upload in line (the round-1 path, for comparison)."""
        if os.environ.get("NCF_HOST_EPOCH", "0") != "1":
            if self._pipe is None:
                from .pipeline import EpochPipeline
                self._pipe = EpochPipeline(self.ds, self.device, self.batch_size, int(self.model.item_num),
                                           user_num=int(self.model.user_num), canonical=self.world_size > 1)
                self.engine.stream_buffers = self._pipe.buffers  # step graphs captured for both
                self._pipe.on_built = self.engine.owner_prebuild  # dp_mode "owner": lists built with each epoch
            # fit() evaluates after every epoch (one torch draw): the next epoch's
            # sampler seed is peeked past it
            return self._pipe.next_epoch(peek_eval_draw=True)
        self.ds.ng_sample()
        u, i, y = self.ds.arrays()
        n = len(u)
        ops.check_ids(u, i, int(self.model.user_num), int(self.model.item_num))
        perm = epoch_permutation(n).to(self.device)
        if getattr(self, "_rows", None) is None or self._rows.numel() != n:
            self._rows = torch.empty(n, dtype=torch.int64, device=self.device)
            self._prep = ops.EpochPrep(self.device, canonical=self.world_size > 1)
        # packed on the host (one int64 per row), one upload, shuffle+group on the device
        self._rows.copy_(torch.from_numpy(ops.pack_rows_host(u, i, y)))
        return self._prep(self._rows, perm, self.batch_size, int(self.model.item_num))

    def _test_arrays(self):
        if self._test is None:
            us, its, sizes = [], [], []
            if self.test_loader is None:
                raise RuntimeError("no test_loader given")
            ds = getattr(self.test_loader, "dataset", None)
            bs = getattr(self.test_loader, "batch_size", None)
            if isinstance(ds, NCFData) and bs and not ds.is_training:
                u, i, _ = ds.arrays()
                self._test = (u.astype(np.int32), i.astype(np.int32), int(bs))
            else:
                for user, item, _ in self.test_loader:
                    us.append(np.asarray(user).reshape(-1))
                    its.append(np.asarray(item).reshape(-1))
                    sizes.append(len(us[-1]))
                self._test = (np.concatenate(us).astype(np.int32), np.concatenate(its).astype(np.int32),
                              int(sizes[0]))
        return self._test

    def _test_device(self):
        """The test candidate stream packed on the device, ids checked once
        (nn.Embedding's IndexError, models.py:108-112)."""
        if getattr(self, "_test_dev", None) is None:
            u, i, bs = self._test_arrays()
            ops.check_ids(u, i, int(self.model.user_num), int(self.model.item_num))
            ud = torch.as_tensor(u, dtype=torch.int32).to(self.device)
            idv = torch.as_tensor(i, dtype=torch.int32).to(self.device)
            self._test_dev = (ops.pack_rows(ud, idv), idv, bs)
        return self._test_dev

    def _evaluate_device(self, top_k=None):
        k = self.top_k if top_k is None else int(top_k)
        rows, items, bs = self._test_device()
        consume_test_pass()  # the test DataLoader iteration's base_seed draw
        return evaluate_rows_device(self.model, rows, items, bs, k)

    # ------------------------------------------------------------------ API
    def evaluate(self, top_k=None):
        """metrics(model, test_loader, top_k) (metrics.py:4-25): per-batch HR/NDCG lists."""
        hr, nd = self._evaluate_device(top_k)
        return hr.cpu().tolist(), nd.double().cpu().tolist()

    def train_epoch(self):
        rows = self._epoch_stream()
        self.engine.set_epoch_stream(rows, self.batch_size, checked=True)  # ids checked on the host
        self.engine.run(self.engine.num_batches, use_graph=self.use_graph)
        return float(np.mean(self.engine.epoch_losses()))

    def _report(self, epoch, avg_loss, hr, ndcg, el, save_fn, snap, device_time=None):
        self.history.append({"epoch": epoch + 1, "loss": avg_loss, "hr": hr, "ndcg": ndcg, "time": el,
                             "device_time": device_time})
        if self.verbose:
            print(f"Epoch {epoch + 1:03d}: Loss={avg_loss:.4f}, HR={hr:.3f}, NDCG={ndcg:.3f}, Time={el:.1f}s")
        if hr > self._best[0]:
            self._best = [hr, ndcg, epoch + 1]
            if save_fn is not None and self.rank == 0:
                if snap is None:
                    save_fn(self.model)
                else:
                    with ops.params_view(self.model, snap):  # the parameters as that epoch ended
                        save_fn(self.model)

    def _report_pending(self, pending, save_fn):
        epoch, ev0, ev1, out, snap, t0 = pending
        ev1.synchronize()
        # like the reference: from the epoch's start to its metrics -- the moment the
        # device finished the epoch's metrics pass (ev1), mapped onto the host clock
        # through the anchor event of fit(), not the later moment this readback runs
        # (after epoch e + 1 was enqueued)
        anchor, host_anchor = self._clock
        wall = host_anchor + anchor.elapsed_time(ev1) / 1e3 - t0
        avg_loss = float(np.mean(out["loss"].numpy().astype(np.float64)))
        hr = float(np.mean(out["hr"].numpy().astype(np.float64)))
        ndcg = float(np.mean(out["nd"].numpy().astype(np.float64)))
        self._report(epoch, avg_loss, hr, ndcg, wall, save_fn, snap, ev0.elapsed_time(ev1) / 1e3)

    def fit(self, epochs, model_type=None, pretraining=False, save_fn=None):
        """The reference loop (train_neumf.py:98-144).  Single rank: epoch e's loss,
        HR and NDCG are copied to pinned host buffers as the epoch ends (and, with a
        save_fn, the parameters to a device snapshot), epoch e + 1 is enqueued, and
        only then is epoch e read back, printed and checkpointed -- the same values,
        the same generator draws in the same order, no idle device between epochs.
        Time= (history "time") is wall-clock from the epoch's start to the end of its
        metrics pass, as train_neumf.py:100,130 measures it (the device's completion
        of the pass, mapped onto the host clock by an anchor event, so epoch e's time
        does not include epoch e + 1's host work); history "device_time" is the
        epoch's device time (steps + evaluation)."""
        self._best = [0, 0, 0]  # hr, ndcg, epoch
        if self.world_size > 1:  # the loss readback is a collective there: in line
            for epoch in range(int(epochs)):
                self.model.train()
                t0 = time.time()
                avg_loss = self.train_epoch()
                self.model.eval()
                if self.rank == 0:
                    HR, NDCG = self.evaluate()
                    hr, ndcg = float(np.mean(HR)), float(np.mean(NDCG))
                else:
                    consume_test_pass()
                    hr = ndcg = 0.0
                self._report(epoch, avg_loss, hr, ndcg, time.time() - t0, save_fn, None)
        else:
            pending = None
            anchor = torch.cuda.Event(enable_timing=True)
            anchor.record()
            anchor.synchronize()
            self._clock = (anchor, time.time())
            for epoch in range(int(epochs)):
                self.model.train()
                t0 = time.time()
                ev0 = torch.cuda.Event(enable_timing=True)
                ev0.record()
                rows = self._epoch_stream()
                self.engine.set_epoch_stream(rows, self.batch_size, checked=True)
                self.engine.run(self.engine.num_batches, use_graph=self.use_graph)
                self.model.eval()
                nb = self.engine.num_batches
                out = {"loss": torch.empty(nb, dtype=torch.float32).pin_memory()}
                out["loss"].copy_(self.engine.loss_hist[:nb], non_blocking=True)
                hr_d, nd_d = self._evaluate_device()
                out["hr"] = torch.empty(hr_d.numel(), dtype=torch.int32).pin_memory()
                out["nd"] = torch.empty(nd_d.numel(), dtype=torch.float32).pin_memory()
                out["hr"].copy_(hr_d, non_blocking=True)
                out["nd"].copy_(nd_d, non_blocking=True)
                snap = self.engine.flat.clone() if save_fn is not None else None
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record()
                if pending is not None:
                    self._report_pending(pending, save_fn)
                pending = (epoch, ev0, ev1, out, snap, t0)
            if pending is not None:
                self._report_pending(pending, save_fn)
        best_hr, best_ndcg, best_epoch = self._best
        n_params = sum(p.numel() for p in self.model.parameters() if p.requires_grad)
        return {
            "best_hr": best_hr,
            "best_ndcg": best_ndcg,
            "best_epoch": best_epoch,
            "parameters": n_params,
            "num_layers": self.model.num_layers,
            "pretraining": pretraining,
            "model_type": model_type or self.model.model_type,
        }
