"""Device-resident NeuMF training engine (the fast path behind ``Trainer.fit``).

One optimizer step over one global batch is four launches on the current
stream, with no host synchronisation and no per-step allocation, so the whole
step is captured once into a hipGraph and replayed (world > 1: two graphs
with the all-reduce issued between them, see ``_capture_collective``):

  1. ``ncf_train_step``  fused gather / GMF / MFMA tower fwd / BCE / MFMA tower
                         bwd / embedding scatter-add   (models.py:97-118,
                         train_neumf.py:111-114); on the factored path it also
                         launches the expansion (per-user/item sums -> dUm, dIm, dW0)
  2. ``ncf_reduce_slab`` per-workgroup tower grads -> flat grad buffer
  3. world > 1, dp_mode "zero1": RCCL reduce-scatter of the flat grad buffer;
     dp_mode "allreduce": RCCL all-reduce of the flat grad buffer
  4. ``ncf_adam_step``   dense Adam over the active parameters (zero1: of this
                         rank's shard only) + grad zeroing + loss bookkeeping
                         (train_neumf.py:90,115)
  5. zero1: RCCL all-gather of the updated parameter shards (in place)

dp_mode "owner" (ncf_owner_* in include/ncf_hip.h): embedding row id is owned by
rank id % W; per step train + ncf_owner_pack (this rank's gradient rows bucketed by
owner, the tower gradient in every bucket) -> all_to_all -> ncf_owner_adam (the
owner sums the W contributions in rank order and runs dense Adam over all its rows;
tower Adam replicated; the rows each rank's next batch reads packed) -> all_to_all
-> ncf_owner_unpack.  No host synchronisation: the bucket lists of every step are
built once per epoch from the stream every rank holds.

Data parallelism: every rank holds the same epoch stream (same seeds, same
sampler, same permutation); rank r processes rows [r*ceil(gb/W), ...) of each
global batch, with dlogit scaled by 1/global_batch, so the summed gradient is
the single-device mean gradient of ``BCEWithLogitsLoss``.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib as L
from . import distributed as D
from . import ops


def _active_ranges(model, lay, extra=None):
    """Merged [begin, end) float ranges of the parameters that get gradients
    (``extra``: per-parameter mask OR-ed in, e.g. the embedding tables that the
    feature-distillation terms reach)."""
    segs = []
    sizes = [p.numel() for p in model.ordered_params()]
    offs = [lay.ug, lay.ig, lay.um, lay.im]
    for k in range(model.num_layers):
        offs += [lay.w[k], lay.b[k]]
    offs += [lay.wp, lay.bp]
    mask = ops.active_mask(model)
    if extra is not None:
        mask = [a or b for a, b in zip(mask, extra)]
    for off, n, act in zip(offs, sizes, mask):
        if act:
            segs.append([int(off), int(off + (n + 63) // 64 * 64)])
    merged = []
    for b, e in sorted(segs):
        if merged and merged[-1][1] == b:
            merged[-1][1] = e
        else:
            merged.append([b, e])
    return merged


def touched_segments(buf, nb):
    """Host view of an ncf_batch_touched buffer (int32 numpy copy): [b][k] id arrays,
    k = 2 * list + side (lists A, B, C; side 0 users, 1 items) -- include/ncf_hip.h."""
    import numpy as np
    seg = np.ascontiguousarray(buf[:2 * (6 * nb + 1)]).view(np.int64)
    ids = buf[2 * (6 * nb + 1):]
    return [[ids[seg[6 * b + k]:seg[6 * b + k + 1]] for k in range(6)] for b in range(nb)]


class TrainEngine:
    # world > 1 default exchange: one all-reduce + replicated Adam up to this many flat
    # floats, zero1 (reduce-scatter, shard Adam, all-gather: the same wire bytes) above.
    # Sharding saves 7/8 of a 32 B/param Adam pass at W = 8 (~5 ps/param at ~6 TB/s)
    # but costs two more launches and a collective (~16 us per step measured with a
    # one-rank RCCL group, scripts/dp_overhead.py): break-even near 3-4M floats
    # (C3 0.79M: allreduce; C4 13.2M: zero1).
    ALLREDUCE_MAX_FLOATS = 4 << 20

    # dp_mode "auto" (the world > 1 default where deferred Adam applies) resolves at the
    # first epoch stream: "touched" when the packed buffer of a global batch's rows is
    # at most this fraction of the flat gradient, else "allreduce".  Measured per rank
    # at N = 8 on one GPU (scripts/dp_modes.py): at C3 the packed buffer equals the flat
    # gradient (a 65,536-row batch touches every row) and the pack + deferred Adam cost
    # 55.1 us against 43.3 for all-reduce + dense Adam; at C4 it is 0.56 of it and saves
    # 23 MB of wire per step against ~33 us of local work.
    TOUCHED_MAX_FRACTION = 0.8

    @classmethod
    def default_dp_mode(cls, total_floats, touched_ok=False):
        """world > 1: "auto" (touched or allreduce by the global batch, see
        TOUCHED_MAX_FRACTION) where the model supports deferred Adam; else one
        all-reduce up to ALLREDUCE_MAX_FLOATS, zero1 above."""
        if touched_ok:
            return "auto"
        return "allreduce" if total_floats <= cls.ALLREDUCE_MAX_FLOATS else "zero1"

    # dp_mode "auto" picks the owner-sharded exchange from this many ranks up even where
    # a global batch touches every row (C3): two all-to-alls of the touched rows over the
    # point-to-point xGMI links against a ring all-reduce of the whole flat gradient
    # (the projection of DESIGN.md section 6, from per-rank costs measured at emulated
    # N = 2 / 4 / 8); at 2 ranks the all-reduce's one collective wins there
    OWNER_MIN_WORLD = 4

    @classmethod
    def auto_dp_mode(cls, lay, ranges, nranges, batch_size, world=2, owner_ok=False):
        """("owner" | "touched" | "allreduce" | "zero1", packed floats) for dp_mode "auto"
        at this global batch and world: owner (where it applies) when the batch touches
        a small part of the tables (packed buffer <= TOUCHED_MAX_FRACTION of the flat
        gradient, C4) or from OWNER_MIN_WORLD ranks up; else touched where the packed
        buffer is small enough; else the size rule of default_dp_mode (all-reduce up to
        ALLREDUCE_MAX_FLOATS, zero1 above: the optimizer state stays sharded)."""
        pf = int(L.hip().ncf_touched_packed_floats(ctypes.byref(lay), ranges, nranges, int(batch_size)))
        sparse = 0 < pf <= cls.TOUCHED_MAX_FRACTION * int(lay.total)
        if owner_ok and (sparse or int(world) >= cls.OWNER_MIN_WORLD):
            return "owner", pf
        if sparse:
            return "touched", pf
        return cls.default_dp_mode(int(lay.total), touched_ok=False), pf

    def _owner_ok(self):
        """dp_mode "owner" applies: Adam, no distillation, at most 16 ranks, rows of at
        most 1,024 floats (ncf_owner_plan_init) -- touched_ok's other limits."""
        if self.optimizer != "adam" or self.distill is not None or self.world_size > 16:
            return False
        P = L.NcfOwnerPlan()
        return L.hip().ncf_owner_plan_init(ctypes.byref(self.lay), self._ranges, self._nranges, 1, 1,
                                           self.world_size, self.rank, 0, 0, ctypes.byref(P)) == L.NCF_OK

    def _resolve_auto(self, batch_size):
        self.dp_mode, pf = self.auto_dp_mode(self.lay, self._ranges, self._nranges, batch_size, self.world_size,
                                             self._owner_ok())
        if self.dp_mode == "touched":
            self._packed = torch.zeros(pf, dtype=torch.float32, device=self.device)
        elif self.dp_mode == "zero1":
            # the flat buffers were padded to world x shard floats at construction
            # (__init__): keep this rank's slice of the optimizer state
            self._init_shards()
            if self.optimizer == "adam":
                r, S = self.rank, self.shard
                self.exp_avg = self.exp_avg[r * S:(r + 1) * S].clone()
                self.exp_avg_sq = self.exp_avg_sq[r * S:(r + 1) * S].clone()
            self._set_fact_shard()
            self._drop_graphs()

    def __init__(self, model, lr=1e-3, optimizer="adam", betas=(0.9, 0.999), eps=1e-8,
                 world_size=1, rank=0, process_group=None, max_batches=1 << 16, dp_mode=None, distill=None):
        """distill: an ``ncf_amd.distill.DeviceDistillPlan`` -- the student step then
        runs ncf_train_step_kd (teacher logits of the epoch stream computed once per
        epoch by ncf_forward) plus ncf_kd_feature_step for the feature terms."""
        self.model = model
        self.distill = distill
        if process_group is None and int(world_size) > 1:
            # no group given: the collectives run over the default group, so the
            # owner all-gather and the stream agreement check must use it too
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                process_group = dist.group.WORLD
        self.world_size, self.rank, self.group = int(world_size), int(rank), process_group
        lay = L.layout(model.user_num, model.item_num, model.factor_num, model.num_layers, model.model_type)
        touched_ok = (optimizer == "adam" and model.factor_num % 4 == 0 and model.user_num <= (1 << 19)
                      and model.item_num <= (1 << 19))
        if dp_mode is None:
            dp_mode = os.environ.get("NCF_DP_MODE", self.default_dp_mode(int(lay.total), touched_ok)) \
                if self.world_size > 1 else "single"
        # an explicit exchange mode stands at world 1 (a one-rank group still runs the
        # real collectives: how the captured-collective graph is tested on one GPU)
        if dp_mode not in ("single", "zero1", "allreduce", "touched", "auto", "owner"):
            raise ValueError(f"dp_mode {dp_mode!r}")
        if dp_mode in ("touched", "auto", "owner") and not touched_ok:
            raise ValueError(f"dp_mode {dp_mode!r} needs Adam, factor_num % 4 == 0 and tables of <= 2^19 rows")
        if dp_mode == "owner" and (distill is not None or self.world_size > 16):
            raise ValueError("dp_mode 'owner': no distillation, at most 16 ranks")
        self.dp_mode = dp_mode
        # flat buffers padded to world x shard floats where the exchange shards them
        # (rank r owns [r*S, (r+1)*S)); "auto" pads too when its fallback would be zero1
        shards = dp_mode == "zero1" or (
            dp_mode == "auto" and self.default_dp_mode(int(lay.total)) == "zero1")
        self.shard = None
        n = int(lay.total)
        if shards:
            n = D.shard_floats(int(lay.total), self.world_size) * self.world_size
        self.flat, lay0 = ops.ensure_flat(model, n)
        # the engine's own copy: ncf_layout_tune shapes it for the batch size
        self.lay = type(lay0).from_buffer_copy(lay0)
        # nn.Dropout(p) before every tower Linear (models.py:23): training steps with
        # p > 0 run the layered path, keep masks hashed from (seed, step, layer, row,
        # column) -- include/ncf_hip.h ncf_dropout_hash
        ops.set_dropout(self.lay, model)
        dev = self.flat.device
        self.device = dev
        n = self.flat.numel()
        self.grads = torch.zeros(n, dtype=torch.float32, device=dev)
        self.optimizer = optimizer
        n_opt = D.shard_floats(int(lay.total), self.world_size) if dp_mode == "zero1" else n
        if optimizer == "adam":
            self.exp_avg = torch.zeros(n_opt, dtype=torch.float32, device=dev)
            self.exp_avg_sq = torch.zeros(n_opt, dtype=torch.float32, device=dev)
        elif optimizer != "sgd":
            raise ValueError(optimizer)
        self.lr, self.betas, self.eps = float(lr), (float(betas[0]), float(betas[1])), float(eps)
        self.ws = None  # ncf_train_step workspace, sized by set_epoch_stream
        self._fact_shard = False  # zero1: the factored expansion sharded into the optimizer (_set_fact_shard)
        self.ctl = ops.new_ctl(0, dev)
        rng = _active_ranges(model, self.lay, None if distill is None else distill.active_extra)
        self._ranges = (ctypes.c_int64 * (2 * len(rng)))(*[x for r in rng for x in r])
        self._nranges = len(rng)
        self._loss_slot = int(self.lay.loss_slot)
        self._opt_ptrs = (self.flat.data_ptr(), self.grads.data_ptr())
        if dp_mode == "zero1":
            self._init_shards()
        self.loss_hist = torch.zeros(max_batches, dtype=torch.float32, device=dev)
        self.rows = None
        self.n_total = 0
        self.batch_size = None
        self._graph = None
        self._graph_k = None
        # captured step graphs per epoch-stream buffer (the epoch pipeline alternates
        # two): key (batch_size, n_total, rows pointer) -> (graph(s), k-step graph)
        self._graphs = {}
        # other epoch-stream buffers this engine will be handed (same layout as
        # the current one): captured together with it, so a buffer switch at an
        # epoch boundary replays graphs already built
        self.stream_buffers = []
        # ncf_user_order output per epoch-stream buffer (key: pointer, rows)
        self._orders = {}
        self._uses_order = False
        # deferred Adam (ncf_lazy_adam_step): per-row last step, step scalars ring,
        # ncf_batch_touched lists per epoch-stream buffer (key: pointer, rows, batch)
        self.lazy = False
        self._last = None
        self._ring = None
        self._touched_lists = {}
        # dp_mode "owner": plan (ncf_owner_plan), list slots high-water (max_u, max_i),
        # per-stream-buffer bucket lists, the four exchange buffers
        self._ow_plan = None
        self._ow_M = (0, 0)
        self._ow_lists = {}
        self._ow_bufs = None
        self._ow_max = None
        self._ow_pre = {}  # owner_prebuild results per stream buffer
        self._ow_old = []  # replaced list buffers (a side-stream prebuild may still write them)
        if dp_mode == "touched":  # packed gradients of the touched rows + tower, all-reduced
            self._packed = torch.zeros(int(L.hip().ncf_touched_packed_floats(ctypes.byref(self.lay), self._ranges,
                                                                             self._nranges, 1)),
                                       dtype=torch.float32, device=dev)  # resized per batch size

    def _init_shards(self):
        """zero1: this rank's shard of the flat buffers, its active ranges,
        the loss slot's owner and the optimizer's pointers."""
        S = self.shard = D.shard_floats(int(self.lay.total), self.world_size)
        r = self.rank
        assert self.flat.numel() >= S * self.world_size
        rng = [[self._ranges[2 * k], self._ranges[2 * k + 1]] for k in range(self._nranges)]
        self.gshard = torch.zeros(S, dtype=torch.float32, device=self.device)
        # an empty [0, 0) range when no active parameter falls in the shard: the
        # launch still records the loss if this rank owns the loss slot
        srng = D.shard_ranges(rng, self.world_size, r, S) or [[0, 0]]
        self._sranges = (ctypes.c_int64 * (2 * len(srng)))(*[x for q in srng for x in q])
        self._nsranges = len(srng)
        slot = int(self.lay.loss_slot)
        self.loss_owner = slot // S
        self._loss_slot = slot - r * S
        self._opt_ptrs = (self.flat.data_ptr() + 4 * r * S, self.gshard.data_ptr())
        self._ag_scratch = None

    # ------------------------------------------------------------------ data
    def set_epoch_stream(self, rows, batch_size, checked=False):
        """Packed int64 rows (ops.pack_rows / ncf_prepare_epoch output) already in
        training order: batch b is rows[b*batch_size, ...).  Ids are range-checked
        once here (IndexError like nn.Embedding) unless the caller already did
        (`checked`, e.g. Trainer on the host arrays)."""
        if rows.dtype != torch.int64 or not rows.is_contiguous() or rows.device != self.device:
            raise ValueError("epoch stream: contiguous int64 packed rows on the engine's device")
        if not checked:
            ops.check_rows(rows, self.model.user_num, self.model.item_num)
        n = rows.numel()
        self.rows = rows
        self.n_total = n
        if self.batch_size != batch_size or self.ws is None:
            self._drop_graphs()
            per = (int(batch_size) + self.world_size - 1) // self.world_size
            # launch shape for this batch size: workgroups = its 128-row tiles (64-row
            # tiles of 4-wave workgroups for small per-rank batches; up to one per CU),
            # per-row layer 0 for batches small against the tables.  NCF_WG_WAVES=4|8
            # forces the workgroup geometry (A/B measurements).
            wg = os.environ.get("NCF_WG_WAVES")
            if wg:
                L.check(L.hip().ncf_debug_set_geometry(int(wg)), "ncf_debug_set_geometry")
            # user store-and-sum (NCF_LAYOUT_USER_STORE, off by default): NCF_USER_STORE=1
            # forces it, =auto applies the per-rank batch rule (A/B)
            pr = os.environ.get("NCF_PER_ROW")  # 0|1: force the layer-0 form (A/B)
            if pr in ("0", "1"):
                L.check(L.hip().ncf_debug_set_per_row(int(pr)), "ncf_debug_set_per_row")
            us = os.environ.get("NCF_USER_STORE")
            if us in ("0", "1", "auto"):
                L.check(L.hip().ncf_debug_set_user_store(-1 if us == "auto" else int(us)), "ncf_debug_set_user_store")
            L.check(L.hip().ncf_layout_tune(ctypes.byref(self.lay), per), "ncf_layout_tune")
            if os.environ.get("NCF_FORCE_LAYERED", "0") == "1":  # A/B: the layered path for any shape
                self.lay.flags |= L.LAYOUT_LAYERED
            self._set_fact_shard()
            self.ws = ops.new_workspace(self.lay, per, self.device)
        self.batch_size = int(batch_size)
        if self.num_batches > self.loss_hist.numel():
            # the optimizer launches write loss_hist[b % num_batches]: one slot per
            # batch of the epoch (a captured graph holds the old pointer: re-capture)
            self.loss_hist = torch.zeros(self.num_batches, dtype=torch.float32, device=self.device)
            self._drop_graphs()
        # device-side fills (an assignment from a host scalar is a pageable copy that
        # blocks the host until the stream drains, i.e. until the previous epoch ends)
        if n != getattr(self, "_ctl_n", None):
            self.ctl[0:4:3].zero_()
            self.ctl[2:3].fill_(n)
            self._ctl_n = n
        else:
            self.ctl[0:1].zero_()
        self._check_stream_agreement(rows)
        if self.dp_mode == "auto":
            self._resolve_auto(batch_size)
        if self.dp_mode == "owner":
            self._owner_prepare(rows)
        # deferred Adam: touched rows of every batch of this stream (once per epoch)
        lazy = self._lazy_wanted()
        if self.lazy and not lazy:
            self.flush()  # back to dense Adam: every row current first
        if self.dp_mode == "touched":
            pf = int(L.hip().ncf_touched_packed_floats(ctypes.byref(self.lay), self._ranges, self._nranges,
                                                       self.batch_size))
            if self._packed.numel() != pf:
                self._packed = torch.zeros(pf, dtype=torch.float32, device=self.device)
                self._drop_graphs()
        if lazy:
            lib = L.hip()
            if self._last is None:
                U, I = self.model.user_num, self.model.item_num
                self._last = torch.zeros(U + I, dtype=torch.int32, device=self.device)
                self._ring = torch.zeros(2 * self.LAZY_RING, dtype=torch.float32, device=self.device)
            if not self.lazy:  # rows are current as of the present step
                self._last.copy_(self.ctl[1:2].to(torch.int32).expand_as(self._last))
            L.check(lib.ncf_batch_touched(rows.data_ptr(), n, self.batch_size, self.model.user_num,
                                          self.model.item_num, self._touched_buf(rows).data_ptr(),
                                          L.stream_ptr(self.device)), "ncf_batch_touched")
        self.lazy = lazy
        # the rows of each rank slice by user, once per epoch (ncf_user_order): the layered
        # factored layer 0 sums user runs before its atomics; the fused step with
        # NCF_LAYOUT_USER_STORE sums its stored user-side rows over them
        self._uses_order = (os.environ.get("NCF_USER_ORDER", "1") == "1"
                            and bool(L.hip().ncf_uses_user_order(ctypes.byref(self.lay))))
        if self._uses_order:
            L.check(L.hip().ncf_user_order(rows.data_ptr(), n, self.batch_size, self.world_size,
                                           self.model.user_num, self._order_buf(rows).data_ptr(),
                                           L.stream_ptr(self.device)), "ncf_user_order")
        if self.distill is not None:
            # the frozen teacher's logit for every row of the epoch stream (one
            # forward launch per epoch instead of one no_grad forward per step)
            self.distill.teacher_logits(rows)

    def _set_fact_shard(self):
        """zero1 on the factored fused path (dm <= 64, Adam): the step forms only the
        dW0 partials (NCF_LAYOUT_FACT_DEFER_DX) and each rank expands the summed G rows
        of its own shard inside its Adam launch (ncf_adam_step_fact) -- the expansion
        and the optimizer sharded together, 1/W of each per rank.  NCF_FACT_SHARD=0
        keeps the full expansion before the reduce-scatter (A/B)."""
        lay, m = self.lay, self.model
        self._fact_shard = bool(
            self.dp_mode == "zero1" and self.optimizer == "adam" and self.distill is None
            and os.environ.get("NCF_FACT_SHARD", "1") == "1"
            and not (lay.flags & L.LAYOUT_LAYERED) and lay.dropout == 0.0
            and L.supported(m.model_type, m.factor_num, m.num_layers) == L.PATH_FUSED
            and (m.factor_num << (m.num_layers - 1)) <= 64
            and L.hip().ncf_fact_mode(ctypes.byref(lay)) == 1)
        if self._fact_shard:
            lay.flags |= L.LAYOUT_FACT_DEFER_DX
        else:
            lay.flags &= ~L.LAYOUT_FACT_DEFER_DX

    def _check_stream_agreement(self, rows):
        """world > 1: every rank must train on the same epoch stream (same seeds, and
        the canonical grouping of ncf_prepare_epoch2): a device checksum of the stream,
        max and -min over the ranks in one all-reduce.  The first stream is checked at
        once; later ones asynchronously (flag copied to pinned memory, read at a later
        epoch boundary when done), so the host does not wait for the running epoch.
        Raises RuntimeError on a mismatch."""
        if self.world_size == 1 or self.group is None:
            return
        import torch.distributed as dist
        if dist.get_world_size(self.group) != self.world_size:
            return  # an emulated world (scripts/dp_modes.py)
        self._poll_stream_checks(block=False)
        c = ops.stream_checksum(rows)
        t = torch.stack([c, -c])
        if D._coll_ok(t, self.group):
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        else:
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.MAX, group=self.group)
            t = h.to(self.device)
        bad = (t[0] + t[1]) != 0
        flag = torch.empty(1, dtype=torch.bool, pin_memory=True)
        flag.copy_(bad.view(1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._stream_checks = getattr(self, "_stream_checks", []) + [(flag, ev)]
        if not getattr(self, "_stream_checked_once", False):
            self._stream_checked_once = True
            self._poll_stream_checks(block=True)

    def _poll_stream_checks(self, block):
        keep = []
        for flag, ev in getattr(self, "_stream_checks", []):
            if block:
                ev.synchronize()
            if not ev.query():
                keep.append((flag, ev))
                continue
            if bool(flag.item()):
                raise RuntimeError("data-parallel ranks hold different epoch streams: build them from the same "
                                   "seeds with the canonical grouping (ncf_prepare_epoch2 NCF_PREP_CANONICAL, "
                                   "ops.EpochPrep(canonical=True) / EpochPipeline(canonical=True))")
        self._stream_checks = keep

    # ------------------------------------------------------------ owner exchange
    # list slots grow to OWNER_SLACK x the longest list seen (+16, multiples of 16): the
    # exchange chunks keep one size (and the captured graphs stay valid) across epochs
    OWNER_SLACK = 1.08

    def _owner_plan_for(self, mu, mi, n=None, batch=None):
        P = L.NcfOwnerPlan()
        L.check(L.hip().ncf_owner_plan_init(ctypes.byref(self.lay), self._ranges, self._nranges,
                                            self.n_total if n is None else int(n),
                                            self.batch_size if batch is None else int(batch), self.world_size,
                                            self.rank, int(mu), int(mi), ctypes.byref(P)), "ncf_owner_plan_init")
        return P

    def owner_prebuild(self, rows, stream):
        """EpochPipeline.on_built (dp_mode "owner"): the epoch's bucket lists built on
        the pipeline's side stream right after the stream itself, with the current list
        slots, and their maxima copied to pinned memory -- so at the epoch boundary
        set_epoch_stream only reads two numbers of a build that finished long before
        (the host does not wait for the running epoch).  Lists longer than the slots are
        rebuilt there, synchronously."""
        if self.dp_mode != "owner" or self.batch_size is None or self._ow_plan is None:
            return
        mu, mi = self._ow_M
        plan = self._owner_plan_for(mu, mi, n=rows.numel())
        key = (rows.data_ptr(), rows.numel(), self.batch_size)
        lists = self._owner_lists_buf(rows, plan)
        dmax = torch.zeros(2, dtype=torch.int32, device=self.device)
        L.check(L.hip().ncf_owner_lists(ctypes.byref(plan), ctypes.byref(self.lay), rows.data_ptr(),
                                        lists.data_ptr(), dmax.data_ptr(), stream.cuda_stream), "ncf_owner_lists")
        host = torch.empty(2, dtype=torch.int32, pin_memory=True)
        host.copy_(dmax, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        self._ow_pre[key] = ((mu, mi), host, ev, dmax)

    def _owner_lists_buf(self, rows, plan):
        key = (rows.data_ptr(), rows.numel(), self.batch_size)
        ints = (int(plan.lists_bytes) + 3) // 4
        buf = self._ow_lists.get(key)
        if buf is None or buf.numel() < ints:
            if buf is not None:  # work already queued may still use it: kept until it is done
                ev = torch.cuda.Event()
                ev.record()  # the current stream (the side stream inside a prebuild)
                self._ow_old.append((buf, [ev], False))
            buf = self._ow_lists[key] = torch.zeros(ints, dtype=torch.int32, device=self.device)
        return buf

    def _owner_prepare(self, rows):
        """The epoch's bucket lists (ncf_owner_lists) for stream buffer `rows`; the list
        slots grow (the exchange buffers with them, graphs re-captured) when a list of
        this stream is longer than the slots -- the same decision on every rank, which
        all hold the same stream.  One host read of the two maxima per epoch."""
        lib = L.hip()
        st = L.stream_ptr(self.device)
        self._owner_retire()
        if self._ow_max is None:
            self._ow_max = torch.zeros(2, dtype=torch.int32, device=self.device)
        mu, mi = self._ow_M
        key = (rows.data_ptr(), rows.numel(), self.batch_size)
        pre = self._ow_pre.pop(key, None)
        if (pre is not None and pre[0] == (mu, mi) and self._ow_plan is not None
                and int(self._ow_plan.n_total) == rows.numel() and int(self._ow_plan.batch_global) == self.batch_size):
            _, host, ev, _ = pre
            ev.synchronize()  # the side-stream build (a prefetched epoch: finished long before)
            need_u, need_i = (int(x) for x in host.tolist())
            if need_u <= mu and need_i <= mi:
                torch.cuda.current_stream(self.device).wait_event(ev)
                return
        while True:
            plan = self._owner_plan_for(mu, mi)
            lists = self._owner_lists_buf(rows, plan)
            L.check(lib.ncf_owner_lists(ctypes.byref(plan), ctypes.byref(self.lay), rows.data_ptr(), lists.data_ptr(),
                                        self._ow_max.data_ptr(), st), "ncf_owner_lists")
            need_u, need_i = (int(x) for x in self._ow_max.cpu().tolist())
            if need_u <= mu and need_i <= mi:
                break
            grow = lambda need, cur: max(cur, (int(need * self.OWNER_SLACK) + 16 + 15) // 16 * 16)  # noqa: E731
            mu, mi = grow(need_u, mu), grow(need_i, mi)
        old = self._ow_plan
        self._ow_plan, self._ow_M = plan, (mu, mi)
        same = old is not None and all(getattr(old, k) == getattr(plan, k) for k in ("max_u", "max_i", "n_total",
                                                                                      "batch_global", "send_floats"))
        if not same:
            W = self.world_size
            mk = lambda n: torch.zeros(W * int(n), dtype=torch.float32, device=self.device)  # noqa: E731
            self._ow_bufs = (mk(plan.send_floats), mk(plan.send_floats), mk(plan.param_floats), mk(plan.param_floats))
            self._drop_graphs()

    def _owner_retire(self):
        """Free replaced list buffers once the work queued before their replacement is
        done: an event from the stream that replaced them, one from this (the step)
        stream at the first epoch boundary after it."""
        keep = []
        for buf, evs, main in self._ow_old:
            if not main:
                ev = torch.cuda.Event()
                ev.record()
                evs = evs + [ev]
            if not all(e.query() for e in evs):
                keep.append((buf, evs, True))
        self._ow_old = keep

    def owner_bytes_per_step(self):
        """(sent, received) bytes of this rank per step in the two all-to-alls (the chunk
        for itself excluded)."""
        P = self._ow_plan
        per = 4 * (int(P.send_floats) + int(P.param_floats)) * (self.world_size - 1)
        return per, per

    def _owner_pack(self):
        send = self._ow_bufs[0]
        L.check(L.hip().ncf_owner_pack(ctypes.byref(self._ow_plan), ctypes.byref(self.lay), self.ws.data_ptr(),
                                       self.grads.data_ptr(), self._owner_lists_buf(self.rows, self._ow_plan).data_ptr(),
                                       self.ctl.data_ptr(), send.data_ptr(), L.stream_ptr(self.device)),
                "ncf_owner_pack")

    def _owner_a2a(self, k):
        """k = 0: gradient buckets to their owners; 1: updated rows to their readers."""
        out, inp = (self._ow_bufs[1], self._ow_bufs[0]) if k == 0 else (self._ow_bufs[3], self._ow_bufs[2])
        if self.world_size == 1 and self.group is None:
            out.copy_(inp)
            return
        D.all_to_all_equal(out, inp, self.group)

    def _owner_adam(self):
        _, recv, send2, _ = self._ow_bufs
        L.check(L.hip().ncf_owner_adam(ctypes.byref(self._ow_plan), ctypes.byref(self.lay), self.flat.data_ptr(),
                                       self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), self._ranges,
                                       self._nranges, self._owner_lists_buf(self.rows, self._ow_plan).data_ptr(),
                                       self.ctl.data_ptr(), self.lr, self.betas[0], self.betas[1], self.eps,
                                       self.loss_hist.data_ptr(), self.num_batches, recv.data_ptr(),
                                       send2.data_ptr(), L.stream_ptr(self.device)), "ncf_owner_adam")

    def _owner_unpack(self):
        L.check(L.hip().ncf_owner_unpack(ctypes.byref(self._ow_plan), ctypes.byref(self.lay), self.flat.data_ptr(),
                                         self._owner_lists_buf(self.rows, self._ow_plan).data_ptr(),
                                         self.ctl.data_ptr(), self._ow_bufs[3].data_ptr(), L.stream_ptr(self.device)),
                "ncf_owner_unpack")

    def _owner_tables(self):
        lay, m = self.lay, self.model
        f, dm = m.factor_num, m.factor_num << (m.num_layers - 1)
        P = self._ow_plan
        return [(int(P.off[k]), w, n) for k, (w, n) in enumerate(((f, m.user_num), (f, m.item_num),
                                                                   (dm, m.user_num), (dm, m.item_num)))
                if P is not None and int(P.off[k]) >= 0]

    def owner_sync(self):
        """dp_mode "owner": every owner's rows of every table to every rank (the replica
        of a rank is otherwise current only on the rows it reads).  A collective."""
        if self.dp_mode != "owner" or self._ow_plan is None or self.world_size == 1:
            return
        import torch.distributed as dist
        if self.group is None or dist.get_world_size(self.group) != self.world_size:
            return  # an emulated world on a smaller group (scripts/dp_modes.py): timing only
        D.owner_gather_rows(self.flat, self._owner_tables(), self.world_size, self.rank, self.group)

    def _order_buf(self, rows):
        """The user-order buffer that goes with epoch-stream buffer `rows`."""
        key = (rows.data_ptr(), rows.numel())
        buf = self._orders.get(key)
        if buf is None:
            n = rows.numel()  # n int64 entries + n int32 inverse positions (ncf_user_order)
            buf = self._orders[key] = torch.empty(n + (n + 1) // 2, dtype=torch.int64, device=self.device)
        return buf

    # deferred Adam: steps a row may sit out are replayed from this ring of step
    # scalars (a row's gap is at most NCF_LAZY_SPAN steps; > 514 entries required)
    LAZY_RING = 1 << 12
    # on by default where it moves fewer bytes than dense Adam: tables with more rows
    # than LAZY_RATIO x the global batch (C2, C4, C5; not C3's ml-1m at 65,536)
    LAZY_RATIO = float(os.environ.get("NCF_LAZY_RATIO", "2"))

    def _lazy_wanted(self):
        """Deferred Adam for this stream (always with dp_mode "touched"): single-process
        Adam (the fused optimizer launch), factor_num % 4 == 0, tables <= 2^20 rows,
        tables <= 2^19 rows; NCF_LAZY_ADAM=1 turns it on for single-process
        training (auto: tables larger than LAZY_RATIO x the global batch), 0 (the
        default) keeps the dense launch, measured faster on MI355X at C2, C4 and C5
        (DESIGN 3.2a)."""
        if self.dp_mode == "touched":
            return True
        env = os.environ.get("NCF_LAZY_ADAM", "0")
        if env == "0" or not self._fused_optimizer:
            return False
        U, I = self.model.user_num, self.model.item_num
        if self.model.factor_num % 4 or U > (1 << 19) or I > (1 << 19):
            return False
        return env == "1" or (U + I) > self.LAZY_RATIO * self.batch_size

    def _touched_buf(self, rows):
        key = (rows.data_ptr(), rows.numel(), self.batch_size)
        buf = self._touched_lists.get(key)
        if buf is None:
            nbytes = int(L.hip().ncf_touched_bytes(rows.numel(), self.batch_size, self.model.user_num,
                                                   self.model.item_num))
            buf = self._touched_lists[key] = torch.empty((nbytes + 3) // 4, dtype=torch.int32, device=self.device)
        return buf

    def flush(self):
        """Deferred Adam: every embedding row brought up to the current step (the
        parameters and moments are then the dense optimizer's).  In-step Adam: the
        pending update written (ncf_ais_flush).  No-op otherwise."""
        if self.dp_mode == "owner":
            self.owner_sync()
        if getattr(self, "_ais_live", False):
            b = self._ais_bufs()
            L.check(L.hip().ncf_ais_flush(ctypes.byref(self.lay), self.flat.data_ptr(), self.grads.data_ptr(),
                                          self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), ctypes.byref(b),
                                          self._ranges, self._nranges, self.ctl.data_ptr(), self.lr,
                                          self.betas[0], self.betas[1], self.eps, self.loss_hist.data_ptr(),
                                          self.num_batches, L.stream_ptr(self.device)), "ncf_ais_flush")
            self._ais_live = False
        if not self.lazy:
            return
        L.check(L.hip().ncf_lazy_adam_flush(ctypes.byref(self.lay), self.flat.data_ptr(), self.grads.data_ptr(),
                                            self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), self._ranges,
                                            self._nranges, self.ctl.data_ptr(), self.betas[0], self.betas[1],
                                            self.eps, self._last.data_ptr(), self._ring.data_ptr(),
                                            self.LAZY_RING, L.stream_ptr(self.device)), "ncf_lazy_adam_flush")

    def optimizer_state_set(self):
        """Call after writing flat / exp_avg / exp_avg_sq / ctl from outside (e.g. a
        loaded or teacher-forced optimizer state): every row is current as of step
        ctl.adam_t."""
        if self._last is not None:
            self._last.copy_(self.ctl[1:2].to(torch.int32).expand_as(self._last))

    def user_order_ptr(self):
        """ncf_train_step's user_order argument for the current stream (None: unused)."""
        return self._order_buf(self.rows).data_ptr() if self._uses_order else None

    @property
    def num_batches(self):
        return (self.n_total + self.batch_size - 1) // self.batch_size

    # ------------------------------------------------------------------ step
    def _compute(self):
        """Launches 1-2: fused (or layered) step + slab reduction (advances ctl);
        dp_mode "touched": step + ncf_touched_pack (the touched rows' and the tower's
        gradients into the buffer the all-reduce sums; ctl advances in the optimizer)."""
        st = L.stream_ptr(self.device)
        self._train_launch()
        if self.dp_mode == "owner":
            self._owner_pack()
            return
        if self.dp_mode == "touched":
            L.check(L.hip().ncf_touched_pack(ctypes.byref(self.lay), self.ws.data_ptr(), self.grads.data_ptr(),
                                             self._ranges, self._nranges, self._touched_buf(self.rows).data_ptr(),
                                             self.n_total, self.batch_size, self.ctl.data_ptr(),
                                             self._packed.data_ptr(), st),
                    "ncf_touched_pack")
            return
        L.check(L.hip().ncf_reduce_slab(ctypes.byref(self.lay), self.ws.data_ptr(), self.grads.data_ptr(),
                                        self.ctl.data_ptr(), st), "ncf_reduce_slab")

    def _allreduce(self):
        """Launch 3 (world > 1): gradient exchange over ranks (RCCL on ROCm).
        zero1: reduce-scatter of the flat gradient into this rank's shard;
        allreduce: in-place sum of the whole flat gradient."""
        if self.dp_mode == "single":
            return
        if self.dp_mode == "owner":
            self._owner_a2a(0)
        elif self.dp_mode == "touched":
            D.allreduce_flat_grads(self._packed, self.group)
        elif self.dp_mode == "zero1":
            D.reduce_scatter_flat(self.gshard, self.grads, self.rank, self.group)
        else:
            D.allreduce_flat_grads(self.grads, self.group)

    def _allgather(self):
        """Launch 5 (zero1): every rank's updated parameter shard to every rank;
        owner: the rows of every rank's next batch to it, then unpacked."""
        if self.dp_mode == "owner":
            self._owner_a2a(1)
            self._owner_unpack()
        elif self.dp_mode == "zero1":
            if self._ag_scratch is None and not D._native_ok(self.flat, self.group):
                self._ag_scratch = torch.empty_like(self.flat)
            D.all_gather_flat(self.flat, self.rank, self.shard, self.group, self._ag_scratch)

    def _optimize(self):
        """Launch 4: dense Adam / SGD + grad zeroing + loss bookkeeping (zero1: over
        this rank's shard; the full local gradient buffer is zeroed for the next
        step's accumulation, and only the loss slot's owner records the loss)."""
        st = L.stream_ptr(self.device)
        lib = L.hip()
        hist_len = self.num_batches
        if self.dp_mode == "owner":
            self._owner_adam()
            return
        if self.dp_mode == "touched":
            L.check(lib.ncf_lazy_adam_step_packed(ctypes.byref(self.lay), self.flat.data_ptr(), self.exp_avg.data_ptr(),
                                                  self.exp_avg_sq.data_ptr(), self._ranges, self._nranges,
                                                  self.ctl.data_ptr(), self.lr, self.betas[0], self.betas[1], self.eps,
                                                  self.loss_hist.data_ptr(), hist_len,
                                                  self._touched_buf(self.rows).data_ptr(), self.n_total,
                                                  self.batch_size, self._last.data_ptr(), self._ring.data_ptr(),
                                                  self.LAZY_RING, self._packed.data_ptr(), st),
                                                  "ncf_lazy_adam_step_packed")
            return
        if self.dp_mode == "zero1":
            if not self._fact_shard:
                # the shard gradient is in gshard: clear the local bucket now (the
                # factored launch below clears it itself)
                L.check(lib.ncf_zero_f32(self.grads.data_ptr(), self.grads.numel(), st), "ncf_zero_f32")
            ranges, nr = self._sranges, self._nsranges
            hist = self.loss_hist.data_ptr() if self.rank == self.loss_owner else None
        else:
            ranges, nr = self._ranges, self._nranges
            hist = self.loss_hist.data_ptr()
        p, g = self._opt_ptrs
        if self._fact_shard:  # the shard's G rows expanded inside the optimizer launch (+ the bucket cleared)
            L.check(lib.ncf_adam_step_fact(ctypes.byref(self.lay), self.ws.data_ptr(), p, g, self.exp_avg.data_ptr(),
                                           self.exp_avg_sq.data_ptr(), ranges, nr, self.rank * self.shard,
                                           self.grads.data_ptr(), self.grads.numel(),
                                           self.ctl.data_ptr(), self.lr, self.betas[0], self.betas[1], self.eps,
                                           self._loss_slot, hist, hist_len, st), "ncf_adam_step_fact")
        elif self.optimizer == "adam":
            L.check(lib.ncf_adam_step(p, g, self.exp_avg.data_ptr(),
                                      self.exp_avg_sq.data_ptr(), ranges, nr,
                                      self.ctl.data_ptr(), self.lr, self.betas[0], self.betas[1], self.eps,
                                      self._loss_slot, hist, hist_len, st),
                    "ncf_adam_step")
        else:
            L.check(lib.ncf_sgd_step(p, g, ranges, nr,
                                     self.ctl.data_ptr(), self.lr, self._loss_slot,
                                     hist, hist_len, st), "ncf_sgd_step")

    @property
    def _fused_optimizer(self):
        """Single process + Adam: slab reduction and Adam in one launch
        (ncf_reduce_adam_step); otherwise reduce, [all-reduce], optimizer."""
        return self.dp_mode == "single" and self.optimizer == "adam" and os.environ.get("NCF_FUSED_ADAM", "1") == "1"

    # NCF_ADAM_IN_STEP: "auto" (default) -- the in-step optimizer where the step has at most
    # AIS_MAX_WG training workgroups (C5's 256-row batch: 11.7 against 12.0 us/step; at
    # C2's 16 workgroups the on-the-fly update quadruples each CU's gather loads and the
    # step takes 22.7 against 18.4 us, profiles/r05_evidence/ais_ab/); "1" wherever the
    # kernel exists, "0" never
    ADAM_IN_STEP = os.environ.get("NCF_ADAM_IN_STEP", "auto")
    AIS_MAX_WG = int(os.environ.get("NCF_AIS_MAX_WG", "4"))

    @property
    def _ais_active(self):
        """In-step Adam (ABI 18, ncf_train_step_ais): single process, dense Adam, the fused
        small-batch kernel with per-row layer 0; response distillation only (its logits
        ride in the launch, feature terms would add into the gradient separately)."""
        mode = {True: "1", False: "0"}.get(self.ADAM_IN_STEP, self.ADAM_IN_STEP)
        if mode == "0" or not self._fused_optimizer or self.lazy:
            return False
        if self.distill is not None and self.distill.keys:
            return False
        if not L.hip().ncf_ais_supported(ctypes.byref(self.lay)):
            return False
        if mode == "auto":
            wg = (int(self.lay.flags) >> L.LAYOUT_WG_SHIFT) & L.LAYOUT_WG_MASK
            return 0 < wg <= self.AIS_MAX_WG
        return True

    def _ais_bufs(self):
        if getattr(self, "_ais_b", None) is None:
            n = int(self.lay.total)
            z = lambda: torch.zeros(n, dtype=torch.float32, device=self.device)  # noqa: E731
            self._ais_t = [z() for _ in range(5)] + [torch.zeros(4, dtype=torch.int64, device=self.device)]
            self._ais_b = L.NcfAisBufs(*[t.data_ptr() for t in self._ais_t])
        return self._ais_b

    def _ais_begin(self):
        if getattr(self, "_ais_live", False):
            return
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("in-step Adam: ncf_ais_begin must run before graph capture")
        b = self._ais_bufs()
        L.check(L.hip().ncf_ais_begin(ctypes.byref(self.lay), self.flat.data_ptr(), self.grads.data_ptr(),
                                      self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), ctypes.byref(b),
                                      self._ranges, self._nranges, self.ctl.data_ptr(), L.stream_ptr(self.device)),
                "ncf_ais_begin")
        self._ais_live = True

    def _ais_launch(self, step_i):
        st = L.stream_ptr(self.device)
        b = self._ais_bufs()
        if self.distill is not None:
            d = self.distill
            dl, dz, kd = d.tlog.data_ptr(), L.DZ_KD, (d.w_task, d.w_resp, d.temperature)
        else:
            dl, dz, kd = None, L.DZ_BCE, (0.0, 0.0, 0.0)
        L.check(L.hip().ncf_train_step_ais(ctypes.byref(self.lay), self.flat.data_ptr(), self.grads.data_ptr(),
                                           self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), ctypes.byref(b),
                                           self._ranges, self._nranges, self.rows.data_ptr(), dl, self.ctl.data_ptr(),
                                           self.batch_size, dz, kd[0], kd[1], kd[2], self.lr, self.betas[0],
                                           self.betas[1], self.eps, self.loss_hist.data_ptr(), self.num_batches,
                                           step_i, st), "ncf_train_step_ais")

    def _ais_bump(self, k):
        L.check(L.hip().ncf_ais_bump(self.ctl.data_ptr(), ctypes.byref(self._ais_bufs()), k,
                                     L.stream_ptr(self.device)), "ncf_ais_bump")

    def _train_launch(self):
        st = L.stream_ptr(self.device)
        if self._ais_active:  # one whole step: the previous step's Adam rides in this launch
            self._ais_begin()
            self._ais_launch(0)
            self._ais_bump(1)
            return
        if self.distill is not None:
            self.distill.launch(self, st)
            return
        L.check(L.hip().ncf_train_step(ctypes.byref(self.lay), self.flat.data_ptr(), self.grads.data_ptr(),
                                       self.rows.data_ptr(), self.user_order_ptr(), None, self.ctl.data_ptr(),
                                       self.batch_size,
                                       self.world_size, self.rank, L.DZ_BCE, self.ws.data_ptr(),
                                       self.ws.numel() * 4, None, st), "ncf_train_step")

    def _reduce_adam(self):
        st = L.stream_ptr(self.device)
        if self._ais_active:  # inside the next training launch (or ncf_ais_flush)
            return
        if self.lazy:
            L.check(L.hip().ncf_lazy_adam_step(ctypes.byref(self.lay), self.ws.data_ptr(), self.flat.data_ptr(),
                                               self.grads.data_ptr(), self.exp_avg.data_ptr(),
                                               self.exp_avg_sq.data_ptr(), self._ranges, self._nranges,
                                               self.ctl.data_ptr(), self.lr, self.betas[0], self.betas[1], self.eps,
                                               self.loss_hist.data_ptr(), self.num_batches,
                                               self._touched_buf(self.rows).data_ptr(), self.n_total,
                                               self.batch_size, self._last.data_ptr(), self._ring.data_ptr(),
                                               self.LAZY_RING, st), "ncf_lazy_adam_step")
            return
        L.check(L.hip().ncf_reduce_adam_step(ctypes.byref(self.lay), self.ws.data_ptr(), self.flat.data_ptr(),
                                             self.grads.data_ptr(), self.exp_avg.data_ptr(),
                                             self.exp_avg_sq.data_ptr(), self._ranges, self._nranges,
                                             self.ctl.data_ptr(), self.lr, self.betas[0], self.betas[1], self.eps,
                                             self.loss_hist.data_ptr(), self.num_batches, st),
                "ncf_reduce_adam_step")

    def _step_body(self):
        if self._fused_optimizer:
            self._train_launch()
            self._reduce_adam()
            return
        self._compute()
        self._allreduce()
        self._optimize()
        self._allgather()

    def time_kernels(self, n_steps):
        """Run n_steps eager steps with HIP events between the launches (on the
        stream they run on) and return mean milliseconds per launch group."""
        st = torch.cuda.current_stream(self.device)
        if self._ais_active:  # one launch per step: the previous step's Adam rides in it
            parts = [("ncf_train_step_ais", self._train_launch)]
        elif self._fused_optimizer:
            parts = [("ncf_train_step", self._train_launch),
                     ("ncf_lazy_adam_step" if self.lazy else "ncf_reduce_adam_step", self._reduce_adam)]
        else:
            parts = [("ncf_train_step", self._train_launch),
                     ("ncf_reduce_slab", lambda: L.check(L.hip().ncf_reduce_slab(
                         ctypes.byref(self.lay), self.ws.data_ptr(), self.grads.data_ptr(), self.ctl.data_ptr(),
                         L.stream_ptr(self.device)), "ncf_reduce_slab")),
                     ("reduce_scatter" if self.dp_mode == "zero1" else "allreduce",
                      self._allreduce),
                     ("optimizer", self._optimize)]
            if self.dp_mode == "owner":  # the pack is part of _compute
                parts = [("ncf_train_step+ncf_owner_pack", self._compute),
                         ("all_to_all_grads", lambda: self._owner_a2a(0)), ("ncf_owner_adam", self._optimize),
                         ("all_to_all_params", lambda: self._owner_a2a(1)), ("ncf_owner_unpack", self._owner_unpack)]
            if self.dp_mode == "touched":  # the pack is part of _compute
                parts = [("ncf_train_step+ncf_touched_pack", self._compute), ("allreduce", self._allreduce),
                         ("ncf_lazy_adam_step_packed", self._optimize)]
            if self.dp_mode == "zero1":
                parts.append(("all_gather", self._allgather))
        acc = {k: 0.0 for k, _ in parts}
        evs = []
        self.flush()  # timing starts from current rows (as a fresh epoch would)
        for _ in range(n_steps):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(len(parts) + 1)]
            e[0].record(st)
            for k, (_, fn) in enumerate(parts):
                fn()
                e[k + 1].record(st)
            evs.append(e)
        self.flush()
        torch.cuda.synchronize(self.device)
        for e in evs:
            for k, (name, _) in enumerate(parts):
                acc[name] += e[k].elapsed_time(e[k + 1])
        return {k: v / max(1, n_steps) for k, v in acc.items()}

    def time_train_kernel(self, reps):
        """Mean duration (ms) of the gradient-forming launches of one step -- the
        fused step kernel and, on the factored path, ncf_expand_grads: `reps`
        back-to-back launch groups on the current batch between one HIP event pair
        on the launch stream (per-launch event pairs add several microseconds each).
        The gradient buffer is zeroed afterwards (the launches accumulate into it)."""
        st = torch.cuda.current_stream(self.device)
        lib = L.hip()
        lay = ctypes.byref(self.lay)
        sp = L.stream_ptr(self.device)

        def launch():
            if self.distill is not None:  # the student's step: ncf_train_step_kd [+ feature terms]
                self.distill.launch(self, sp)
                return
            L.check(lib.ncf_train_step(lay, self.flat.data_ptr(), self.grads.data_ptr(), self.rows.data_ptr(),
                                       self.user_order_ptr(), None, self.ctl.data_ptr(), self.batch_size, self.world_size, self.rank,
                                       L.DZ_BCE, self.ws.data_ptr(), self.ws.numel() * 4, None, sp), "ncf_train_step")
        launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            launch()
        e1.record(st)
        torch.cuda.synchronize(self.device)
        self.grads.zero_()
        return e0.elapsed_time(e1) / reps

    def step(self):
        """One optimizer step on global batch ctl.batch (eager launches)."""
        self._step_body()
        if getattr(self, "_ais_live", False):
            self.flush()  # in-step Adam: the update written now, not in the next launch

    @property
    def _capture_collective(self):
        """Capture the all-reduce inside the step graph (one graph per step).  Off by
        default for world > 1: the step is then two graphs (compute, optimizer)
        with the collective issued eagerly between them, which needs nothing of
        the process group beyond a plain all_reduce (any backend)."""
        if self.dp_mode == "single":
            return True
        if self.dp_mode == "owner":  # RCCL: both all-to-alls inside the step graph unless turned off
            if getattr(self, "_owner_capture_failed", False):
                return False
            default = "1" if D.capturable(self.grads, self.group) else "0"
            return os.environ.get("NCF_CAPTURE_ALLREDUCE", default) == "1"
        return os.environ.get("NCF_CAPTURE_ALLREDUCE", "0") == "1"

    def _graph_of(self, fn):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                fn()
        torch.cuda.current_stream(self.device).wait_stream(s)
        return g

    # steps unrolled into one graph when the collective is captured too (single
    # process): fewer graph launches, no host work between consecutive steps.
    # NCF_GRAPH_STEPS fixes it; by default the whole epoch for epochs of at most 128
    # steps (C3's 76: 56.6 -> 56.1 us/step against 8 -- no single-step remainder
    # replays), else 32 (C2 19.10 -> 18.42 us, C5 12.57 -> 12.18 us against 8; 128 no
    # better), profiles/r04_evidence/graph_steps_ab.log
    GRAPH_STEPS = int(os.environ.get("NCF_GRAPH_STEPS", "0"))

    @property
    def graph_steps(self):
        if self.GRAPH_STEPS > 0:
            return self.GRAPH_STEPS
        return self.num_batches if self.num_batches <= 128 else 32

    def capture(self):
        """Capture the step into hipGraph(s) (after at least one eager step).  dp_mode
        "owner": if capturing the all-to-alls raises, the collectives go eager between
        graphs from then on (a warning says so) instead of failing the run."""
        if self.dp_mode == "owner" and self._capture_collective:
            try:
                return self._capture()
            except RuntimeError as e:
                import warnings
                warnings.warn(f"owner exchange: capturing the all-to-alls failed ({e}); eager collectives")
                self._owner_capture_failed = True
                torch.cuda.synchronize(self.device)
        return self._capture()

    def _capture(self):
        if self._capture_collective:
            self._graph = (self._graph_of(self._step_body),)
            k = self.graph_steps
            self._graph_k = None
            if k > 1:
                if self._ais_active:
                    def body():  # k launches, one bump: each launch applies its predecessor's Adam
                        for j in range(k):
                            self._ais_launch(j)
                        self._ais_bump(k)
                else:
                    def body():
                        for _ in range(k):
                            self._step_body()
                self._graph_k = (self._graph_of(body), k)  # the k-step graph and its step count
        elif self.dp_mode == "owner":
            # (compute, optimize, unpack + next compute, unpack): the collectives between
            # them from the host (_run_owner)
            def unpack_compute():
                self._owner_unpack()
                self._compute()
            self._graph = ("owner", self._graph_of(self._compute), self._graph_of(self._optimize),
                           self._graph_of(unpack_compute), self._graph_of(self._owner_unpack))
            self._graph_k = None
        else:
            self._graph = (self._graph_of(self._compute), self._graph_of(self._optimize))
            if self.dp_mode in ("allreduce", "touched"):
                # step t's optimizer and step t + 1's compute in one graph: one replay and
                # one collective per step from the host (run())
                def opt_compute():
                    self._optimize()
                    self._compute()
                self._graph = self._graph + (self._graph_of(opt_compute),)
            self._graph_k = None
        self._graphs[(self.batch_size, self.n_total, self.rows.data_ptr())] = (self._graph, self._graph_k)
        return self._graph

    def _capture_buffers(self):
        """Capture for every registered stream buffer not captured yet (the
        launches read the rows pointer only when replayed)."""
        cur = (self.rows, self._graph, self._graph_k)
        try:
            for buf in self.stream_buffers:
                key = (self.batch_size, self.n_total, buf.data_ptr())
                if (buf.numel() != self.n_total or buf.dtype != torch.int64 or buf.device != self.device
                        or key in self._graphs):
                    continue
                self.rows = buf
                if self._uses_order:
                    self._order_buf(buf)  # allocated outside the capture (filled when the buffer is set)
                if self.lazy:
                    self._touched_buf(buf)
                if self.dp_mode == "owner":  # allocated outside the capture (filled when the buffer is set)
                    self._owner_lists_buf(buf, self._ow_plan)
                self.capture()
        finally:
            self.rows, self._graph, self._graph_k = cur

    def _drop_graphs(self):
        self._graph = self._graph_k = None
        self._graphs = {}

    def _replay(self):
        if self._graph[0] == "owner":
            self._run_owner(1)
            return
        if len(self._graph) == 1:
            self._graph[0].replay()
        else:  # (compute, optimize[, optimize + compute])
            self._graph[0].replay()
            self._allreduce()
            self._graph[1].replay()
            self._allgather()

    def run(self, n_steps, use_graph=True):
        """n_steps consecutive optimizer steps (batches advance on device).  With
        deferred Adam the embedding rows are brought up to the last step at the end
        (ncf_lazy_adam_flush: a pass over the per-row step counters; rows the last
        batch of an epoch already caught up cost nothing), so the parameters are the
        dense optimizer's whenever run() returns."""
        if self._ais_active:
            self._ais_begin()  # eager: the step graphs may replay without an eager step first
        self._run(n_steps, use_graph)
        self.flush()

    def _run(self, n_steps, use_graph=True):
        if not use_graph:
            for _ in range(n_steps):
                self._step_body()
            return
        key = (self.batch_size, self.n_total, self.rows.data_ptr())
        done = 0
        self._graph, self._graph_k = self._graphs.get(key, (None, None))
        if self._graph is None:
            # eager first step also sets kernel attributes outside the capture
            self._step_body()
            done = 1
            if n_steps <= 1:
                return
            self.capture()  # captured launches are recorded, not executed
            self._capture_buffers()
        left = n_steps - done
        if self._graph_k is not None:
            gk, k = self._graph_k
            for _ in range(left // k):
                gk.replay()
            left %= k
        if self._graph[0] == "owner":
            self._run_owner(left)
            return
        if len(self._graph) == 3 and left >= 2:
            # eager all-reduce between graphs: compute(t0), then [optimize(t), compute(t+1)]
            # per step, the last optimize after the loop -- the launch order of
            # left x _replay() with one host replay per step fewer
            self._graph[0].replay()
            self._allreduce()
            for _ in range(left - 1):
                self._graph[2].replay()
                self._allreduce()
            self._graph[1].replay()
            return
        for _ in range(left):
            self._replay()

    def _run_owner(self, n):
        """n owner-mode steps from the graphs of capture(): compute(t0), then per step
        a2a, optimize, a2a, [unpack(t) + compute(t + 1)], and the last unpack."""
        if n <= 0:
            return
        _, g_c, g_o, g_uc, g_u = self._graph
        g_c.replay()
        for s in range(n):
            self._owner_a2a(0)
            g_o.replay()
            self._owner_a2a(1)
            (g_uc if s + 1 < n else g_u).replay()

    def epoch_losses(self):
        """Per-batch mean BCE of the last epoch (host copy).  zero1: the rank owning
        the loss slot recorded it; it is broadcast to the others (a collective: every
        rank calls this)."""
        if self.dp_mode == "zero1":
            import torch.distributed as dist
            h = self.loss_hist[: self.num_batches].clone()
            if D._native_ok(h, self.group):
                dist.broadcast(h, src=self.loss_owner, group=self.group)
            else:
                h = h.cpu()
                dist.broadcast(h, src=self.loss_owner, group=self.group)
            return h.double().cpu().numpy()
        return self.loss_hist[: self.num_batches].double().cpu().numpy()

    def state_step(self):
        return int(self.ctl[1].item())

    def zero_state(self):
        self.grads.zero_()
        if self.optimizer == "adam":
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
        self.ctl[1] = 0
        if self._last is not None:
            self._last.zero_()
