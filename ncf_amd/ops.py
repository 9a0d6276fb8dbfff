"""Device-side operators of the NeuMF hot path (torch tensors -> C ABI pointers).

``ensure_flat`` packs a HIP-resident NCF's parameters into one flat fp32 buffer
laid out by ``ncf_layout_init`` (include/ncf_hip.h) and rebinds every
``nn.Parameter`` to a view of it, so the kernels read the live weights and the
module's ``state_dict`` / stock optimizers keep working.

``ncf_forward`` is the autograd-visible forward of ``NCF`` on a HIP device
(reference models.py:97-118); its backward is the same fused kernel in
``NCF_DZ_DLOGIT`` mode (replacing the ATen autograd graph that
``loss.backward()`` walks in train_neumf.py:114).  Everything runs on
``torch.cuda.current_stream()``.
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch

from . import _lib as L


def _segments(model, lay):
    """(param, flat offset) in model.ordered_params() order."""
    offs = [lay.ug, lay.ig, lay.um, lay.im]
    for k in range(model.num_layers):
        offs += [lay.w[k], lay.b[k]]
    offs += [lay.wp, lay.bp]
    return list(zip(model.ordered_params(), offs))


@contextlib.contextmanager
def params_view(model, flat_snapshot):
    """The model's parameters temporarily viewing `flat_snapshot` (a copy of its
    flat buffer): e.g. a checkpoint of the parameters as an earlier step left them
    while later steps are already queued.  Nothing may repack the model inside."""
    lay = model._ncf_layout
    segs = _segments(model, lay)
    saved = [p.data for p, _ in segs]
    try:
        for p, off in segs:
            p.data = flat_snapshot[off:off + p.numel()].view_as(p)
        yield model
    finally:
        for (p, _), d in zip(segs, saved):
            p.data = d


def active_mask(model):
    """Which ordered params receive gradients (reference: unused tables keep
    .grad None in GMF / MLP mode, so torch Adam skips them)."""
    n_tower = 2 * model.num_layers
    if model.model_type == "GMF":
        return [True, True, False, False] + [False] * n_tower + [True, True]
    if model.model_type == "MLP":
        return [False, False, True, True] + [True] * n_tower + [True, True]
    return [True] * (4 + n_tower + 2)


def ensure_flat(model, min_floats=0):
    """Return (flat, layout) for a HIP-resident NCF, (re)packing if needed.
    ``min_floats``: the flat buffer is at least this long (zero padding after
    ``lay.total``; the sharded data-parallel optimizer needs world * shard floats)."""
    lay = getattr(model, "_ncf_layout", None)
    flat = getattr(model, "_ncf_flat", None)
    dev = model.embed_user_GMF.weight.device
    if lay is None:
        lay = L.layout(model.user_num, model.item_num, model.factor_num, model.num_layers, model.model_type)
        model._ncf_layout = lay
    if flat is not None and flat.device == dev and flat.numel() >= min_floats:
        ok = all(p.data_ptr() == flat.data_ptr() + 4 * off for p, off in _segments(model, lay))
        if ok:
            return flat, lay
    if not L.supported(model.model_type, model.factor_num, model.num_layers):
        raise NotImplementedError(
            f"no HIP path for model_type={model.model_type} factor_num={model.factor_num} "
            f"num_layers={model.num_layers}")
    flat = torch.zeros(max(int(lay.total), int(min_floats)), dtype=torch.float32, device=dev)
    with torch.no_grad():
        for p, off in _segments(model, lay):
            n = p.numel()
            view = flat[off:off + n].view_as(p)
            view.copy_(p.data)
            p.data = view
    model._ncf_flat = flat
    return flat, lay


def _as_i32(x, dev):
    x = torch.as_tensor(x, device=dev)
    if x.dtype != torch.int32:
        x = x.to(torch.int32)
    return x.contiguous()


def pack_rows(users_i32, items_i32, labels_f32=None, out=None):
    """Packed uint64 rows (stored as int64): user | item << 32 | (label != 0) << 63
    (include/ncf_hip.h NCF_ROW_PACK), built on the device by ncf_pack_rows."""
    n = users_i32.numel()
    dev = users_i32.device
    if items_i32.numel() != n or (labels_f32 is not None and labels_f32.numel() != n):
        raise ValueError("users/items/labels must have equal length")
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=dev)
    L.check(L.hip().ncf_pack_rows(users_i32.data_ptr(), items_i32.data_ptr(),
                                  None if labels_f32 is None else labels_f32.data_ptr(), n, out.data_ptr(),
                                  L.stream_ptr(dev)), "ncf_pack_rows")
    return out


def check_ids(users, items, user_num, item_num):
    """nn.Embedding's range check (reference models.py:98-112 raise IndexError on an
    id outside the table) for host arrays; the kernels do not bound-check gathers."""
    u = np.asarray(users)
    i = np.asarray(items)
    if u.size and (int(u.min()) < 0 or int(u.max()) >= user_num):
        raise IndexError("index out of range in self (user id)")
    if i.size and (int(i.min()) < 0 or int(i.max()) >= item_num):
        raise IndexError("index out of range in self (item id)")


def check_rows(rows, user_num, item_num):
    """Range check of a packed device stream (padding rows, user -1, allowed): a
    few reductions on the device and one host read."""
    if rows.numel() == 0:
        return
    u = (rows & 0xFFFFFFFF).to(torch.int64)
    it = (rows >> 32) & 0x7FFFFFFF
    pad = u == 0xFFFFFFFF
    bad_u = ((u >= user_num) & ~pad).any()
    bad_i = ((it >= item_num) & ~pad).any()
    bu, bi = torch.stack([bad_u, bad_i]).tolist()
    if bu:
        raise IndexError("index out of range in self (user id)")
    if bi:
        raise IndexError("index out of range in self (item id)")


def pack_rows_host(users, items, labels=None):
    """Host-side NCF_ROW_PACK of numpy arrays -> int64 numpy array."""
    r = np.asarray(users).astype(np.int64) & 0xFFFFFFFF
    r |= (np.asarray(items).astype(np.int64) & 0x7FFFFFFF) << 32
    if labels is not None:
        r |= (np.asarray(labels) != 0).astype(np.int64) << 63
    return r


def default_canonical():
    """True when torch.distributed runs more than one rank (the grouping must then be
    NCF_PREP_CANONICAL so every rank's stream is identical)."""
    import torch.distributed as dist
    return bool(dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1)


_CHECK_W = {}


def stream_checksum(rows):
    """Order-sensitive int64 checksum of a device epoch stream (a few launches per
    chunk, no host sync): sum_k rows[k] * w_k (mod 2^64), w_k = (k * K) | 1.  Chunked:
    w of a chunk at offset o is (j * K + o * K) | 1 from one cached chunk-sized j * K,
    so no stream-length temporary is kept or allocated (C4: 99M rows)."""
    n = rows.numel()
    K = -7046029254386353131
    c = min(n, _CHECK_CHUNK)
    key = (c, rows.device)
    base = _CHECK_W.get(key)
    if base is None:
        base = torch.arange(c, dtype=torch.int64, device=rows.device) * K
        _CHECK_W.clear()
        _CHECK_W[key] = base
    total = torch.zeros((), dtype=torch.int64, device=rows.device)
    for o in range(0, n, c):
        m = min(c, n - o)
        # o * K wraps in int64 like the device product does
        ok = ((o * K + (1 << 63)) % (1 << 64)) - (1 << 63)
        total += (rows[o:o + m] * ((base[:m] + ok) | 1)).sum()
    return total


_CHECK_CHUNK = 1 << 22


class EpochPrep:
    """ncf_prepare_epoch with its device workspace kept between epochs (stable
    pointers, so the output can feed a captured step graph).  canonical: the rows
    of one item inside a batch in (user, label) order (NCF_PREP_CANONICAL), so that
    every data-parallel rank building the stream gets the same positions."""

    def __init__(self, device, canonical=None):
        """canonical None: on whenever torch.distributed is initialised with more than
        one rank (a data-parallel caller needs it; TrainEngine also checks that the
        ranks' streams agree)."""
        self.device = torch.device(device)
        self.ws = None
        self.out = None
        self.canonical = default_canonical() if canonical is None else bool(canonical)

    def __call__(self, rows, perm, batch_size, item_num, out=None):
        """On the current stream; into `out` (n int64 on the device) if given."""
        n = rows.numel()
        need = int(L.hip().ncf_prepare_epoch_workspace(n, int(batch_size), int(item_num)))
        if need < 0:
            raise ValueError("bad ncf_prepare_epoch sizes")
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        if out is None:
            if self.out is None or self.out.numel() != n:
                self.out = torch.empty(n, dtype=torch.int64, device=self.device)
            out = self.out
        elif out.numel() != n or out.dtype != torch.int64 or not out.is_contiguous():
            raise ValueError("prepare_epoch out: n contiguous int64")
        L.check(L.hip().ncf_prepare_epoch2(rows.data_ptr(), perm.data_ptr(), n, int(batch_size), int(item_num),
                                           L.PREP_CANONICAL if self.canonical else 0, out.data_ptr(),
                                           self.ws.data_ptr(), self.ws.numel(), L.stream_ptr(self.device)),
                "ncf_prepare_epoch2")
        return out


def _ws(owner, attr, nbytes, dev):
    """Device workspace of at least nbytes, cached on `owner` (grown, never shrunk)."""
    if nbytes <= 0:
        return None
    ws = getattr(owner, attr, None)
    if ws is None or ws.numel() * 4 < nbytes or ws.device != dev:
        ws = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=dev)
        setattr(owner, attr, ws)
    return ws


def forward_logits(flat, lay, rows, out=None, ws_owner=None):
    n = rows.numel()
    dev = flat.device
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=dev)
    need = int(L.hip().ncf_forward_workspace_bytes(L.ctypes.byref(lay), n))
    ws = _ws(ws_owner if ws_owner is not None else _scratch, "_ncf_fwd_ws", need, dev)
    L.check(L.hip().ncf_forward(L.ctypes.byref(lay), flat.data_ptr(), rows.data_ptr(), n, out.data_ptr(),
                                None if ws is None else ws.data_ptr(), 0 if ws is None else ws.numel() * 4,
                                L.stream_ptr(dev)), "ncf_forward")
    return out


def fact_mode(lay):
    """Whether the factored layer-0 path runs for this layout (include/ncf_hip.h
    ncf_fact_mode; fused or layered path)."""
    return bool(L.hip().ncf_fact_mode(L.ctypes.byref(lay)))


def new_workspace(lay, rows, dev):
    """ncf_train_step workspace for up to `rows` rows per launch (float32 storage)."""
    need = int(L.hip().ncf_workspace_bytes(L.ctypes.byref(lay), int(rows)))
    if need < 0:
        raise ValueError("ncf_workspace_bytes failed")
    return torch.zeros((need + 3) // 4, dtype=torch.float32, device=dev)


def fused_backward(flat, lay, rows, dlogit, gflat, ws, ctl):
    """grads of sum_i dlogit[i] * logit[i] into gflat (zero-initialised)."""
    n = rows.numel()
    dev = flat.device
    st = L.stream_ptr(dev)
    L.check(L.hip().ncf_train_step(L.ctypes.byref(lay), flat.data_ptr(), gflat.data_ptr(), rows.data_ptr(), None,
                                   dlogit.data_ptr(), ctl.data_ptr(), int(n), 1, 0, L.DZ_DLOGIT,
                                   ws.data_ptr(), ws.numel() * 4, None, st), "ncf_train_step")
    L.check(L.hip().ncf_reduce_slab(L.ctypes.byref(lay), ws.data_ptr(), gflat.data_ptr(), ctl.data_ptr(), st),
            "ncf_reduce_slab")


class _Scratch:
    pass


_scratch = _Scratch()


def new_ctl(n_total, dev, batch=0, adam_t=0):
    """ncf_step_ctl: batch, adam_t, n_total, reserved, snap_batch, snap_t."""
    return torch.tensor([batch, adam_t, n_total, 0, 0, 0], dtype=torch.int64, device=dev)


def dropout_seed(dev):
    """The dropout hash seed: the device generator's seed (torch.manual_seed sets it)."""
    return int(torch.cuda.initial_seed()) & 0xFFFFFFFF


def set_dropout(lay, model):
    """Copy the model's tower dropout into a training layout (GMF has no tower)."""
    p = float(getattr(model, "dropout", 0.0) or 0.0)
    if p > 0 and model.model_type != "GMF":
        lay.dropout = p
        lay.dropout_seed = dropout_seed(model.embed_user_GMF.weight.device)
    else:
        lay.dropout = 0.0


def _dropout_layout(model):
    """Training-mode layout with the model's dropout, or None when dropout is off."""
    if not model.training:
        return None
    lay = type(model._ncf_layout).from_buffer_copy(model._ncf_layout)
    set_dropout(lay, model)
    if not lay.dropout > 0:
        return None
    model._ncf_drop_t = getattr(model, "_ncf_drop_t", -1) + 1  # a fresh mask per forward
    return lay, model._ncf_drop_t


def _dropout_logits(model, rows, drop):
    """Training-mode logits under dropout: the train step with dL/dlogit = 0 (same
    masks as the backward, which reruns it with the same step index)."""
    lay, t = drop
    flat = model._ncf_flat
    dev = flat.device
    n = rows.numel()
    logits = torch.empty(n, dtype=torch.float32, device=dev)
    scratch = torch.zeros(int(lay.total), dtype=torch.float32, device=dev)
    ws = new_workspace(lay, n, dev)
    ctl = new_ctl(n, dev, adam_t=t)
    dl = torch.zeros(n, dtype=torch.float32, device=dev)
    L.check(L.hip().ncf_train_step(L.ctypes.byref(lay), flat.data_ptr(), scratch.data_ptr(), rows.data_ptr(), None,
                                   dl.data_ptr(), ctl.data_ptr(), int(n), 1, 0, L.DZ_DLOGIT,
                                   ws.data_ptr(), ws.numel() * 4, logits.data_ptr(), L.stream_ptr(dev)),
            "ncf_train_step")
    return logits


class _NCFFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rows, model, *params):
        flat, lay = model._ncf_flat, model._ncf_layout
        drop = _dropout_layout(model)
        if drop is None:
            logits = forward_logits(flat, lay, rows, ws_owner=model)
        else:
            logits = _dropout_logits(model, rows, drop)
        ctx.model = model
        ctx.drop = drop
        ctx.save_for_backward(rows)
        return logits

    @staticmethod
    def backward(ctx, grad_out):
        (rows,) = ctx.saved_tensors
        model = ctx.model
        flat, lay = model._ncf_flat, model._ncf_layout
        if ctx.drop is not None:
            lay = ctx.drop[0]
        dev = flat.device
        gflat = torch.zeros(int(lay.total), dtype=torch.float32, device=dev)
        ws = new_workspace(lay, rows.numel(), dev)
        ctl = new_ctl(rows.numel(), dev, adam_t=ctx.drop[1] if ctx.drop is not None else 0)
        dlogit = grad_out.contiguous().to(torch.float32)
        fused_backward(flat, lay, rows, dlogit, gflat, ws, ctl)
        grads = []
        for (p, off), act in zip(_segments(model, lay), active_mask(model)):
            grads.append(gflat[off:off + p.numel()].view_as(p) if act and p.requires_grad else None)
        return (None, None, *grads)


def ncf_forward(model, user, item):
    flat, lay = ensure_flat(model)
    dev = flat.device
    u = _as_i32(user, dev).view(-1)
    i = _as_i32(item, dev).view(-1)
    if u.numel() != i.numel():
        raise ValueError("user and item must have the same number of elements")
    if u.numel():
        # nn.Embedding raises on an out-of-range id (models.py:98-103); the kernel
        # does not bound-check its gathers, so check here (one host sync).
        lo_hi = torch.stack([u.min(), u.max(), i.min(), i.max()]).tolist()
        if lo_hi[0] < 0 or lo_hi[1] >= model.user_num or lo_hi[2] < 0 or lo_hi[3] >= model.item_num:
            raise IndexError("index out of range in self")
    rows = pack_rows(u, i)
    if torch.is_grad_enabled() and any(p.requires_grad for p in model.ordered_params()):
        return _NCFFunction.apply(rows, model, *model.ordered_params())
    drop = _dropout_layout(model)  # train mode: nn.Dropout applies under no_grad too
    if drop is not None:
        return _dropout_logits(model, rows, drop)
    return forward_logits(flat, lay, rows, ws_owner=model)
