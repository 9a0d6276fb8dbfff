"""HR@K / NDCG@K leave-one-out evaluation (reference src/training/metrics.py:4-25).

``metrics(model, test_loader, top_k)`` keeps the reference signature and return
value (per-batch lists).  For a HIP-resident model it scores every candidate of
every batch with one forward launch and ranks all batches with one
``ncf_hr_ndcg`` launch (one wave per batch); the loader is still iterated
exactly once, so the torch generator consumption (one base_seed draw) is the
reference's.  For a CPU model it runs the reference's per-batch loop.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L


def _hr_ndcg_topk(logits, items, sizes, top_k):
    """Loaders ncf_hr_ndcg does not take (batches above 1024 rows, or of unequal
    sizes): the reference's per-batch ranking (metrics.py:10-22) with torch.topk on
    the device logits -- HR = gt in the top k, NDCG = 1 / log2(first hit + 2)."""
    hr, nd = [], []
    pos = 0
    for s in sizes:
        if top_k > s:
            raise RuntimeError("selected index k out of range")  # torch.topk's error (metrics.py:13)
        pred, item = logits[pos:pos + s], items[pos:pos + s]
        _, idx = torch.topk(pred, top_k)
        hit = torch.take(item, idx) == item[0]
        first = torch.argmax(hit.to(torch.int32))
        any_hit = hit.any()
        hr.append(any_hit.to(torch.int32))
        nd.append(torch.where(any_hit, 1.0 / torch.log2(first.to(torch.float64) + 2.0),
                              torch.zeros((), dtype=torch.float64, device=logits.device)))
        pos += s
    return torch.stack(hr), torch.stack(nd)


def _hr_ndcg_device(logits, items_i32, batch, top_k):
    n = items_i32.numel()
    nb = (n + batch - 1) // batch
    last = n - (nb - 1) * batch
    if top_k > last or top_k > batch:
        raise RuntimeError("selected index k out of range")  # torch.topk's error (metrics.py:13)
    if batch > 1024:  # beyond ncf_hr_ndcg's LDS staging
        return _hr_ndcg_topk(logits, items_i32, [batch] * (nb - 1) + [last], top_k)
    hr = torch.empty(nb, dtype=torch.int32, device=logits.device)
    nd = torch.empty(nb, dtype=torch.float32, device=logits.device)
    L.check(L.hip().ncf_hr_ndcg(logits.data_ptr(), items_i32.data_ptr(), n, int(batch), int(top_k),
                                hr.data_ptr(), nd.data_ptr(), L.stream_ptr(logits.device)), "ncf_hr_ndcg")
    return hr, nd


def evaluate_rows_device(model, rows, items_i32, batch, top_k):
    """Per-batch HR (int32) and NDCG (float32) on the device for a packed candidate
    stream whose ids the caller has checked; nothing is synchronised."""
    from . import ops
    flat, lay = ops.ensure_flat(model)
    with torch.no_grad():
        logits = ops.forward_logits(flat, lay, rows, ws_owner=model)
    return _hr_ndcg_device(logits, items_i32, batch, top_k)


def evaluate_arrays(model, users, items, batch, top_k, sizes=None):
    """HR/NDCG lists for a flat candidate stream cut into `batch`-row batches (or into
    the given batch `sizes`, a loader's unequal batches)."""
    from . import ops
    flat, lay = ops.ensure_flat(model)
    dev = flat.device
    ops.check_ids(users, items, model.user_num, model.item_num)  # nn.Embedding raises (models.py:108-112)
    u = torch.as_tensor(np.asarray(users), dtype=torch.int32).to(dev)
    i = torch.as_tensor(np.asarray(items), dtype=torch.int32).to(dev)
    with torch.no_grad():
        logits = ops.forward_logits(flat, lay, ops.pack_rows(u, i), ws_owner=model)
    if sizes is not None:
        hr, nd = _hr_ndcg_topk(logits, i, sizes, top_k)
    else:
        hr, nd = _hr_ndcg_device(logits, i, batch, top_k)
    return hr.cpu().tolist(), nd.double().cpu().tolist()


def metrics(model, test_loader, top_k):
    dev_model = model.embed_user_GMF.weight.is_cuda
    if not dev_model:
        return _metrics_cpu(model, test_loader, top_k)
    us, its, sizes = [], [], []
    for user, item, _ in test_loader:
        us.append(torch.as_tensor(user).view(-1))
        its.append(torch.as_tensor(item).view(-1))
        sizes.append(its[-1].numel())
    if not sizes:
        return [], []
    bs = sizes[0]
    ragged = any(s != bs for s in sizes[:-1]) or sizes[-1] > bs  # e.g. a batch_sampler: per-batch ranking
    if top_k > min(sizes):
        raise RuntimeError("selected index k out of range")
    HR, NDCG = evaluate_arrays(model, torch.cat(us), torch.cat(its), bs, top_k, sizes if ragged else None)
    return HR, [float(x) for x in NDCG]


def _metrics_cpu(model, test_loader, top_k):
    HR, NDCG = [], []
    for user, item, _ in test_loader:
        with torch.no_grad():
            predictions = model(user, item)
            _, indices = torch.topk(predictions, top_k)
            recommends = torch.take(item, indices).cpu().numpy()
        gt_item = item[0].item()
        HR.append(int(gt_item in recommends))
        ndcg = 0.0
        if gt_item in recommends:
            index = np.where(recommends == gt_item)[0][0]
            ndcg = 1.0 / np.log2(index + 2)
        NDCG.append(ndcg)
    return HR, NDCG
