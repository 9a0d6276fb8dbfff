"""The reference-side binding documented in INTEGRATION.md section 2, executed as
written (its ```python blocks, with only the library path filled in), on a C3
batch against the oracle and on the C5 feature-distillation case against the
reference's own outputs (G8).  Reference: src/ncf/models.py:97-118,
scripts/train_neumf.py:111-115, src/distillation/feature.py:125-147."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _binding():
    """exec the INTEGRATION.md section-2 code blocks in one namespace."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text.split("## 2.", 1)[1].split("\n## 3.", 1)[0]
    blocks = re.findall(r"```python\n(.*?)```", sec, re.S)
    assert len(blocks) == 4, ("INTEGRATION.md section 2 must hold the train, in-step-Adam, distill and "
                              "deferred-Adam stubs")
    lib = os.path.join(ROOT, "ncf_amd", "libncf_hip.so")
    ns = {}
    for b in blocks:
        exec(compile(b.replace("/path/to/ncf_amd/libncf_hip.so", lib), "INTEGRATION.md", "exec"), ns)
    return ns


def _ranges(model, lay, extra=None):
    from ncf_amd.engine import _active_ranges
    r = _active_ranges(model, lay, extra)
    return (ctypes.c_int64 * (2 * len(r)))(*[x for q in r for x in q])


def test_documented_train_step_on_c3_batch_vs_oracle():
    from ncf_amd import ops
    from ncf_amd.models import NCF
    ns = _binding()
    U, I, f, Lyr, B = 6041, 3707, 16, 3, 65536
    torch.manual_seed(5)
    ref = O.OracleNCF(U, I, f, Lyr, 0.0, "NeuMF-end")
    torch.manual_seed(5)
    m = NCF(U, I, f, Lyr, 0.0, "NeuMF-end").to(DEV)
    flat, _ = ops.ensure_flat(m)          # parameters as views of one flat buffer
    lay = ns["layout"](m)
    rng = np.random.default_rng(17)
    users = rng.integers(0, U, B)
    items = np.minimum(rng.zipf(1.3, B) - 1, I - 1)
    labels = (rng.random(B) < 0.2).astype(np.int64)
    u = torch.as_tensor(users, device=DEV)
    it = torch.as_tensor(items, device=DEV)
    y = torch.as_tensor(labels, device=DEV)
    rows = ns["pack"](u, it, y)
    ops.check_rows(rows, U, I)  # the packed ids must be the inputs (IndexError, not a fault, if not)
    assert np.array_equal(rows.cpu().numpy(), ops.pack_rows_host(users, items, labels))
    with torch.no_grad():
        lg_ref = ref(torch.from_numpy(users), torch.from_numpy(items)).numpy()
    got = ns["forward"](flat, lay, rows)
    np.testing.assert_allclose(got.cpu().numpy(), lg_ref, rtol=1e-5, atol=1e-7)
    grads = torch.zeros(int(lay.total), device=DEV)
    mom = torch.zeros_like(grads)
    vel = torch.zeros_like(grads)
    ctl = torch.tensor([0, 0, B, 0, 0, 0], dtype=torch.int64, device=DEV)
    ws = ns["workspace"](ns["_lib"].ncf_workspace_bytes(ctypes.byref(lay), B), DEV)
    ns["train_step"](flat, grads, mom, vel, lay, rows, ctl, ws, B, _ranges(m, lay))
    torch.cuda.synchronize()
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    O.train_steps(ref, opt, [users], [items], [labels])
    # one Adam step: lr * g / (|g| + eps) -- parameters to rtol 1e-5 plus 5e-3 * lr
    # absolute (a gradient within ~eps of zero turns summation-order noise into
    # parameter movement; see __graft_entry__.smoke)
    for (k, v), (_, r) in zip(m.state_dict().items(), ref.state_dict().items()):
        np.testing.assert_allclose(v.cpu().numpy(), r.numpy(), rtol=1e-5, atol=5e-6, err_msg=k)
    assert ctl.cpu().tolist()[:2] == [1, 1]


def test_documented_distill_step_vs_reference(golden):
    from test_distill_host import build
    from ncf_amd import ops
    ns = _binding()
    g = golden("G8_distill")
    teacher, student, d = build("cli", "feature")
    teacher.to(DEV)
    student.to(DEV)
    d.to(DEV)
    plan = d.device_plan()
    s_flat, _ = ops.ensure_flat(student)
    t_flat, _ = ops.ensure_flat(teacher)
    s_lay, t_lay = ns["layout"](student), ns["layout"](teacher)
    (gw, gb, gc), (mw, mb, mc) = plan.keys["gmf_features"], plan.keys["mlp_input"]
    assert abs(gc - 0.3 / 2) < 1e-12 and abs(mc - 0.3 / 2) < 1e-12  # beta / count, as the stub assumes
    B = g["users"].shape[1]
    rows = torch.as_tensor(ops.pack_rows_host(g["users"].reshape(-1), g["items"].reshape(-1),
                                              g["labels"].reshape(-1)), device=DEV)
    tlog = ns["forward"](t_flat, t_lay, rows)   # teacher logits of the stream, once
    grads = torch.zeros(int(s_lay.total), device=DEV)
    mom = torch.zeros_like(grads)
    vel = torch.zeros_like(grads)
    ctl = torch.tensor([0, 0, rows.numel(), 0, 0, 0], dtype=torch.int64, device=DEV)
    ws = ns["workspace"](ns["_lib"].ncf_workspace_bytes(ctypes.byref(s_lay), B), DEV)
    rng = _ranges(student, ops.ensure_flat(student)[1], plan.active_extra)
    for _ in range(5):
        ns["distill_step"](s_flat, grads, mom, vel, s_lay, t_flat, t_lay, rows, tlog, ctl, ws, B, rng,
                           alpha=0.5, T=2.0, beta=0.3, gmf_adapter=(gw, gb), mlp_adapter=(mw, mb))
    torch.cuda.synchronize()
    for k, v in student.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), g[f"cli_feature::student_t5::{k}"], rtol=1e-4, atol=1e-6,
                                   err_msg=k)


def test_documented_deferred_adam_steps_vs_oracle():
    """The section-2 deferred-Adam stub (ncf_batch_touched, ncf_lazy_adam_step,
    ncf_lazy_adam_flush) on a C2-shaped stream (ml-1m ids, bs 1,024: each batch
    touches a fraction of the rows): 6 steps, flushed, vs 6 steps of the oracle's
    torch.optim.Adam on the same batches."""
    from ncf_amd import ops
    from ncf_amd.models import NCF
    ns = _binding()
    U, I, f, Lyr, B, T = 6041, 3707, 8, 3, 1024, 6
    torch.manual_seed(9)
    ref = O.OracleNCF(U, I, f, Lyr, 0.0, "NeuMF-end")
    torch.manual_seed(9)
    m = NCF(U, I, f, Lyr, 0.0, "NeuMF-end").to(DEV)
    flat, _ = ops.ensure_flat(m)
    lay = ns["layout"](m)
    ns["_lib"].ncf_layout_tune(ctypes.byref(lay), B)
    rng = np.random.default_rng(23)
    n = B * T
    users = rng.integers(1, U, n)
    items = np.minimum(rng.zipf(1.3, n), I - 1)
    labels = (rng.random(n) < 0.2).astype(np.int64)
    rows = ns["pack"](torch.as_tensor(users, device=DEV), torch.as_tensor(items, device=DEV),
                      torch.as_tensor(labels, device=DEV))
    touched = ns["touched_lists"](rows, B, lay)
    last, ring = ns["lazy_state"](lay, DEV)
    grads = torch.zeros(int(lay.total), device=DEV)
    mom, vel = torch.zeros_like(grads), torch.zeros_like(grads)
    ctl = torch.tensor([0, 0, n, 0, 0, 0], dtype=torch.int64, device=DEV)
    ws = ns["workspace"](ns["_lib"].ncf_workspace_bytes(ctypes.byref(lay), B), DEV)
    rg = _ranges(m, lay)
    for _ in range(T - 1):  # stop before the epoch's last batch: rows left behind until the flush
        ns["train_step_lazy"](flat, grads, mom, vel, lay, rows, ctl, ws, B, rg, touched, last, ring)
    ns["flush"](flat, grads, mom, vel, lay, ctl, rg, last, ring)
    torch.cuda.synchronize()
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    O.train_steps(ref, opt, [users[k * B:(k + 1) * B] for k in range(T - 1)],
                  [items[k * B:(k + 1) * B] for k in range(T - 1)], [labels[k * B:(k + 1) * B] for k in range(T - 1)])
    for (k, v), (_, r) in zip(m.state_dict().items(), ref.state_dict().items()):
        np.testing.assert_allclose(v.cpu().numpy(), r.numpy(), rtol=1e-4, atol=2e-5, err_msg=k)
    assert ctl.cpu().tolist()[:2] == [T - 1, T - 1]
    assert int(last.min()) == T - 1 and float(grads.abs().max()) == 0.0


def test_documented_in_step_adam_steps_vs_oracle():
    """The section-2 in-step-Adam stub (ncf_ais_begin, ncf_train_step_ais, ncf_ais_bump,
    ncf_ais_flush) on a C2-shaped stream (ml-1m ids, bs 1,024): 6 steps in one chunk,
    flushed, vs 6 steps of the oracle's torch.optim.Adam on the same batches."""
    from ncf_amd import ops
    from ncf_amd.models import NCF
    ns = _binding()
    U, I, f, Lyr, B, T = 6041, 3707, 8, 3, 1024, 6
    torch.manual_seed(9)
    ref = O.OracleNCF(U, I, f, Lyr, 0.0, "NeuMF-end")
    torch.manual_seed(9)
    m = NCF(U, I, f, Lyr, 0.0, "NeuMF-end").to(DEV)
    flat, _ = ops.ensure_flat(m)
    lay = ns["layout"](m)
    ns["_lib"].ncf_layout_tune(ctypes.byref(lay), B)
    assert ns["_lib"].ncf_ais_supported(ctypes.byref(lay)) == 1
    rng = np.random.default_rng(29)
    n = B * T
    users = rng.integers(0, U, n)
    items = np.minimum(rng.zipf(1.3, n) - 1, I - 1)
    labels = (rng.random(n) < 0.2).astype(np.int64)
    rows = ns["pack"](torch.as_tensor(users, device=DEV), torch.as_tensor(items, device=DEV),
                      torch.as_tensor(labels, device=DEV))
    grads = torch.zeros(int(lay.total), device=DEV)
    mom, vel = torch.zeros_like(grads), torch.zeros_like(grads)
    ctl = torch.tensor([0, 0, n, 0, 0, 0], dtype=torch.int64, device=DEV)
    keep, bufs = ns["ais_buffers"](lay, DEV)
    ns["train_steps_ais"](flat, grads, mom, vel, lay, rows, ctl, B, _ranges(m, lay), bufs, T)
    torch.cuda.synchronize()
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    O.train_steps(ref, opt, [users[k * B:(k + 1) * B] for k in range(T)],
                  [items[k * B:(k + 1) * B] for k in range(T)], [labels[k * B:(k + 1) * B] for k in range(T)])
    for (k, v), (_, r) in zip(m.state_dict().items(), ref.state_dict().items()):
        np.testing.assert_allclose(v.cpu().numpy(), r.numpy(), rtol=1e-4, atol=2e-5, err_msg=k)
    assert ctl.cpu().tolist()[:2] == [T, T]
    del keep
