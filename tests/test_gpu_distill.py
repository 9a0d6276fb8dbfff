"""Distillation on the GPU (config C5) against the reference's outputs
(tests/golden/G8_distill.npz):
  * the fused device plan -- TrainEngine(distill=module.device_plan()): teacher
    logits of the stream by ncf_forward, ncf_train_step_kd (BCE + response term in
    the student's fused step), ncf_kd_feature_step (adapted GMF / MLP-input
    features), reduce + Adam -- over 5 steps: per-step loss rtol 1e-5, student
    parameters rtol 1e-4 / atol 1e-6 (fp32 summation order differs);
  * the module API (loss = module(user, item, label); loss.backward()) with both
    models on the device: loss rtol 1e-5, gradients rtol 1e-4 + atol 1e-6 * max|g|.
The attention term is identically zero in exact arithmetic (ncf_amd/distill.py);
its reference value (~1e-16) is inside the loss tolerance."""
import numpy as np
import pytest
import torch

from test_distill_host import build

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("case", ["c5", "cli"])
@pytest.mark.parametrize("strategy", ["response", "feature", "attention"])
@pytest.mark.parametrize("use_graph", [False, True])
def test_device_plan_trajectory_vs_reference(golden, case, strategy, use_graph):
    from ncf_amd import ops
    from ncf_amd.engine import TrainEngine
    g = golden("G8_distill")
    tag = f"{case}_{strategy}"
    teacher, student, d = build(case, strategy)
    teacher.to(DEV)
    student.to(DEV)
    d.to(DEV)
    eng = TrainEngine(student, lr=1e-3, distill=d.device_plan())
    rows = ops.pack_rows_host(g["users"].reshape(-1), g["items"].reshape(-1), g["labels"].reshape(-1))
    eng.set_epoch_stream(torch.as_tensor(rows, device=DEV), 256)
    eng.run(5, use_graph=use_graph)
    torch.cuda.synchronize()
    np.testing.assert_allclose(eng.epoch_losses()[:5], g[f"{tag}::losses"], rtol=1e-5)
    for k, v in student.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), g[f"{tag}::student_t5::{k}"], rtol=1e-4, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("strategy", ["response", "feature", "attention"])
def test_module_api_on_device_vs_reference(golden, strategy):
    g = golden("G8_distill")
    tag = f"c5_{strategy}"
    teacher, student, d = build("c5", strategy)
    teacher.to(DEV)
    student.to(DEV)
    d.to(DEV)
    u = torch.from_numpy(g["users"][0]).to(DEV)
    i = torch.from_numpy(g["items"][0]).to(DEV)
    y = torch.from_numpy(g["labels"][0]).to(DEV)
    loss = d(u, i, y)
    loss.backward()
    np.testing.assert_allclose(loss.item(), float(g[f"{tag}::loss0"]), rtol=1e-5)
    for k, p in student.named_parameters():
        key = f"{tag}::grad0::{k}"
        if key in g.files and p.grad is not None:
            exp = g[key]
            if float(np.abs(exp).max()) < 1e-12:
                # an identically-zero gradient (the attention term's): both sides are
                # rounding noise of order 1e-18
                assert float(p.grad.abs().max()) < 1e-12, k
                continue
            np.testing.assert_allclose(p.grad.cpu().numpy(), exp, rtol=1e-4,
                                       atol=1e-6 * max(float(np.abs(exp).max()), 1e-30), err_msg=k)


def test_feature_plan_rejects_matched_tower_features():
    teacher, student, d = build("same", "feature")
    teacher.to(DEV)
    student.to(DEV)
    with pytest.raises(NotImplementedError):
        d.device_plan()
