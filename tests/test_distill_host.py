"""Distillation API on the CPU (config C5): ncf_amd.distill's reference-compatible
modules (src.distillation) evaluated with stock torch CPU ops against the
reference's own outputs (tests/golden/G8_distill.npz, make_golden_kd.py):
construction (adapter RNG order), loss, gradients, 5 Adam steps."""
import numpy as np
import pytest
import torch

CASES = {"c5": ((16, 3, "NeuMF-end"), (8, 2, "MLP")),
         "cli": ((32, 2, "NeuMF-end"), (16, 1, "NeuMF-end")),
         "same": ((8, 2, "GMF"), (8, 2, "GMF"))}


def build(case, strategy):
    from src.distillation import AttentionDistillation, FeatureDistillation, ResponseDistillation
    from src.ncf.models import NCF
    (tf, tl, tm), (sf, sl, sm) = CASES[case]
    torch.manual_seed(7)
    teacher = NCF(50, 80, tf, tl, 0.0, tm)
    student = NCF(50, 80, sf, sl, 0.0, sm)
    if strategy == "response":
        d = ResponseDistillation(teacher, student, temperature=2.0, alpha=0.5)
    elif strategy == "feature":
        d = FeatureDistillation(teacher, student, temperature=2.0, alpha=0.5, beta=0.3)
    else:
        d = AttentionDistillation(teacher, student, temperature=2.0, alpha=0.5, gamma=0.2)
    return teacher, student, d


@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("strategy", ["response", "feature", "attention"])
def test_distill_modules_match_reference_on_cpu(golden, case, strategy):
    g = golden("G8_distill")
    tag = f"{case}_{strategy}"
    teacher, student, d = build(case, strategy)
    for k, v in student.state_dict().items():
        assert np.array_equal(v.numpy(), g[f"{tag}::student0::{k}"]), k
    if strategy == "feature":
        for k, v in d.adaptation_layers.state_dict().items():
            assert np.array_equal(v.numpy(), g[f"{tag}::adapter::{k}"]), k
    assert all(not p.requires_grad for p in teacher.parameters())
    opt = torch.optim.Adam(student.parameters(), lr=1e-3)
    losses = []
    for s in range(5):
        opt.zero_grad()
        loss = d(torch.from_numpy(g["users"][s]), torch.from_numpy(g["items"][s]), torch.from_numpy(g["labels"][s]))
        loss.backward()
        if s == 0:
            for k, p in student.named_parameters():
                key = f"{tag}::grad0::{k}"
                assert (p.grad is not None) == (key in g.files), k
        opt.step()
        losses.append(loss.item())
    np.testing.assert_allclose(losses, g[f"{tag}::losses"], rtol=1e-6)
    for k, v in student.state_dict().items():
        np.testing.assert_allclose(v.numpy(), g[f"{tag}::student_t5::{k}"], rtol=1e-5, atol=1e-7, err_msg=k)


def test_unified_is_exported_and_combines_terms():
    """scripts/train_student.py imports UnifiedDistillation (empty in the reference):
    it must construct and reduce to feature distillation when gamma = 0."""
    from src.distillation import FeatureDistillation, UnifiedDistillation
    from src.ncf.models import NCF
    torch.manual_seed(3)
    t, s = NCF(30, 40, 16, 3, 0.0, "NeuMF-end"), NCF(30, 40, 8, 2, 0.0, "MLP")
    uni = UnifiedDistillation(t, s, temperature=2.0, alpha=0.5, beta=0.3, gamma=0.0)
    torch.manual_seed(3)
    t2, s2 = NCF(30, 40, 16, 3, 0.0, "NeuMF-end"), NCF(30, 40, 8, 2, 0.0, "MLP")
    fea = FeatureDistillation(t2, s2, temperature=2.0, alpha=0.5, beta=0.3)
    u, i = torch.arange(30) % 30, torch.arange(30) % 40
    y = (torch.arange(30) % 3 == 0).float()
    np.testing.assert_allclose(uni(u, i, y).item(), fea(u, i, y).item(), rtol=1e-6)
