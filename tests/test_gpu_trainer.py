"""End-to-end parity of Trainer.fit() / scripts/train_neumf.py against the
reference's own scripts/train_neumf.py (tests/golden/G7_script.npz: seeded,
2 epochs, NCF(944, 1683, 8, 3) on the ml-100k-shaped synthetic files).

Same seeds -> same negatives (bit-exact), same batches (bit-exact), same init
(bit-exact); the fp32 trajectory differs only in summation order, so per-epoch
loss must agree to 1e-3 relative and HR@10 / NDCG@10 within 0.01 (SURVEY.md
8(d) parity gate)."""
import os
import re
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _parse(lines):
    out = []
    for ln in lines:
        m = re.match(r"Epoch (\d+): Loss=([\d.]+), HR=([\d.]+), NDCG=([\d.]+)", str(ln))
        if m:
            out.append((int(m.group(1)), float(m.group(2)), float(m.group(3)), float(m.group(4))))
    return out


@pytest.fixture()
def ml100k_dir(tmp_path, monkeypatch):
    from ncf_amd import synthetic
    monkeypatch.chdir(tmp_path)
    synthetic.write_reference_files(synthetic.make_dataset("ml-100k", seed=0), "data/processed")
    return tmp_path


def test_trainer_matches_reference_script(golden, ml100k_dir):
    import torch.utils.data as data
    from ncf_amd.data import NCFData, load_all
    from ncf_amd.models import NCF
    from ncf_amd.trainer import Trainer
    g = golden("G7_script")
    ref = _parse(g["f8_L3_stdout"])
    np.random.seed(0)
    torch.manual_seed(0)
    train_data, test_data, U, I, mat = load_all()
    train_ds = NCFData(train_data, I, mat, 4, True)
    test_ds = NCFData(test_data, I, mat, 0, False)
    loader = data.DataLoader(test_ds, batch_size=100, shuffle=False, num_workers=0)
    model = NCF(U, I, 8, 3, 0.0, "NeuMF-end").to("cuda:0")
    tr = Trainer(model, train_ds, loader, batch_size=256, lr=1e-3, top_k=10)
    t0 = time.time()
    res = tr.fit(2)
    wall = time.time() - t0
    assert res["parameters"] == 107841
    # Time= of each epoch runs from its start to the end of its metrics pass: the
    # epochs follow each other, so the times do not overlap and sum to at most fit()
    assert all(h["time"] > 0 for h in tr.history)
    assert sum(h["time"] for h in tr.history) <= wall, (tr.history, wall)
    for h, (e, l, hr, nd) in zip(tr.history, ref):
        assert h["epoch"] == e
        assert abs(h["loss"] - l) <= 1e-3 * l + 1e-4, (tr.history, ref)
        assert abs(h["hr"] - hr) <= 0.01 and abs(h["ndcg"] - nd) <= 0.01, (tr.history, ref)


def test_script_stdout_matches_reference(golden, ml100k_dir):
    g = golden("G7_script")
    ref = _parse(g["f8_L3_stdout"])
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "train_neumf.py"), "--epochs", "2",
                          "--factor_num", "8", "--num_layers", "3", "--seed", "0"],
                         capture_output=True, text=True, timeout=600, cwd=str(ml100k_dir))
    assert out.returncode == 0, out.stderr[-2000:]
    got = _parse(out.stdout.splitlines())
    assert len(got) == 2, out.stdout
    for (e1, l1, h1, n1), (e2, l2, h2, n2) in zip(got, ref):
        assert e1 == e2
        assert abs(l1 - l2) <= 1e-3 * l2 + 1e-4, (got, ref)
        assert abs(h1 - h2) <= 0.01 and abs(n1 - n2) <= 0.01, (got, ref)
    assert "Parameters: 107841" in out.stdout and "--- RESULTS ---" in out.stdout
    assert os.path.exists(os.path.join(str(ml100k_dir), "results", "models", "NeuMF_end_3l_8f_best.pth"))


def _parse_student(lines):
    out = []
    for ln in lines:
        m = re.match(r"(\d+) - Loss: ([\d.]+), HR: ([\d.]+), NDCG: ([\d.]+)", str(ln))
        if m:
            out.append((int(m.group(1)), float(m.group(2)), float(m.group(3)), float(m.group(4))))
    return out


@pytest.mark.parametrize("strategy", ["response", "feature"])
def test_student_script_matches_reference_loop(golden, ml100k_dir, strategy):
    """scripts/train_student.py (config C5 shapes: teacher NCF(16,3) -> student
    NCF(8,2,MLP)) against the reference's train_student loop run with the
    reference's own objects (tests/golden/G9_student_loop.npz): same seeds, same
    negatives/batches/init, loss within 1e-3 relative, HR/NDCG within 0.01."""
    from ncf_amd.data import load_all
    from ncf_amd.models import NCF
    g = golden("G9_student_loop")
    ref = _parse_student(g[f"{strategy}_stdout"])
    _, _, U, I, _ = load_all()
    torch.manual_seed(123)  # the teacher checkpoint the golden run loaded
    sd = NCF(U, I, 16, 3, 0.0, "NeuMF-end").state_dict()
    os.makedirs("results/models", exist_ok=True)
    torch.save(sd, "results/models/teacher_NeuMF-end_best.pth")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "train_student.py"), "--epochs", "1",
                          "--factor_num", "8", "--num_layers", "2", "--student_model", "MLP",
                          "--teacher_model", "NeuMF-end", "--distillation", strategy, "--seed", "0"],
                         capture_output=True, text=True, timeout=600, cwd=str(ml100k_dir))
    assert out.returncode == 0, out.stderr[-2000:]
    got = _parse_student(out.stdout.splitlines())
    assert len(got) == 1, out.stdout[-2000:]
    (e1, l1, h1, n1), (e2, l2, h2, n2) = got[0], ref[0]
    assert e1 == e2
    assert abs(l1 - l2) <= 1e-3 * l2, (got, ref)
    assert abs(h1 - h2) <= 0.01 and abs(n1 - n2) <= 0.01, (got, ref)
    assert "End. Best epoch 000" in out.stdout
    assert os.path.exists(os.path.join(str(ml100k_dir), "results", "models", "student_MLP_best.pth"))


def test_teacher_script_runs(ml100k_dir):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "train_teacher.py"), "--epochs", "1",
                          "--factor_num", "16", "--num_layers", "3", "--seed", "0"],
                         capture_output=True, text=True, timeout=600, cwd=str(ml100k_dir))
    assert out.returncode == 0, out.stderr[-2000:]
    assert re.search(r"Epoch 001: Loss=[\d.]+, HR=[\d.]+, NDCG=[\d.]+, Time=\d\d:\d\d:\d\d", out.stdout), out.stdout
    assert re.search(r"Best Epoch 000: Loss=", out.stdout), out.stdout
    assert os.path.exists(os.path.join(str(ml100k_dir), "results", "models", "teacher_NeuMF-end_best.pth"))


def test_pretrain_chain_matches_reference(golden, ml100k_dir):
    """The NeuMF-pre chain (tests/golden/G11_pretrain_chain.npz, the reference's own
    run): scripts/pretrain.py GMF -> MLP -> scripts/train_neumf.py --model NeuMF-pre
    --pretraining, which loads both checkpoints (models.py:48-95) and trains with
    SGD(lr * 10) (train_neumf.py:62-90).  Each run seeded 0 like the golden; epoch
    lines within G7's tolerances (loss 1e-3 relative, HR/NDCG 0.01), the same
    checkpoint files, the same parameter counts and loading messages."""
    g = golden("G11_pretrain_chain")
    runs = [("gmf", "pretrain.py", ["--model", "GMF", "--epochs", "2", "--factor_num", "8"]),
            ("mlp", "pretrain.py", ["--model", "MLP", "--epochs", "2", "--factor_num", "8", "--num_layers", "3"]),
            ("neumf_pre", "train_neumf.py", ["--model", "NeuMF-pre", "--pretraining", "--epochs", "2",
                                             "--factor_num", "8", "--num_layers", "3"])]
    models = os.path.join(str(ml100k_dir), "results", "models")
    for tag, script, args in runs:
        before = set(os.listdir(models)) if os.path.isdir(models) else set()
        out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", script)] + args + ["--seed", "0"],
                             capture_output=True, text=True, timeout=600, cwd=str(ml100k_dir))
        assert out.returncode == 0, out.stderr[-2000:]
        ref_lines = [str(x) for x in g[f"{tag}_stdout"]]
        got, ref = _parse(out.stdout.splitlines()), _parse(ref_lines)
        assert len(got) == len(ref) == 2, (tag, out.stdout[-2000:])
        for (e1, l1, h1, n1), (e2, l2, h2, n2) in zip(got, ref):
            assert e1 == e2
            assert abs(l1 - l2) <= 1e-3 * l2 + 1e-4, (tag, got, ref)
            assert abs(h1 - h2) <= 0.01 and abs(n1 - n2) <= 0.01, (tag, got, ref)
        for ln in ref_lines:
            if ln.startswith(("Parameters:", "Model parameters:", "Loading pretrained", "Pretrained weights loaded",
                              "Pretraining:")):
                assert ln in out.stdout, (tag, ln)
        new = sorted(set(os.listdir(models)) - before)
        assert new == [str(x) for x in g[f"{tag}_checkpoints"]], (tag, new)
