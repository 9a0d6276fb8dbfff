"""The reference's own scripts, unchanged, against this repo's ``src/`` import
surface (CPU, in this container only: /root/reference is absent elsewhere and
the tests skip there).  SURVEY.md section 8(c) allows running the reference here
to validate; nothing of it is copied.

* scripts/train_neumf.py   (NCF, NCFData, load_all, config, metrics)
* scripts/evaluate_models.py  (src.ncf.nmf_model.run_nmf_experiment, which the
  reference itself lacks, then metrics at several K and test batch sizes up to the
  point where the reference's own metrics() raises)
* the NMF baseline classes against the reference's src/ncf/nmf_model.py."""
import importlib.util
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present (GPU box)")


@pytest.fixture
def tiny_dir(tmp_path):
    from ncf_amd import synthetic
    ds = synthetic.make_dataset("tiny", seed=3)
    synthetic.write_reference_files(ds, str(tmp_path / "data" / "processed"))
    return tmp_path, ds


def _run(script, cwd, *args, timeout=600):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT  # this repo's src/ and ncf_amd/ first; the script appends the reference root
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    return subprocess.run([sys.executable, os.path.join(REF, "scripts", script), *args], cwd=str(cwd), env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_reference_train_neumf_runs_on_our_src(tiny_dir):
    cwd, _ = tiny_dir
    out = _run("train_neumf.py", cwd, "--epochs", "2", "--num_layers", "2")
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("Epoch ")]
    assert len(lines) == 2 and "Loss=" in lines[0] and "HR=" in lines[0] and "NDCG=" in lines[0]
    assert "Best Result:" in out.stdout
    assert list((cwd / "results" / "models").glob("NeuMF_*_2l_32f_best.pth"))


def test_reference_evaluate_models_runs_on_our_src(tiny_dir):
    """On the reference itself the script dies at import (no run_nmf_experiment).
    With this src/ it loads the checkpoint, runs and plots the Top-K sweep, then
    stops exactly where the reference's own metrics() would: the negative-sampling
    sweep evaluates DataLoader batches of num_neg + 1 = 2 rows at top_k = 10, and
    torch.topk raises "selected index k out of range" (metrics.py:13,
    evaluate_models.py:39-45).  Same error, same point: parity, not a fix."""
    import torch
    from ncf_amd.models import NCF
    cwd, ds = tiny_dir
    (cwd / "results" / "models").mkdir(parents=True, exist_ok=True)
    torch.manual_seed(0)
    m = NCF(ds["user_num"], ds["item_num"], 32, 2, 0.0, "NeuMF-end")
    torch.save(m.state_dict(), cwd / "results" / "models" / "NeuMF-end_pretrain_best.pth")
    out = _run("evaluate_models.py", cwd)
    for s in ("Loaded model from", "Evaluating Top-K performance", "Saved Top-K performance plot",
              "Evaluating with 1 negative samples..."):
        assert s in out.stdout, s
    assert (cwd / "results" / "figures" / "neumf_top_k_performance.png").exists()
    assert out.returncode != 0 and "selected index k out of range" in out.stderr


def test_reference_metrics_raise_like_ours():
    """The reference's metrics() on a 2-row batch with top_k=10 raises the same
    error ours does (run on the reference's own function, CPU)."""
    import torch
    spec = importlib.util.spec_from_file_location("ref_metrics", os.path.join(REF, "src", "training", "metrics.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    from ncf_amd.metrics import metrics
    from ncf_amd.models import NCF
    torch.manual_seed(0)
    m = NCF(10, 20, 8, 2, 0.0, "NeuMF-end")
    loader = [(torch.tensor([1, 1]), torch.tensor([3, 4]), torch.tensor([0, 0]))]
    for fn in (mod.metrics, metrics):
        with pytest.raises(RuntimeError, match="k out of range"):
            fn(m, loader, 10)


def _reference_nmf_module():
    spec = importlib.util.spec_from_file_location("ref_nmf_model", os.path.join(REF, "src", "ncf", "nmf_model.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_nmf_baseline_matches_reference_classes(tiny_dir):
    import scipy.sparse as sp
    from ncf_amd import nmf
    _, ds = tiny_dir
    ref = _reference_nmf_module()
    U, I = ds["user_num"], ds["item_num"]
    mat = sp.dok_matrix((U, I), dtype=np.float32)
    for u, i in zip(ds["train_users"], ds["train_items"]):
        mat[int(u), int(i)] = 1.0
    test = []
    for u, p, negs in zip(ds["test_users"], ds["test_items"], ds["test_negatives"]):
        test.append([int(u), int(p)])
        test += [[int(u), int(n)] for n in negs]
    for n in (1, 6):
        a = ref.NMFRecommender(n_components=n, random_state=43, max_iter=200).fit(mat)
        b = nmf.NMFRecommender(n_components=n, random_state=43, max_iter=200).fit(mat)
        uu, ii = np.array([0, 3, U - 1, U + 5]), np.array([1, 0, I - 1, 2])
        np.testing.assert_allclose(b.predict(uu, ii), a.predict(uu, ii), rtol=1e-6)  # float32 factors, dot order
        assert b.get_n_parameters() == a.get_n_parameters()
        assert nmf.NMFEvaluator(b, test, mat).evaluate() == pytest.approx(ref.NMFEvaluator(a, test, mat).evaluate())
    res = nmf.run_nmf_experiment(mat, test, [1, 6], num_runs=2, max_iter=100)
    assert set(res) == {1, 6} and set(res[1]) >= {"hr_mean", "hr_std", "ndcg_mean", "ndcg_std", "parameters"}
    assert res[6]["parameters"] == (U + I) * 6
