#!/usr/bin/env python3
"""Generate golden vectors for the NeuMF hot path by running the REFERENCE itself.

Run in the build container only (``/root/reference`` does not exist on the GPU
box):  ``python tests/golden/make_golden.py``.  It copies the read-only
reference into a scratch directory (its ``Config`` singleton needs a writable,
cwd-relative ``configs/`` + ``results/``; src/utils/config.py:5,53-58,65),
imports ``src.ncf.models.NCF``, ``src.data.datasets.NCFData`` and
``src.training.metrics.metrics`` from there, seeds numpy/torch, and writes
small ``.npz`` fixtures next to this script.  Only inputs and the reference's
outputs are stored -- no reference source text.

Fixture map (names follow SURVEY.md section 8c):
  G1_negatives.npz   NCFData.ng_sample()            (datasets.py:53-69)
  G2_shuffle.npz     DataLoader(shuffle=True) order (train_neumf.py:55-56)
  G3_init.npz        NCF.__init__/_init_weight      (models.py:5-46)
  G4_fwd_bwd.npz     forward/BCE/backward           (models.py:97-118, train_neumf.py:86,112-114)
  G5_steps.npz       Adam / SGD trajectories        (train_neumf.py:87-90,111-115)
  G6_metrics.npz     metrics()                      (metrics.py:4-25)
"""
import hashlib
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
MODEL_TYPES = ["GMF", "MLP", "NeuMF-end", "NeuMF-pre"]


def _import_reference():
    work = tempfile.mkdtemp(prefix="ncf_ref_")
    dst = os.path.join(work, "ref")
    shutil.copytree(REF, dst, ignore=shutil.ignore_patterns(".git", "results"))
    for root, dirs, files in os.walk(dst):
        os.chmod(root, 0o755)
    os.chdir(dst)
    sys.path.insert(0, dst)
    import torch  # noqa: F401
    from src.ncf.models import NCF
    from src.data.datasets import NCFData
    from src.training.metrics import metrics
    return NCF, NCFData, metrics


def sha(arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def random_positives(rng, n_users, n_items, per_user_lo, per_user_hi):
    """Random (u, i) training positives, file order = by user, like u.train.rating."""
    pairs = []
    for u in range(n_users):
        k = int(rng.integers(per_user_lo, per_user_hi + 1))
        items = rng.choice(n_items, size=k, replace=False)
        for i in items:
            pairs.append([u, int(i)])
    return np.asarray(pairs, dtype=np.int64)


def dok_from(pairs, n_users, n_items):
    import scipy.sparse as sp
    m = sp.dok_matrix((n_users, n_items), dtype=np.float32)
    for u, i in pairs.tolist():
        m[u, i] = 1.0
    return m


def g1_negatives(NCFData):
    out = {}
    # Toy known-answer case quoted in SURVEY.md 8(a) row a10.
    toy = np.array([[0, 1], [0, 2], [1, 0], [2, 3]], dtype=np.int64)
    np.random.seed(0)
    ds = NCFData(toy.tolist(), 5, dok_from(toy, 3, 5), 4, True)
    ds.ng_sample()
    out["toy_pos"] = toy
    out["toy_num_item"] = np.int64(5)
    out["toy_neg_seed0"] = np.asarray(ds.features_ng, dtype=np.int64)[:, 1]

    # Dense-ish small set (many rejections) and an ml-100k-shaped set.
    rng = np.random.default_rng(12345)
    small = random_positives(rng, 40, 30, 5, 25)          # up to 83% density -> rejection-heavy
    out["small_pos"] = small
    out["small_num_item"] = np.int64(30)
    for seed in (0, 1):
        np.random.seed(seed)
        ds = NCFData(small.tolist(), 30, dok_from(small, 40, 30), 4, True)
        ds.ng_sample()
        f = np.asarray(ds.features_ng, dtype=np.int64)
        assert (f[:, 0] == np.repeat(small[:, 0], 4)).all()
        out[f"small_neg_seed{seed}"] = f[:, 1].astype(np.int16)
        # the full fill (positives then negatives) and labels
        assert len(ds.features_fill) == len(small) * 5
        assert ds.labels_fill == [1] * len(small) + [0] * len(small) * 4

    rng = np.random.default_rng(100)
    big = random_positives(rng, 943, 1682, 20, 150)       # ml-100k-shaped
    out["big_pos"] = big.astype(np.int32)
    out["big_num_item"] = np.int64(1682)
    np.random.seed(0)
    ds = NCFData(big.tolist(), 1682, dok_from(big, 943, 1682), 4, True)
    ds.ng_sample()
    f = np.asarray(ds.features_ng, dtype=np.int64)[:, 1].astype(np.int32)
    out["big_neg_seed0_sha256"] = np.array(sha([f]))
    out["big_neg_seed0_head"] = f[:4096]
    np.savez_compressed(os.path.join(HERE, "G1_negatives.npz"), **out)


class _IdxData:
    """Dataset whose item i is (i, i, i%2): the loader order is then readable."""

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return i, i, i % 2


def g2_shuffle():
    import torch
    import torch.utils.data as data
    out = {}
    for seed in (0, 7):
        for n, bs in ((1000, 64), (257, 256)):
            torch.manual_seed(seed)
            train = data.DataLoader(_IdxData(n), batch_size=bs, shuffle=True, num_workers=0)
            test = data.DataLoader(_IdxData(300), batch_size=100, shuffle=False, num_workers=0)
            for ep in range(2):
                order = []
                sizes = []
                for u, i, lab in train:
                    order.extend(u.tolist())
                    sizes.append(len(u))
                    assert u.dtype == torch.int64 and lab.dtype == torch.int64
                out[f"s{seed}_n{n}_ep{ep}"] = np.asarray(order, dtype=np.int32)
                out[f"s{seed}_n{n}_ep{ep}_sizes"] = np.asarray(sizes, dtype=np.int32)
                for _ in test:                    # metrics() pass: one more base_seed draw
                    pass
            # a "script" with 4 workers consumes the generator identically (checked here on 1 epoch)
            torch.manual_seed(seed)
            train4 = data.DataLoader(_IdxData(n), batch_size=bs, shuffle=True, num_workers=2)
            order = []
            for u, _, _ in train4:
                order.extend(u.tolist())
            assert order == out[f"s{seed}_n{n}_ep0"].tolist(), "worker count changed the order"
    np.savez_compressed(os.path.join(HERE, "G2_shuffle.npz"), **out)


def _state_arrays(model):
    sd = model.state_dict()
    return {k: v.detach().cpu().numpy().copy() for k, v in sd.items()}


def g3_init(NCF):
    import torch
    out = {}
    torch.manual_seed(0)
    m = NCF(944, 1683, 8, 3, 0.0, "NeuMF-end")
    sd = _state_arrays(m)
    out["big_keys"] = np.array(list(sd.keys()))
    out["big_sha256"] = np.array(sha(list(sd.values())))
    for mt in MODEL_TYPES:
        for (f, L) in ((8, 3), (16, 3), (8, 1)):
            torch.manual_seed(1)
            m = NCF(50, 80, f, L, 0.0, mt)
            sd = _state_arrays(m)
            tag = f"{mt}_f{f}_L{L}"
            out[f"{tag}_keys"] = np.array(list(sd.keys()))
            for k, v in sd.items():
                out[f"{tag}::{k}"] = v
            out[f"{tag}_nparams"] = np.int64(sum(p.numel() for p in m.parameters() if p.requires_grad))
    np.savez_compressed(os.path.join(HERE, "G3_init.npz"), **out)


def g4_fwd_bwd(NCF):
    import torch
    import torch.nn as nn
    out = {}
    rng = np.random.default_rng(7)
    B = 256
    users = rng.integers(0, 50, size=B)
    items = rng.integers(0, 80, size=B)
    labels = (rng.random(B) < 0.2).astype(np.int64)
    out["users"], out["items"], out["labels"] = users, items, labels
    for mt in MODEL_TYPES:
        for (f, L) in ((8, 3), (16, 3), (8, 1)):
            torch.manual_seed(1)
            m = NCF(50, 80, f, L, 0.0, mt)
            m.train()
            pred = m(torch.from_numpy(users), torch.from_numpy(items))
            loss = nn.BCEWithLogitsLoss()(pred, torch.from_numpy(labels).float())
            loss.backward()
            tag = f"{mt}_f{f}_L{L}"
            out[f"{tag}_logits"] = pred.detach().numpy()
            out[f"{tag}_loss"] = np.float32(loss.item())
            for k, p in m.named_parameters():
                if p.grad is not None:
                    out[f"{tag}::grad::{k}"] = p.grad.numpy().copy()
    # spot values quoted in SURVEY.md 8(a) rows a2, a7
    torch.manual_seed(0)
    m = NCF(944, 1683, 8, 3, 0.0, "NeuMF-end")
    u = torch.tensor([0, 1, 2, 943])
    i = torch.tensor([0, 1, 2, 1682])
    p = m(u, i)
    out["spot_logits"] = p.detach().numpy()
    out["spot_loss"] = np.float32(nn.BCEWithLogitsLoss()(p, torch.tensor([1., 0., 0., 1.])).item())
    np.savez_compressed(os.path.join(HERE, "G4_fwd_bwd.npz"), **out)


def g5_steps(NCF):
    import torch
    import torch.nn as nn
    import torch.optim as optim
    out = {}
    rng = np.random.default_rng(11)
    B, T = 256, 100
    users = rng.integers(0, 50, size=(T, B))
    items = rng.integers(0, 80, size=(T, B))
    labels = (rng.random((T, B)) < 0.2).astype(np.int64)
    out["users"], out["items"], out["labels"] = users, items, labels
    for mt in ("NeuMF-end", "GMF", "MLP"):
        for opt_name in ("adam", "sgd"):
            if opt_name == "sgd" and mt != "NeuMF-end":
                continue
            torch.manual_seed(3)
            m = NCF(50, 80, 8, 3, 0.0, mt)
            crit = nn.BCEWithLogitsLoss()
            opt = optim.Adam(m.parameters(), lr=1e-3) if opt_name == "adam" \
                else optim.SGD(m.parameters(), lr=1e-3 * 10)
            losses = []
            steps = T if opt_name == "adam" else 10
            for t in range(steps):
                opt.zero_grad()
                pred = m(torch.from_numpy(users[t]), torch.from_numpy(items[t]))
                loss = crit(pred, torch.from_numpy(labels[t]).float())
                loss.backward()
                opt.step()
                losses.append(loss.item())
                if t + 1 in (1, 10, 100):
                    for k, v in _state_arrays(m).items():
                        out[f"{mt}_{opt_name}_t{t + 1}::{k}"] = v
            out[f"{mt}_{opt_name}_losses"] = np.asarray(losses, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "G5_steps.npz"), **out)


def g6_metrics(NCF, NCFData):
    import torch
    import torch.utils.data as data
    out = {}
    rng = np.random.default_rng(5)
    n_users, n_items = 50, 400
    test = []
    for u in range(n_users):
        cand = rng.choice(n_items, size=100, replace=False)
        pos, negs = int(cand[0]), sorted(int(x) for x in cand[1:])
        test.append([u, pos])
        test.extend([u, j] for j in negs)
    test = np.asarray(test, dtype=np.int64)
    out["test_pairs"] = test
    torch.manual_seed(2)
    m = NCF(n_users, n_items, 8, 3, 0.0, "NeuMF-end")
    # make the ranking non-trivial: scale up the item GMF table
    with torch.no_grad():
        m.embed_item_GMF.weight.mul_(50.0)
        m.embed_user_GMF.weight.mul_(50.0)
    m.eval()
    for k, v in _state_arrays(m).items():
        out[f"model::{k}"] = v
    ds = NCFData(test.tolist(), n_items, None, 0, False)
    for bs, k in ((100, 10), (100, 1), (100, 5), (25, 10)):
        loader = data.DataLoader(ds, batch_size=bs, shuffle=False, num_workers=0)
        HR, NDCG = metrics(m, loader, k)
        out[f"bs{bs}_k{k}_HR"] = np.asarray(HR, dtype=np.int64)
        out[f"bs{bs}_k{k}_NDCG"] = np.asarray(NDCG, dtype=np.float64)
    # a batch smaller than top_k raises inside torch.topk (metrics.py:13), as
    # evaluate_models.py:44 does for num_neg + 1 < top_k
    loader = data.DataLoader(ds, batch_size=7, shuffle=False, num_workers=0)
    try:
        metrics(m, loader, 10)
        raise AssertionError("expected topk failure")
    except RuntimeError:
        out["bs7_k10_raises"] = np.bool_(True)
    with torch.no_grad():
        logits = m(torch.from_numpy(test[:, 0]), torch.from_numpy(test[:, 1])).numpy()
    out["logits"] = logits
    np.savez_compressed(os.path.join(HERE, "G6_metrics.npz"), **out)


def g7_script(NCF):
    """The reference's scripts/train_neumf.py, end to end (seeded, 2 epochs) on
    the ml-100k-shaped synthetic files written by ncf_amd.synthetic (seed 0),
    plus load_all's output hash on those files."""
    import contextlib
    import io
    import runpy
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from ncf_amd import synthetic
    from src.data.datasets import load_all
    ds = synthetic.make_dataset("ml-100k", seed=0)
    synthetic.write_reference_files(ds, "data/processed")
    tr, te, un, inum, mat = load_all()
    out = {"load_all_sha256": np.array(sha([np.asarray(tr, dtype=np.int64), np.asarray(te, dtype=np.int64)])),
           "user_num": np.int64(un), "item_num": np.int64(inum), "nnz": np.int64(mat.nnz)}
    for f, L in ((8, 3),):
        np.random.seed(0)
        torch.manual_seed(0)
        argv = sys.argv
        sys.argv = ["train_neumf.py", "--epochs", "2", "--factor_num", str(f), "--num_layers", str(L)]
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            runpy.run_path("scripts/train_neumf.py", run_name="__main__")
        sys.argv = argv
        lines = [l for l in buf.getvalue().splitlines() if l.startswith("Epoch ") or l.startswith("HR@")
                 or l.startswith("NDCG@") or l.startswith("Parameters:") or l.startswith("Best Result")]
        out[f"f{f}_L{L}_stdout"] = np.array(lines)
        sd = torch.load(f"results/models/NeuMF_end_{L}l_{f}f_best.pth", weights_only=True)
        out[f"f{f}_L{L}_best_sha256"] = np.array(sha([v.numpy() for v in sd.values()]))
    np.savez_compressed(os.path.join(HERE, "G7_script.npz"), **out)


def main():
    here_cwd = os.getcwd()
    NCF, NCFData, metrics_fn = _import_reference()
    global metrics
    metrics = metrics_fn
    g1_negatives(NCFData)
    g2_shuffle()
    g3_init(NCF)
    g4_fwd_bwd(NCF)
    g5_steps(NCF)
    g6_metrics(NCF, NCFData)
    g7_script(NCF)
    os.chdir(here_cwd)
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
