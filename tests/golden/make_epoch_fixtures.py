"""G12 / G13: the oracle's whole epoch at C4 and at the stress shape, computed once in
the build container.

* G12 (``c4``): NCF(16,3) NeuMF-end at the ml-20m-shaped synthetic data set (138,494
  users x 26,745 items), 4 negatives per positive, global batch 65,536: 99.3M rows,
  1,516 Adam steps.
* G13 (``stress``): NCF(64,4) NeuMF-end at the ml-1m-shaped set, global batch 65,536:
  76 Adam steps of a 6.4M-parameter model.

Both are the reference loop (scripts/train_neumf.py:98-131) as oracle/ncf_oracle.py
restates it (src/ncf/models.py, src/data/datasets.py:53-69, DataLoader(shuffle=True)
at train_neumf.py:55, src/training/metrics.py:4-25), from the seeds
tests/test_gpu_fullsize.py uses.

tests/test_gpu_fullsize.py::test_full_epoch_vs_oracle ran these epochs on the box's
CPU inside the GPU test (C4: ~450 s, once killed at its 500-s limit; stress ~50 s)
while checking only the first 100 losses, the epoch mean and HR/NDCG.  For these two
configs the test now runs the first 10 oracle steps live and checks them against the
fixture at 1e-5 (which pins the fixture to the oracle on the box's CPU), and takes the
later losses, the epoch mean and the final HR@10 / NDCG@10 from the fixture.

This is the oracle's output (our CPU restatement, itself pinned to the reference by
G1-G11 in tests/test_oracle.py), not a run of the reference.

Usage: python tests/golden/make_epoch_fixtures.py [c4|stress ...]
(C4 about 4 min, stress about 2 min on 8 CPU threads)
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import ncf_oracle as O  # noqa: E402
from ncf_amd import synthetic  # noqa: E402

# name -> (fixture file, data shape, factor_num, num_layers, global batch)
FIXTURES = {"c4": ("G12_c4_epoch.npz", "ml-20m", 16, 3, 65536),
            "stress": ("G13_stress_epoch.npz", "ml-1m", 64, 4, 65536)}


def make(name):
    fname, shape, f, L, B = FIXTURES[name]
    ds = synthetic.make_dataset(shape, seed=0)
    U, I = ds["user_num"], ds["item_num"]
    pu, pi = ds["train_users"], ds["train_items"]
    tu = np.repeat(ds["test_users"], 100)
    ti = np.concatenate([ds["test_items"][:, None], ds["test_negatives"]], 1).reshape(-1)
    np.random.seed(0)
    torch.manual_seed(0)
    ref = O.OracleNCF(U, I, f, L, 0.0, "NeuMF-end")
    neg = O.ng_sample(pu, pi, I, 4, 0)
    users = np.concatenate([pu, np.repeat(pu, 4)]).astype(np.int64)
    items = np.concatenate([pi, neg]).astype(np.int64)
    labels = np.concatenate([np.ones(len(pu), np.int64), np.zeros(len(neg), np.int64)])
    perm = O.epoch_order(len(users))
    nb = (len(users) + B - 1) // B
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    losses = []
    t0 = time.time()
    for c in range(0, nb, 50):
        sl = [perm[b * B:(b + 1) * B] for b in range(c, min(nb, c + 50))]
        losses += O.train_steps(ref, opt, [users[s] for s in sl], [items[s] for s in sl], [labels[s] for s in sl])
        print(f"oracle {name} steps {len(losses)}/{nb} ({time.time() - t0:.0f} s)", flush=True)
    with torch.no_grad():
        logits = ref(torch.as_tensor(tu, dtype=torch.int64), torch.as_tensor(ti, dtype=torch.int64)).numpy()
    HR, NDCG = O.metrics_np(logits, ti, 100, 10)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), fname)
    np.savez_compressed(out, losses=np.asarray(losses, dtype=np.float64), hr=float(np.mean(HR)),
                        ndcg=float(np.mean(NDCG)), n_rows=len(users), neg_head=neg[:4096],
                        torch_version=torch.__version__)
    print("wrote", out, "hr", np.mean(HR), "ndcg", np.mean(NDCG), "mean loss", np.mean(losses))


if __name__ == "__main__":
    for n in (sys.argv[1:] or list(FIXTURES)):
        make(n)
