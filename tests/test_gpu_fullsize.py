"""Full-size parity (SURVEY.md 8(d) gates): a whole epoch of the reference loop at
the ml-1m-shaped synthetic data set, run by Trainer.fit (the epoch pipeline, the
production kernels of each config, hipGraph replay) and by the oracle
(oracle/ncf_oracle.py: NCF restated on torch CPU ops + torch.optim.Adam, the C
restatement of ng_sample, the DataLoader's draws and randperm), from the same
seeds and the same init:

  * negatives bit-exact (datasets.py:53-69), batch membership by construction
    (the same permutation, train_neumf.py:55,106);
  * per-step loss of the first 100 steps (all 76 at bs 65,536) to rtol 1e-5,
    free-running (train_neumf.py:112-115; NCF(64,4): 1e-5 for the first 10, 1e-4
    after, see late_rtol);
  * the first steps teacher-forced from the oracle's state (every parameter after
    the step, test_gpu_parity._teacher_forced_steps);
  * the epoch's mean loss to 1e-3 relative, and HR@10 / NDCG@10 of metrics()
    (metrics.py:4-25) on the leave-one-out test set within 0.01 of the oracle's.

Configs: C2 (NCF(8,3), bs 1,024: tuned launch shape, per-row layer 0, deferred Adam), C3
(NCF(16,3), bs 65,536: fused kernel, factored layer 0), the reference's CLI
default NCF(32,3) at bs 65,536 (layered path, step chain, user order), the stress
NCF(64,4) (layered path, dm-512 factored layer 0 with the GEMM expansion) and C4
(NCF(16,3) at the ml-20m shape, bs 65,536: 99.3M rows, 1,516 steps, per-row layer 0,
deferred Adam).  For C4 and stress the oracle's epoch beyond its first 10 steps comes
from the G12 / G13 fixtures (tests/golden/make_epoch_fixtures.py), checked against
those 10 live steps."""
import os

import numpy as np
import pytest
import torch

from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = {"c4": os.path.join(_GOLDEN, "G12_c4_epoch.npz"), "stress": os.path.join(_GOLDEN, "G13_stress_epoch.npz")}


def _data(shape="ml-1m"):
    from ncf_amd import synthetic
    from ncf_amd.data import NCFData
    ds = synthetic.make_dataset(shape, seed=0)
    I = ds["item_num"]
    train = NCFData(np.stack([ds["train_users"], ds["train_items"]], 1), I, None, 4, True)
    tu = np.repeat(ds["test_users"], 100)
    ti = np.concatenate([ds["test_items"][:, None], ds["test_negatives"]], 1).reshape(-1)
    test = NCFData(np.stack([tu, ti], 1), I, None, 0, False)
    return ds, train, test, tu, ti


# late_rtol: free-running loss tolerance past the first 10 steps.  NCF(64,4) (6.4M
# parameters) turns at step 10 (loss 0.457 -> 0.475) and the two fp32 trajectories part
# there to ~4e-5 relative; C4 (13.2M parameters) parts to ~3.6e-5 from step ~12 (a third
# of the first 100 losses beyond 1e-5 on the MI355X); every step is held to 1e-5
# teacher-forced.
@pytest.mark.parametrize("name,f,L,B,forced,late_rtol", [("c2", 8, 3, 1024, 20, 1e-5), ("c3", 16, 3, 65536, 6, 1e-5),
                                                          ("cli", 32, 3, 65536, 4, 1e-5),
                                                          ("stress", 64, 4, 65536, 3, 1e-4),
                                                          ("c4", 16, 3, 65536, 3, 1e-4)])
def test_full_epoch_vs_oracle(name, f, L, B, forced, late_rtol):
    from torch.utils.data import DataLoader
    from ncf_amd.models import NCF
    from ncf_amd.trainer import Trainer
    from test_gpu_parity import _teacher_forced_steps
    ds, train, test, tu, ti = _data("ml-20m" if name == "c4" else "ml-1m")
    U, I = ds["user_num"], ds["item_num"]
    pu, pi = ds["train_users"], ds["train_items"]
    torch.set_num_threads(min(16, torch.get_num_threads()))

    # ---- device: Trainer.fit(1), as scripts/train_neumf.py runs it
    np.random.seed(0)
    torch.manual_seed(0)
    model = NCF(U, I, f, L, 0.0, "NeuMF-end").to(DEV)
    init = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    tr = Trainer(model, train, DataLoader(test, batch_size=100, shuffle=False), batch_size=B, lr=1e-3,
                 top_k=10, verbose=False)
    tr.fit(1)
    torch.cuda.synchronize()
    eng = tr.engine
    nb = eng.num_batches
    got_losses = eng.epoch_losses()[:nb].astype(np.float64).copy()
    h = tr.history[0]
    u_ep, i_ep, _ = train.arrays()

    # ---- oracle: the same draws from the same seeds
    torch.manual_seed(0)
    ref = O.OracleNCF(U, I, f, L, 0.0, "NeuMF-end")
    for k, v in ref.state_dict().items():
        assert torch.equal(v, init[k]), k
    neg = O.ng_sample(pu, pi, I, 4, 0)
    np.testing.assert_array_equal(neg, i_ep[len(pu):])           # bit-exact negatives
    users = np.concatenate([pu, np.repeat(pu, 4)]).astype(np.int64)
    items = np.concatenate([pi, neg]).astype(np.int64)
    labels = np.concatenate([np.ones(len(pu), np.int64), np.zeros(len(neg), np.int64)])
    np.testing.assert_array_equal(users, u_ep)
    perm = O.epoch_order(len(users))                              # DataLoader(shuffle=True)
    assert nb == (len(users) + B - 1) // B
    bu = [users[perm[b * B:(b + 1) * B]] for b in range(nb)]
    bi = [items[perm[b * B:(b + 1) * B]] for b in range(nb)]
    by = [labels[perm[b * B:(b + 1) * B]] for b in range(nb)]
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    # C4 and stress: the oracle's whole epoch (C4 1,516 CPU steps, ~450 s on the box;
    # stress ~50 s) comes from a fixture made by tests/golden/make_epoch_fixtures.py
    # (G12 / G13); the first 10 steps still run live and must agree with it at 1e-5
    fixture = np.load(FIXTURES[name]) if name in FIXTURES else None
    live = min(10, nb) if fixture is not None else nb
    losses = []
    for c in range(0, live, 100):  # progress lines: a long CPU epoch must not look hung
        losses += O.train_steps(ref, opt, bu[c:min(c + 100, live)], bi[c:min(c + 100, live)],
                                by[c:min(c + 100, live)])
        print(f"[{name}] oracle steps {len(losses)}/{nb}", flush=True)
    losses = np.asarray(losses, dtype=np.float64)
    if fixture is not None:
        assert int(fixture["n_rows"]) == len(users) and len(fixture["losses"]) == nb
        np.testing.assert_array_equal(fixture["neg_head"], neg[:len(fixture["neg_head"])])
        np.testing.assert_allclose(losses, fixture["losses"][:live], rtol=1e-5, err_msg="fixture vs live oracle")
        losses = np.concatenate([losses, fixture["losses"][live:]])
        hr, ndcg = float(fixture["hr"]), float(fixture["ndcg"])
    else:
        with torch.no_grad():
            logits = ref(torch.as_tensor(tu, dtype=torch.int64), torch.as_tensor(ti, dtype=torch.int64)).numpy()
        HR, NDCG = O.metrics_np(logits, ti, 100, 10)
        hr, ndcg = float(np.mean(HR)), float(np.mean(NDCG))

    k = min(100, nb)
    np.testing.assert_allclose(got_losses[:10], losses[:10], rtol=1e-5, err_msg=f"{name}: first 10 step losses")
    np.testing.assert_allclose(got_losses[:k], losses[:k], rtol=late_rtol, err_msg=f"{name}: first {k} step losses")
    assert abs(got_losses.mean() - losses.mean()) <= 1e-3 * losses.mean(), (got_losses.mean(), losses.mean())
    assert abs(h["loss"] - losses.mean()) <= 1e-3 * losses.mean()
    assert abs(h["hr"] - hr) <= 0.01 and abs(h["ndcg"] - ndcg) <= 0.01, (name, h, hr, ndcg)
    assert hr > 0.2, hr  # the epoch learned something (random ranking: 0.1)

    # the first steps again, each from the oracle's own state
    ref.load_state_dict(init)
    _teacher_forced_steps(ref, model, eng, bu[:forced], bi[:forced], by[:forced])
