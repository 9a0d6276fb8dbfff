"""Pin the CPU oracle against the reference's own outputs (tests/golden/*.npz).

No GPU needed.  If these fail, nothing downstream (GPU parity) means anything.
"""
import hashlib

import numpy as np
import pytest
import torch

from oracle import ncf_oracle as O

MODEL_TYPES = ["GMF", "MLP", "NeuMF-end", "NeuMF-pre"]
SHAPES = [(8, 3), (16, 3), (8, 1)]


def _sha(arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


# ---------------------------------------------------------------- G1 negatives
def test_toy_negatives_kat(golden):
    g = golden("G1_negatives")
    toy = g["toy_pos"]
    neg = O.ng_sample(toy[:, 0], toy[:, 1], int(g["toy_num_item"]), 4, 0)
    assert neg.tolist() == g["toy_neg_seed0"].tolist() == [4, 0, 3, 3, 3, 3, 4, 0, 4, 2, 1, 1, 1, 0, 1, 4]


@pytest.mark.parametrize("seed", [0, 1])
def test_small_negatives_rejection_heavy(golden, seed):
    g = golden("G1_negatives")
    pos = g["small_pos"]
    neg = O.ng_sample(pos[:, 0], pos[:, 1], int(g["small_num_item"]), 4, seed)
    assert np.array_equal(neg, g[f"small_neg_seed{seed}"].astype(np.int64))
    neg_py = O.ng_sample_py(pos[:, 0], pos[:, 1], int(g["small_num_item"]), 4, seed)
    assert np.array_equal(neg, neg_py)


def test_ml100k_shaped_negatives_hash(golden):
    g = golden("G1_negatives")
    pos = g["big_pos"].astype(np.int64)
    neg = O.ng_sample(pos[:, 0], pos[:, 1], int(g["big_num_item"]), 4, 0).astype(np.int32)
    assert np.array_equal(neg[:4096], g["big_neg_seed0_head"])
    assert _sha([neg]) == str(g["big_neg_seed0_sha256"])


def test_mt_words_match_numpy_legacy():
    for seed in (0, 1, 12345, 2**32 - 1):
        rs = np.random.RandomState(seed)
        ref = rs.randint(0, 2**32, size=5000, dtype=np.uint64).astype(np.uint32)
        assert np.array_equal(O.mt_words(seed, 5000), ref)


# ---------------------------------------------------------------- G2 shuffle
@pytest.mark.parametrize("seed", [0, 7])
@pytest.mark.parametrize("n,bs", [(1000, 64), (257, 256)])
def test_epoch_order_protocol(golden, seed, n, bs):
    g = golden("G2_shuffle")
    torch.manual_seed(seed)
    for ep in range(2):
        order = O.epoch_order(n)
        assert np.array_equal(order.astype(np.int32), g[f"s{seed}_n{n}_ep{ep}"])
        sizes = [min(bs, n - s) for s in range(0, n, bs)]
        assert sizes == g[f"s{seed}_n{n}_ep{ep}_sizes"].tolist()
        O.test_pass_draw()


# ---------------------------------------------------------------- G3 init
def test_init_big_sha(golden):
    g = golden("G3_init")
    torch.manual_seed(0)
    m = O.OracleNCF(944, 1683, 8, 3, 0.0, "NeuMF-end")
    sd = O.flat_state(m)
    assert list(sd.keys()) == g["big_keys"].tolist()
    assert _sha(list(sd.values())) == str(g["big_sha256"])


@pytest.mark.parametrize("mt", MODEL_TYPES)
@pytest.mark.parametrize("f,L", SHAPES)
def test_init_small_exact(golden, mt, f, L):
    g = golden("G3_init")
    tag = f"{mt}_f{f}_L{L}"
    torch.manual_seed(1)
    m = O.OracleNCF(50, 80, f, L, 0.0, mt)
    sd = O.flat_state(m)
    assert list(sd.keys()) == g[f"{tag}_keys"].tolist()
    for k, v in sd.items():
        assert np.array_equal(v, g[f"{tag}::{k}"]), k
    assert sum(p.numel() for p in m.parameters()) == int(g[f"{tag}_nparams"])


# ---------------------------------------------------------------- G4 fwd/bwd
@pytest.mark.parametrize("mt", MODEL_TYPES)
@pytest.mark.parametrize("f,L", SHAPES)
def test_forward_backward(golden, mt, f, L):
    g = golden("G4_fwd_bwd")
    tag = f"{mt}_f{f}_L{L}"
    torch.manual_seed(1)
    m = O.OracleNCF(50, 80, f, L, 0.0, mt)
    logits, loss, grads = O.forward_backward(m, g["users"], g["items"], g["labels"])
    np.testing.assert_allclose(logits.numpy(), g[f"{tag}_logits"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(loss, float(g[f"{tag}_loss"]), rtol=1e-6)
    names = [k.split("::grad::")[1] for k in g.files if k.startswith(tag + "::grad::")]
    assert sorted(names) == sorted(grads.keys())
    for k in names:
        np.testing.assert_allclose(grads[k].numpy(), g[f"{tag}::grad::{k}"], rtol=1e-5, atol=1e-9)


def test_spot_values(golden):
    g = golden("G4_fwd_bwd")
    torch.manual_seed(0)
    m = O.OracleNCF(944, 1683, 8, 3, 0.0, "NeuMF-end")
    p = m(torch.tensor([0, 1, 2, 943]), torch.tensor([0, 1, 2, 1682]))
    np.testing.assert_array_equal(p.detach().numpy(), g["spot_logits"])
    loss = O.bce_mean(p, torch.tensor([1, 0, 0, 1]))
    assert np.float32(loss.item()) == g["spot_loss"]


# ---------------------------------------------------------------- G5 trajectories
@pytest.mark.parametrize("mt,opt", [("NeuMF-end", "adam"), ("GMF", "adam"), ("MLP", "adam"), ("NeuMF-end", "sgd")])
def test_train_trajectory(golden, mt, opt):
    g = golden("G5_steps")
    torch.manual_seed(3)
    m = O.OracleNCF(50, 80, 8, 3, 0.0, mt)
    o = O.make_optimizer(m, 1e-3 if opt == "adam" else 1e-2, opt)
    T = 100 if opt == "adam" else 10
    losses = O.train_steps(m, o, g["users"], g["items"], g["labels"], steps=T)
    np.testing.assert_allclose(losses, g[f"{mt}_{opt}_losses"], rtol=1e-6)
    sd = O.flat_state(m)
    for k, v in sd.items():
        np.testing.assert_allclose(v, g[f"{mt}_{opt}_t{T}::{k}"], rtol=1e-5, atol=1e-7)


# ---------------------------------------------------------------- G6 metrics
@pytest.mark.parametrize("bs,k", [(100, 10), (100, 1), (100, 5), (25, 10)])
def test_metrics(golden, bs, k):
    g = golden("G6_metrics")
    test = g["test_pairs"]
    HR, NDCG = O.metrics_np(g["logits"], test[:, 1], bs, k)
    assert HR == g[f"bs{bs}_k{k}_HR"].tolist()
    np.testing.assert_allclose(NDCG, g[f"bs{bs}_k{k}_NDCG"], rtol=0, atol=0)


def test_metrics_small_batch_raises(golden):
    g = golden("G6_metrics")
    assert bool(g["bs7_k10_raises"])
    with pytest.raises(RuntimeError):
        O.metrics_np(g["logits"], g["test_pairs"][:, 1], 7, 10)


# ---------------------------------------------------------------------------
# G8: distillation (config C5) -- the oracle's restatement of src/distillation/*
# against the reference's own outputs (tests/golden/make_golden_kd.py)
KD_CASES = {"c5": ((16, 3, "NeuMF-end"), (8, 2, "MLP")),
            "cli": ((32, 2, "NeuMF-end"), (16, 1, "NeuMF-end")),
            "same": ((8, 2, "GMF"), (8, 2, "GMF"))}


@pytest.mark.parametrize("case", list(KD_CASES))
@pytest.mark.parametrize("strategy", ["response", "feature", "attention"])
def test_oracle_distillation_vs_reference(golden, case, strategy):
    g = golden("G8_distill")
    tag = f"{case}_{strategy}"
    (tf, tl, tm), (sf, sl, sm) = KD_CASES[case]
    torch.manual_seed(7)
    teacher = O.OracleNCF(50, 80, tf, tl, 0.0, tm)
    student = O.OracleNCF(50, 80, sf, sl, 0.0, sm)
    dist = O.OracleDistill(teacher, student, strategy, 2.0, 0.5, 0.3, 0.2)
    # same construction order -> bit-identical initial weights and adapters
    for k, v in teacher.state_dict().items():
        assert np.array_equal(v.numpy(), g[f"{tag}::teacher::{k}"]), k
    for k, v in student.state_dict().items():
        assert np.array_equal(v.numpy(), g[f"{tag}::student0::{k}"]), k
    for k, v in dist.adaptation_layers.state_dict().items():
        assert np.array_equal(v.numpy(), g[f"{tag}::adapter::{k}"]), k
    opt = torch.optim.Adam(student.parameters(), lr=1e-3)
    losses = []
    for s in range(g["users"].shape[0]):
        u, i = torch.from_numpy(g["users"][s]), torch.from_numpy(g["items"][s])
        y = torch.from_numpy(g["labels"][s])
        opt.zero_grad()
        loss = dist(u, i, y)
        loss.backward()
        if s == 0:
            np.testing.assert_allclose(loss.item(), float(g[f"{tag}::loss0"]), rtol=1e-6)
            for k, p in student.named_parameters():
                key = f"{tag}::grad0::{k}"
                assert (p.grad is not None) == (key in g.files), k
                if p.grad is not None:
                    np.testing.assert_allclose(p.grad.numpy(), g[key], rtol=1e-5,
                                               atol=1e-7 * float(np.abs(g[key]).max() or 1), err_msg=k)
        opt.step()
        losses.append(loss.item())
    np.testing.assert_allclose(losses, g[f"{tag}::losses"], rtol=1e-6)
    for k, v in student.state_dict().items():
        np.testing.assert_allclose(v.numpy(), g[f"{tag}::student_t5::{k}"], rtol=1e-5, atol=1e-7, err_msg=k)


def test_c4_fp32_trajectory_sensitivity():
    """How far two fp32 runs of the reference loop itself part at C4 (NCF(16,3) on the
    ml-20m-shaped stream, batch 65,536; scripts/train_neumf.py:106-118): the oracle
    from the same init over the same 100 batches, once with every initial parameter and
    every gradient element before each Adam step moved by at most one ulp (a random half
    of them, upward) -- the size of the rounding differences an implementation that
    orders its fp32 sums differently makes at every step.  The per-step losses stay within 1e-5 for the first
    10 steps (the bar every full-size GPU test holds); then the dynamics amplify the
    one-ulp differences to the order of 1e-5 within 100 steps (measured 1.3e-5, first
    above 1e-5 at step 88), and they stay under 1e-4.  That is the
    measured basis of the 1e-4 late tolerance of test_gpu_fullsize.py (C4) and
    test_gpu_multirank_fullsize.py.  (Measured: a one-ulp move of the initial
    parameters alone parts first past 1e-5 between steps 57 and 80, max 1.1e-5 to
    4.1e-5 over 100 steps -- 8-thread CPU runs are not bitwise reproducible themselves;
    one-ulp gradient moves alone: step 64, max 1.8e-5.)"""
    from ncf_amd import synthetic
    torch.set_num_threads(8)
    ds = synthetic.make_dataset("ml-20m", seed=0)
    U, I = ds["user_num"], ds["item_num"]
    pu, pi = ds["train_users"], ds["train_items"]
    neg = O.ng_sample(pu, pi, I, 4, 0)
    users = np.concatenate([pu, np.repeat(pu, 4)]).astype(np.int64)
    items = np.concatenate([pi, neg]).astype(np.int64)
    labels = np.concatenate([np.ones(len(pu), np.int64), np.zeros(len(neg), np.int64)])
    perm = O.epoch_order(len(users))
    B, S = 65536, 100
    sl = [perm[b * B:(b + 1) * B] for b in range(S)]
    runs = []
    for ulp in (False, True):
        torch.manual_seed(0)
        ref = O.OracleNCF(U, I, 16, 3, 0.0, "NeuMF-end")
        g = torch.Generator().manual_seed(1)
        if ulp:
            with torch.no_grad():
                for p in ref.parameters():
                    up = torch.rand(p.shape, generator=g) < 0.5
                    p.copy_(torch.where(up, torch.nextafter(p, torch.full_like(p, float("inf"))), p))
        opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
        losses = []
        for s in sl:
            opt.zero_grad()
            loss = O.bce_mean(ref(torch.as_tensor(users[s]), torch.as_tensor(items[s])), torch.as_tensor(labels[s]))
            loss.backward()
            if ulp:
                with torch.no_grad():
                    for p in ref.parameters():
                        up = torch.rand(p.shape, generator=g) < 0.5
                        p.grad.copy_(torch.where(up, torch.nextafter(p.grad, torch.full_like(p.grad, float("inf"))),
                                                 p.grad))
            opt.step()
            losses.append(loss.item())
        runs.append(np.asarray(losses, dtype=np.float64))
    rel = np.abs(runs[0] - runs[1]) / np.abs(runs[0])
    print("C4 oracle vs oracle(1-ulp init + gradients): max rel %.2e, first step > 1e-5: %s; per step (1e-6): %s" %
          (rel.max(), int(np.argmax(rel > 1e-5)) if (rel > 1e-5).any() else None, np.round(rel * 1e6, 1).tolist()))
    assert rel[:10].max() <= 1e-5
    # the reference's own fp32 loop parts to the order of the 1e-5 bar within 100 steps
    # (1.3e-5 and 1.8e-5 measured; the bound leaves room for the CPU runs' own
    # non-reproducibility) and stays within the late tolerance
    assert rel.max() > 5e-6
    assert rel.max() <= 1e-4
