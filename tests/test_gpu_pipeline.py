"""Epoch pipeline (ncf_amd.pipeline; include/ncf_hip.h ncf_randperm,
ncf_build_rows) -- bit-exact against the host path that the reference's own
outputs pin (test_host.py / test_oracle.py, G1 and G2):

  * the permutation == torch.randperm(n, generator) (DataLoader(shuffle=True),
    train_neumf.py:55), including n = 1, 2 and the ml-1m / ml-20m sizes;
  * whole epochs (with the prefetch threads) == ng_sample + epoch_permutation +
    rows[perm] of the host path, batch by batch, and both generators end in the
    same state; a prefetch invalidated by an unexpected draw is discarded.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _dataset(pu, pi, num_item, ng):
    from ncf_amd.data import NCFData
    return NCFData(np.stack([pu, pi], 1), num_item, None, ng, True)


def _randperm(words_u32, n):
    import ncf_amd._lib as L
    words = torch.from_numpy(np.ascontiguousarray(words_u32).view(np.int32)).to(DEV)
    perm = torch.empty(n, dtype=torch.int64, device=DEV)
    ws = torch.empty(int(L.hip().ncf_randperm_workspace(n)), dtype=torch.uint8, device=DEV)
    L.check(L.hip().ncf_randperm(words.data_ptr(), n, perm.data_ptr(), ws.data_ptr(), ws.numel(), L.stream_ptr()),
            "ncf_randperm")
    return perm.cpu()


@pytest.mark.parametrize("n,seed", [(1, 0), (2, 3), (1000, 7), (65537, 2**40 + 5), (4970845, 123),
                                    (99308850, 9)])
def test_randperm_matches_torch(n, seed):
    from ncf_amd.pipeline import torch_words
    g = torch.Generator()
    g.manual_seed(seed)
    exp = torch.randperm(n, generator=g)
    w = np.empty(max(1, n - 1), dtype=np.uint32)
    torch_words(seed, n - 1, w)
    assert torch.equal(_randperm(w, n), exp)


def _fisher_yates(w, n):
    a = np.arange(n, dtype=np.int64)
    for i in range(n - 1):
        h = i + int(w[i]) % (n - i)
        a[i], a[h] = a[h], a[i]
    return a


@pytest.mark.parametrize("kind", ["zeros", "all_to_last", "chain", "few_targets"])
def test_randperm_structured_words(kind):
    """Words far from uniform (identity swaps, every step into the last position,
    one long chain, a handful of hot targets) -- the closed form's list and chain
    walks at their longest -- vs the sequential loop."""
    n = 3000
    i = np.arange(n - 1, dtype=np.int64)
    w = {"zeros": np.zeros(n - 1),
         "all_to_last": n - 1 - i,                       # H[i] = n - 1
         "chain": np.ones(n - 1),                        # H[i] = i + 1
         "few_targets": (np.array([2000, 2500, 2999])[i % 3] - i) % (n - i)}[kind].astype(np.uint32)
    assert np.array_equal(_randperm(w, n).numpy(), _fisher_yates(w, n))


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_pipeline_epochs_equal_host_path(depth):
    """Five epochs with prefetch `depth` epochs ahead and an eval draw between
    them, vs the host path (rotating output buffers: each checked when returned)."""
    from ncf_amd import ops
    from ncf_amd.data import consume_test_pass, epoch_permutation
    from ncf_amd.pipeline import EpochPipeline
    from ncf_amd import synthetic
    d = synthetic.make_dataset("ml-100k", seed=1)
    pu, pi, I, U, B = d["train_users"], d["train_items"], d["item_num"], d["user_num"], 4096
    np.random.seed(3)
    torch.manual_seed(3)
    ds = _dataset(pu, pi, I, 4)
    exp = []
    E = 5
    for _ in range(E):
        ds.ng_sample()
        u, i, y = ds.arrays()
        perm = epoch_permutation(len(u)).numpy()
        exp.append(ops.pack_rows_host(u, i, y)[perm])
        consume_test_pass()
    np_exp, t_exp = np.random.get_state(), torch.get_rng_state()
    np.random.seed(3)
    torch.manual_seed(3)
    ds2 = _dataset(pu, pi, I, 4)
    pipe = EpochPipeline(ds2, DEV, B, I, user_num=U, depth=depth)
    for e in range(E):
        got = pipe.next_epoch(peek_eval_draw=True).cpu().numpy()
        for b0 in range(0, len(got), B):
            assert np.array_equal(np.sort(got[b0:b0 + B]), np.sort(exp[e][b0:b0 + B])), (e, b0)
        consume_test_pass()
    pipe.close()
    assert pipe.stats["prefetch_hits"] == E - 1
    u2, i2, _ = ds2.arrays()  # host views of the device negatives
    assert np.array_equal(ops.pack_rows_host(u2, i2, ds2.arrays()[2]), ops.pack_rows_host(*ds.arrays()))
    st = np.random.get_state()
    assert np.array_equal(st[1], np_exp[1]) and st[2] == np_exp[2]
    assert torch.equal(torch.get_rng_state(), t_exp)


def test_pipeline_discards_prefetch_after_foreign_draws():
    """Another consumer of either generator between epochs: the prefetched epoch
    is rebuilt from the real state, and the result still equals the host path."""
    from ncf_amd import ops
    from ncf_amd.data import epoch_permutation
    from ncf_amd.pipeline import EpochPipeline
    rng = np.random.default_rng(2)
    pu = np.repeat(np.arange(300, dtype=np.int32), 30)
    pi = rng.integers(0, 500, len(pu)).astype(np.int32)
    B = 1000
    np.random.seed(4)
    torch.manual_seed(4)
    ds = _dataset(pu, pi, 500, 4)
    exp = []
    for e in range(3):
        ds.ng_sample()
        u, i, y = ds.arrays()
        exp.append(ops.pack_rows_host(u, i, y)[epoch_permutation(len(u)).numpy()])
        if e == 0:
            np.random.randint(7)      # a foreign NumPy draw
        if e == 1:
            torch.rand(3)             # a foreign torch draw
    np.random.seed(4)
    torch.manual_seed(4)
    ds2 = _dataset(pu, pi, 500, 4)
    pipe = EpochPipeline(ds2, DEV, B, 500, user_num=300)
    for e in range(3):
        got = pipe.next_epoch(peek_eval_draw=False).cpu().numpy()
        assert np.array_equal(got, exp[e]), e  # B < 4096: shuffled, not grouped
        if e == 0:
            np.random.randint(7)
        if e == 1:
            torch.rand(3)
    pipe.close()
    assert pipe.stats["prefetch_hits"] == 0


def test_engine_captures_every_pipeline_buffer_once():
    """The engine captures the step graphs for all of the pipeline's rotating
    output buffers at its first capture; later epoch boundaries replay them."""
    from ncf_amd import synthetic
    from ncf_amd.engine import TrainEngine
    from ncf_amd.models import NCF
    from ncf_amd.pipeline import EpochPipeline
    d = synthetic.make_dataset("ml-100k", seed=2)
    pu, pi, I, U, B = d["train_users"], d["train_items"], d["item_num"], d["user_num"], 8192
    np.random.seed(5)
    torch.manual_seed(5)
    model = NCF(U, I, 8, 3, 0.0, "NeuMF-end").to(DEV)
    pipe = EpochPipeline(_dataset(pu, pi, I, 4), DEV, B, I, user_num=U, depth=2)
    eng = TrainEngine(model, lr=1e-3)
    eng.stream_buffers = pipe.buffers
    seen = set()
    for _ in range(5):
        rows = pipe.next_epoch(peek_eval_draw=False)
        seen.add(rows.data_ptr())
        eng.set_epoch_stream(rows, B, checked=True)
        eng.run(eng.num_batches)
        assert len(eng._graphs) == len(pipe.buffers)
    pipe.close()
    torch.cuda.synchronize()
    assert seen == {b.data_ptr() for b in pipe.buffers}
    assert np.isfinite(eng.epoch_losses()).all()
