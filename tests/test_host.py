"""CPU tests of the host side: C-ABI libraries load and export every declared
symbol, the product sampler / data path / shuffle protocol match the
reference's golden vectors, layout and config agree with the reference."""
import ctypes
import hashlib
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ncf_[a-z0-9_]+)\s*\(", src)))


@pytest.mark.parametrize("header,lib", [("ncf_hip.h", "libncf_hip.so"), ("ncf_sampler.h", "libncf_sampler.so")])
def test_library_exports_every_declared_symbol(header, lib):
    import ncf_amd._lib  # noqa: F401  (torch first, then the HIP runtime it ships)
    so = ctypes.CDLL(os.path.join(ROOT, "ncf_amd", lib))
    names = _declared(header)
    assert len(names) >= 4
    for n in names:
        assert hasattr(so, n), f"{lib} does not export {n}"


def test_integration_stub_abi_matches_header():
    """INTEGRATION.md's binding asserts the header's ABI version (the GPU
    integration tests exec that block)."""
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "include", "ncf_hip.h")).read()
    doc = open(os.path.join(root, "INTEGRATION.md")).read()
    want = int(re.search(r"#define NCF_ABI_VERSION (\d+)", hdr).group(1))
    assert int(re.search(r"ncf_abi_version\(\) == (\d+)", doc).group(1)) == want


def test_abi_version_and_layout():
    import ncf_amd._lib as L
    import re
    hdr = open(os.path.join(ROOT, "include", "ncf_hip.h")).read()
    want = int(re.search(r"#define NCF_ABI_VERSION (\d+)", hdr).group(1))
    assert L.hip().ncf_abi_version() == L.ABI_VERSION == want
    for U, I, f, nl, mt in ((944, 1683, 8, 3, "NeuMF-end"), (6041, 3707, 16, 3, "NeuMF-end"), (50, 80, 8, 1, "GMF")):
        lay = L.layout(U, I, f, nl, mt)
        from ncf_amd.models import NCF
        m = NCF(U, I, f, nl, 0.0, mt)
        sizes = [p.numel() for p in m.ordered_params()]
        offs = [lay.ug, lay.ig, lay.um, lay.im] + [x for k in range(nl) for x in (lay.w[k], lay.b[k])] + [lay.wp, lay.bp]
        for a, b, n in zip(offs, offs[1:], sizes):
            assert a % 64 == 0 and b - a >= n
        assert lay.tower_begin == lay.w[0] and lay.loss_slot == lay.tower_begin + lay.tower_len
        assert lay.total >= lay.loss_slot + 1
        assert L.hip().ncf_slab_stride(ctypes.byref(lay)) == lay.tower_len + 64
    assert L.supported("NeuMF-end", 16, 3) == L.supported("GMF", 8, 3) == L.PATH_FUSED
    # towers too large for LDS and factor sizes without a fused kernel take the layered path
    for mt, f, nl in [("NeuMF-end", 64, 4), ("NeuMF-end", 32, 3), ("MLP", 6, 2), ("GMF", 5, 1)]:
        assert L.supported(mt, f, nl) == L.PATH_LAYERED
    assert L.supported("NeuMF-end", 16, 5) == 0  # num_layers > 4: no layout
    lay = L.layout(6041, 3707, 64, 4, "NeuMF-end")
    ws = L.hip().ncf_workspace_bytes(ctypes.byref(lay), 65536)
    dm = 64 * 8
    acts = 65536 * (dm + dm // 2 + dm // 4 + dm // 8) + 2 * 65536 * dm
    rows = L.hip().ncf_reduce_rows(ctypes.byref(lay))  # layered: slab rows the atomics spread over
    # dm 512: factored layer 0 expanded by GEMMs (W0 into the slab: no partials), the
    # workspace adds the two tables' projections
    assert L.hip().ncf_fact_mode(ctypes.byref(lay)) == 1
    assert 1 <= rows <= 16 and L.hip().ncf_fact_partials_bytes(ctypes.byref(lay)) == 0
    proj = (6041 + 3707) * dm
    # plus the wide step chain's weight images (ncf_chain_wide.inc: 42 chunks of 48 KB and
    # four pre-split W0 images of 1.5 MB)
    wc = 42 * 48 * 1024 // 4 + 4 * 32 * 16 * 3072 // 4
    assert (acts + proj + wc) * 4 <= ws <= (acts + proj + wc + rows * (lay.tower_len + 64) + 64 * 10) * 4
    # NCF(32,3) at ml-1m: factored layer 0 on the layered path (ABI 10): the
    # workspace adds the dW0 partials and the two tables' projections
    lay = L.layout(6041, 3707, 32, 3, "NeuMF-end")
    assert L.hip().ncf_fact_mode(ctypes.byref(lay)) == 1
    pb = L.hip().ncf_fact_partials_bytes(ctypes.byref(lay))
    assert pb > 0 and pb % (128 * 128 * 4) == 0
    ws = L.hip().ncf_workspace_bytes(ctypes.byref(lay), 65536)
    acts = 65536 * (128 + 64 + 32) + 2 * 65536 * 128 + (6041 + 3707) * 128
    assert ws >= acts * 4 + pb
    assert L.hip().ncf_forward_workspace_bytes(ctypes.byref(L.layout(6041, 3707, 16, 3, "NeuMF-end")), 10 ** 6) == 0


def test_product_sampler_bit_exact(golden):
    from ncf_amd.data import NCFData
    g = golden("G1_negatives")
    toy = g["toy_pos"]
    np.random.seed(0)
    d = NCFData(toy.tolist(), 5, None, 4, True)
    d.ng_sample()
    assert d._ng_i.tolist() == g["toy_neg_seed0"].tolist()
    for seed in (0, 1):
        np.random.seed(seed)
        d = NCFData(g["small_pos"], int(g["small_num_item"]), None, 4, True)
        d.ng_sample()
        assert np.array_equal(d._ng_i, g[f"small_neg_seed{seed}"].astype(np.int32))
        assert d.labels_fill == [1] * len(g["small_pos"]) + [0] * 4 * len(g["small_pos"])
    np.random.seed(0)
    d = NCFData(g["big_pos"], int(g["big_num_item"]), None, 4, True)
    d.ng_sample()
    assert hashlib.sha256(d._ng_i.astype(np.int32).tobytes()).hexdigest() == str(g["big_neg_seed0_sha256"])


def test_sampler_continues_numpy_global_stream():
    """After ng_sample the global legacy generator is where the Python loop leaves it."""
    from ncf_amd.data import NCFData
    from oracle import ncf_oracle as O
    rng = np.random.default_rng(4)
    pos = np.stack([np.repeat(np.arange(30), 5), rng.integers(0, 40, 150)], 1)
    pos = np.unique(pos, axis=0)
    np.random.seed(9)
    d = NCFData(pos, 40, None, 3, True)
    d.ng_sample()
    d.ng_sample()
    after = np.random.randint(1000, size=8)
    # pure-Python restatement on numpy's own global generator
    np.random.seed(9)
    train = set(map(tuple, pos.tolist()))
    for _ in range(2):
        for u in pos[:, 0].tolist():
            for _ in range(3):
                j = np.random.randint(40)
                while (u, j) in train:
                    j = np.random.randint(40)
    assert np.array_equal(after, np.random.randint(1000, size=8))
    assert len(O.ng_sample(pos[:, 0], pos[:, 1], 40, 3, 9)) == 3 * len(pos)


@pytest.mark.parametrize("seed", [0, 7])
def test_epoch_permutation_matches_dataloader(golden, seed):
    from ncf_amd.data import consume_test_pass, epoch_permutation
    g = golden("G2_shuffle")
    torch.manual_seed(seed)
    for ep in range(2):
        assert np.array_equal(epoch_permutation(1000).numpy().astype(np.int32), g[f"s{seed}_n1000_ep{ep}"])
        consume_test_pass()


def test_getitems_collates_like_reference():
    import torch.utils.data as data
    from ncf_amd.data import NCFData
    pos = np.array([[0, 1], [0, 2], [1, 0], [2, 3]])
    np.random.seed(0)
    d = NCFData(pos.tolist(), 5, None, 4, True)
    d.ng_sample()
    assert len(d) == 20 and d[0] == (0, 1, 1) and d[4] == (0, 4, 0)
    loader = data.DataLoader(d, batch_size=8, shuffle=False)
    batches = list(loader)
    u, i, y = batches[0]
    assert u.dtype == torch.int64 and y.dtype == torch.int64 and len(u) == 8
    assert u.tolist() == [int(x) for x in d._fill_u[:8]] and y.tolist() == [1, 1, 1, 1, 0, 0, 0, 0]
    assert sum(len(b[0]) for b in batches) == 20


def test_load_all_matches_reference_on_synthetic_files(golden, tmp_path, monkeypatch):
    from ncf_amd import synthetic
    g = golden("G7_script")
    monkeypatch.chdir(tmp_path)
    ds = synthetic.make_dataset("ml-100k", seed=0)
    synthetic.write_reference_files(ds, "data/processed")
    from ncf_amd.data import load_all
    tr, te, un, inum, mat = load_all()
    h = hashlib.sha256()
    for a in (np.asarray(tr, dtype=np.int64), np.asarray(te, dtype=np.int64)):
        h.update(np.ascontiguousarray(a).tobytes())
    assert h.hexdigest() == str(g["load_all_sha256"])
    assert (un, inum, mat.nnz) == (int(g["user_num"]), int(g["item_num"]), int(g["nnz"]))
    assert (0 + 0) == 0 and (int(tr[0][0]), int(tr[0][1])) in mat


def test_config_defaults():
    from ncf_amd.config import Config
    c = Config()
    assert (c.batch_size, c.epochs, c.lr, c.num_ng, c.test_num_ng, c.top_k) == (256, 20, 0.001, 4, 99, 10)
    assert (c.factor_num, c.num_layers, c.dropout, c.model_type) == (32, 2, 0.0, "NeuMF-end")
    assert str(c.train_rating) == "data/processed/u.train.rating"


def test_model_init_and_keys_match_reference(golden):
    from ncf_amd.models import NCF
    g = golden("G3_init")
    torch.manual_seed(0)
    m = NCF(944, 1683, 8, 3, 0.0, "NeuMF-end")
    sd = m.state_dict()
    assert list(sd.keys()) == g["big_keys"].tolist()
    h = hashlib.sha256()
    for v in sd.values():
        h.update(v.numpy().tobytes())
    assert h.hexdigest() == str(g["big_sha256"])


def test_cpu_module_semantics_match_golden(golden):
    """The module on a CPU device is the reference module (stock torch ops)."""
    from ncf_amd.models import NCF
    g = golden("G4_fwd_bwd")
    torch.manual_seed(1)
    m = NCF(50, 80, 16, 3, 0.0, "NeuMF-end")
    p = m(torch.from_numpy(g["users"]), torch.from_numpy(g["items"]))
    np.testing.assert_allclose(p.detach().numpy(), g["NeuMF-end_f16_L3_logits"], rtol=1e-6, atol=1e-7)


def test_pipelined_sampler_many_blocks_matches_oracle():
    """ml-1m-sized pass (~4.3M words: the generator thread's block ring wraps many
    times) vs the oracle's C restatement, twice in a row on the global stream."""
    from ncf_amd.data import NCFData
    from oracle import ncf_oracle as O
    rng = np.random.default_rng(8)
    U, I = 6041, 3707
    counts = rng.integers(1, 330, U)
    pu = np.repeat(np.arange(U), counts)
    pi = rng.integers(0, I, len(pu))
    np.random.seed(21)
    d = NCFData(np.stack([pu, pi], 1), I, None, 4, True)
    d.ng_sample()
    first = d._ng_i.copy()
    d.ng_sample()
    after = np.random.randint(1 << 30, size=4)
    exp = O.ng_sample(pu, pi, I, 4, 21)
    assert np.array_equal(first, exp)
    # the second pass continues the stream: replay both on numpy's own generator state
    np.random.seed(21)
    from ncf_amd.data import HostSampler
    s = HostSampler(pu, pi, U, I)
    s.sample(I, 4)
    assert np.array_equal(s.sample(I, 4), d._ng_i)
    assert np.array_equal(np.random.randint(1 << 30, size=4), after)


def test_dropout_hash_restatement_and_statistics():
    """include/ncf_hip.h ncf_dropout_hash (host export of the device function) ==
    the oracle's numpy restatement; keep rates match 1 - p per layer, step and
    column block; masks of different steps / layers / rows are uncorrelated."""
    import ncf_amd._lib as L
    from oracle import ncf_oracle as O
    rng = np.random.default_rng(1)
    for _ in range(4):
        seed, t, k = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**31)), int(rng.integers(0, 4))
        rows = rng.integers(0, 2**40, 8)
        h = O.dropout_hash(seed, t, k, rows, np.arange(5))
        for a in range(8):
            for c in range(5):
                assert int(h[a, c]) == L.hip().ncf_dropout_hash(seed, t, k, int(rows[a]), c)
    rows, cols = np.arange(50000), np.arange(64)
    for p in (0.1, 0.5, 0.9):
        thr = np.uint32(int(float(np.float32(p)) * 4294967296.0))
        keep = [O.dropout_hash(3, t, k, rows, cols) >= thr for t, k in ((0, 0), (1, 0), (0, 1))]
        for kp in keep:
            assert abs(kp.mean() - (1 - p)) < 0.005
            assert abs(kp[:, :8].mean() - (1 - p)) < 0.01
        for a, b in ((0, 1), (0, 2)):
            assert abs(np.corrcoef(keep[a].ravel(), keep[b].ravel())[0, 1]) < 0.01


def test_prepare_workspace_small_batches():
    """ncf_prepare_epoch_workspace: batches under 4,096 rows are only shuffled, so no
    per-batch item histogram is reserved (the reference default batch_size 256 at
    ml-20m would otherwise reserve ~42 GB)."""
    import ncf_amd._lib as L
    n, items = 4970845, 3707
    small = L.hip().ncf_prepare_epoch_workspace(n, 256, items)
    assert 0 < small <= 256
    big = L.hip().ncf_prepare_epoch_workspace(n, 65536, items)
    nb = (n + 65535) // 65536
    assert big >= n * 8 + nb * items * 4
    assert L.hip().ncf_prepare_epoch_workspace(20_000_000, 256, 26744) <= 256


def test_auto_dp_mode_by_global_batch():
    """dp_mode "auto" (world > 1 default): the packed touched-row exchange only where
    it is well under the flat gradient -- C3's 65,536-row batch touches every ml-1m
    row (all-reduce), C4's ml-20m tables are ~0.56 of it (touched)."""
    import ncf_amd._lib as L
    from ncf_amd.engine import TrainEngine, _active_ranges
    from ncf_amd.models import NCF
    assert TrainEngine.default_dp_mode(10 ** 6, touched_ok=True) == "auto"
    assert TrainEngine.default_dp_mode(10 ** 6) == "allreduce"
    assert TrainEngine.default_dp_mode(10 ** 8) == "zero1"
    # NCF(64,4) at ml-1m (6.45M floats, above ALLREDUCE_MAX_FLOATS): every row touched,
    # so the packed test fails and the size rule keeps the optimizer state sharded
    want = {(6041, 3707, 16, 3): "allreduce", (138494, 26745, 16, 3): "touched", (6041, 3707, 64, 4): "zero1"}
    for (U, I, f, nl), mode in want.items():
        lay = L.layout(U, I, f, nl, "NeuMF-end")
        rng = _active_ranges(NCF(U, I, f, nl, 0.0, "NeuMF-end"), lay)
        ranges = (ctypes.c_int64 * (2 * len(rng)))(*[x for r in rng for x in r])
        got, pf = TrainEngine.auto_dp_mode(lay, ranges, len(rng), 65536)
        assert got == mode, (U, I, pf, int(lay.total))
        # with the owner exchange available: owner for the sparse batch at any world and
        # for every shape from OWNER_MIN_WORLD ranks up
        for world in (2, 4, 8):
            got, _ = TrainEngine.auto_dp_mode(lay, ranges, len(rng), 65536, world, owner_ok=True)
            exp = "owner" if (mode == "touched" or world >= TrainEngine.OWNER_MIN_WORLD) else mode
            assert got == exp, (U, I, world, got)


@pytest.mark.parametrize("bs,k", [(100, 10), (100, 1), (100, 5), (25, 10)])
def test_hr_ndcg_topk_ranking_matches_golden(golden, bs, k):
    """The per-batch torch.topk ranking metrics() uses for loaders ncf_hr_ndcg does not
    take (batches above 1024 rows, unequal batches) against the reference's own
    metrics() output (G6), on CPU tensors."""
    from ncf_amd.metrics import _hr_ndcg_topk
    g = golden("G6_metrics")
    logits = torch.as_tensor(g["logits"])
    items = torch.as_tensor(g["test_pairs"][:, 1], dtype=torch.int32)
    n = items.numel()
    nb = (n + bs - 1) // bs
    hr, nd = _hr_ndcg_topk(logits, items, [bs] * (nb - 1) + [n - (nb - 1) * bs], k)
    assert hr.tolist() == g[f"bs{bs}_k{k}_HR"].tolist()
    np.testing.assert_allclose(nd.numpy(), g[f"bs{bs}_k{k}_NDCG"], rtol=0, atol=0)


def test_layout_tune_launch_geometry():
    """ncf_layout_tune (host logic, no GPU): the fused step runs 8-wave workgroups on
    128-row tiles where a batch has 256 of them, else 4-wave workgroups on 64-row
    tiles (measured faster for C2, C5 and the C3 step at 8,192 rows per rank) where the
    shape has that kernel (the factored kernel and GMF: always; the per-row layer 0:
    where dW0 has at most 8 16x16 tiles); 2 / 1 waves only when forced; the workgroup
    count is the tile count below 256."""
    import ncf_amd._lib as L
    lib = L.hip()

    def tune(U, I, f, nl, rows, waves=0):
        assert lib.ncf_debug_set_geometry(waves) == 0
        try:
            lay = L.layout(U, I, f, nl, "NeuMF-end")
            assert lib.ncf_layout_tune(ctypes.byref(lay), rows) == 0
            g = (lay.flags >> L.LAYOUT_GEO_SHIFT) & L.LAYOUT_GEO_MASK
            return (8, 4, 2, 1)[g], (lay.flags >> L.LAYOUT_WG_SHIFT) & L.LAYOUT_WG_MASK
        finally:
            lib.ncf_debug_set_geometry(0)

    assert tune(6041, 3707, 8, 3, 1024) == (4, 16)         # C2: per-row layer 0, dW0 2 x 4 tiles
    assert tune(6041, 3707, 16, 3, 8192) == (4, 128)       # C3 at N = 8 (factored)
    assert tune(6041, 3707, 16, 3, 65536) == (8, 0)        # C3 at N = 1: 512 tiles -> 256 workgroups
    assert tune(6041, 3707, 16, 3, 32768) == (8, 0)        # 256 tiles of 128 rows
    assert tune(6041, 3707, 16, 3, 32640) == (4, 0)        # 255 tiles of 128 rows: 510 of 64
    assert tune(138494, 26745, 16, 3, 8192) == (8, 64)     # C4 at N = 8: per-row, dW0 4 x 8 tiles
    assert tune(6041, 3707, 8, 3, 1024, waves=8) == (8, 8)
    assert tune(6041, 3707, 8, 3, 1024, waves=1) == (1, 64)
    assert tune(6041, 3707, 8, 3, 8192, waves=2) == (2, 0)
    assert tune(6041, 3707, 16, 3, 8192, waves=2) == (8, 64)  # no 2-wave kernel (weights in 21 registers)
    assert tune(6041, 3707, 16, 3, 65536, waves=4) == (4, 0)
    assert tune(138494, 26745, 16, 3, 8192, waves=1) == (8, 64)  # no 1-wave kernel there
    assert lib.ncf_debug_set_geometry(5) != 0


def test_layout_tune_user_store():
    """NCF_LAYOUT_USER_STORE (the fused step stores its user-side gradient rows and a
    second launch sums them per user over ncf_user_order): never set by default
    (measured slower at C3); with ncf_debug_set_user_store(-1) ncf_layout_tune sets it
    from 16,384 rows per launch up, where the fused path runs and the user order
    exists (user_num <= 32,767), with 1 wherever it applies; the workspace grows by
    (rows + 128, rounded to 64) x ([Um part][Ug part]) floats; ncf_uses_user_order
    follows the flag on the fused path."""
    import ncf_amd._lib as L
    lib = L.hip()

    def tune(U, I, f, nl, rows, mode=-1, mt="NeuMF-end"):
        assert lib.ncf_debug_set_user_store(mode) == 0
        try:
            lay = L.layout(U, I, f, nl, mt)
            assert lib.ncf_layout_tune(ctypes.byref(lay), rows) == 0
            return bool(lay.flags & L.LAYOUT_USER_STORE), lay
        finally:
            lib.ncf_debug_set_user_store(0)

    lay = L.layout(6041, 3707, 16, 3, "NeuMF-end")
    assert lib.ncf_layout_tune(ctypes.byref(lay), 65536) == 0 and not lay.flags & L.LAYOUT_USER_STORE  # default

    assert tune(6041, 3707, 16, 3, 65536)[0]           # C3 at N = 1, 2, 4
    assert tune(6041, 3707, 16, 3, 16384)[0]
    assert not tune(6041, 3707, 16, 3, 8192)[0]        # C3 at N = 8
    assert not tune(6041, 3707, 8, 3, 1024)[0]         # C2
    assert not tune(138494, 26745, 16, 3, 65536)[0]    # C4: no user order above 32,767 users
    assert tune(6041, 3707, 8, 3, 1024, mode=1)[0]
    assert not tune(6041, 3707, 16, 3, 65536, mode=0)[0]
    assert lib.ncf_debug_set_user_store(2) != 0
    on, lay = tune(6041, 3707, 16, 3, 65536)
    off, lay0 = tune(6041, 3707, 16, 3, 65536, mode=0)
    assert lib.ncf_uses_user_order(ctypes.byref(lay)) == 1 and lib.ncf_uses_user_order(ctypes.byref(lay0)) == 0
    extra = lib.ncf_workspace_bytes(ctypes.byref(lay), 65536) - lib.ncf_workspace_bytes(ctypes.byref(lay0), 65536)
    assert extra == 4 * (65536 + 128) * (64 + 16)
    assert not tune(6041, 3707, 32, 3, 65536, mode=1)[0]  # layered path: its own user runs
    for mt, f, nl, uw in (("MLP", 8, 2, 16), ("GMF", 16, 1, 16), ("NeuMF-end", 32, 2, 96), ("NeuMF-end", 64, 1, 128)):
        on, lay = tune(6041, 3707, f, nl, 20000, mt=mt)
        off, lay0 = tune(6041, 3707, f, nl, 20000, mode=0, mt=mt)
        assert on and not off, mt
        extra = lib.ncf_workspace_bytes(ctypes.byref(lay), 20000) - lib.ncf_workspace_bytes(ctypes.byref(lay0), 20000)
        assert extra == 4 * ((20000 + 128 + 63) // 64 * 64) * uw, mt


def test_adam_step_fact_argument_checks():
    """ncf_adam_step_fact (host logic, no GPU launch on these paths): missing pointers
    or an odd bucket size are NCF_E_ARG; a layout without NCF_LAYOUT_FACT_DEFER_DX, a
    per-row layer 0 or a misaligned shard are NCF_E_UNSUPPORTED; the debug switches
    reject values outside their range."""
    import ncf_amd._lib as L
    lib = L.hip()
    lay = L.layout(6041, 3707, 16, 3, "NeuMF-end")
    assert lib.ncf_layout_tune(ctypes.byref(lay), 65536) == 0
    buf = (ctypes.c_float * 64)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    rng = (ctypes.c_int64 * 2)(0, 64)
    ctl = (ctypes.c_int64 * 6)()

    def call(lay_, ws=p, grads=None, gn=0, sb=0, ranges=rng, nr=1):
        return lib.ncf_adam_step_fact(ctypes.byref(lay_), ws, p, p, p, p, ranges, nr, sb, grads, gn,
                                      ctypes.cast(ctl, ctypes.c_void_p), 1e-3, 0.9, 0.999, 1e-8, -1, None, 0, None)
    assert call(lay, ws=None) == L.NCF_E_ARG
    assert call(lay, gn=64) == L.NCF_E_ARG           # a bucket size without the bucket
    assert call(lay, grads=p, gn=6) == L.NCF_E_ARG   # not a multiple of 4
    assert call(lay, nr=0) == L.NCF_E_ARG
    assert call(lay) == L.NCF_E_UNSUPPORTED          # the step did not defer dX
    lay.flags |= L.LAYOUT_FACT_DEFER_DX
    assert call(lay, sb=32) == L.NCF_E_UNSUPPORTED   # shard begin not 64-aligned
    lay.flags |= 0x1                                  # NCF_LAYOUT_PER_ROW_L0: no factored layer 0
    assert call(lay) == L.NCF_E_UNSUPPORTED
    assert lib.ncf_debug_set_per_row(2) != 0 and lib.ncf_debug_set_per_row(-1) == 0
    lay = L.layout(6041, 3707, 16, 3, "NeuMF-end")
    assert lib.ncf_debug_set_per_row(1) == 0
    try:
        assert lib.ncf_layout_tune(ctypes.byref(lay), 65536) == 0 and lay.flags & 0x1
    finally:
        lib.ncf_debug_set_per_row(-1)


def test_sampler_threads_default(monkeypatch):
    """sampler_threads: half the rank's CPU share, at most 12, and at most one thread per
    125,000 positives of the pass (at least 4); NCF_SAMPLER_THREADS overrides."""
    import os
    from ncf_amd.data import sampler_threads
    monkeypatch.delenv("NCF_SAMPLER_THREADS", raising=False)
    monkeypatch.delenv("LOCAL_WORLD_SIZE", raising=False)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(32)))
    assert sampler_threads() == 12
    assert sampler_threads(994_169) == 8          # ml-1m
    assert sampler_threads(19_861_770) == 12      # ml-20m
    assert sampler_threads(1_000) == 4
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")   # 4 CPUs per rank
    assert sampler_threads(994_169) == 2
    monkeypatch.setenv("NCF_SAMPLER_THREADS", "3")
    assert sampler_threads(994_169) == 3


def test_stream_checksum_and_canonical_default():
    """ops.stream_checksum is order-sensitive (ranks holding the same rows in another
    order disagree); EpochPrep / EpochPipeline default to the canonical grouping
    only where torch.distributed runs several ranks (not here)."""
    from ncf_amd import ops
    r = torch.arange(1000, dtype=torch.int64) * 7919 + (1 << 40)
    c0 = int(ops.stream_checksum(r))
    assert c0 == int(ops.stream_checksum(r.clone()))
    assert c0 != int(ops.stream_checksum(r.flip(0)))
    r2 = r.clone()
    r2[[3, 4]] = r2[[4, 3]]
    assert c0 != int(ops.stream_checksum(r2))
    assert ops.default_canonical() is False
    assert ops.EpochPrep("cpu").canonical is False


def test_in_step_adam_kernel_availability():
    """ncf_ais_supported (host logic, no GPU): the fused small-batch geometry with a
    per-row layer 0 has the in-step kernel; the factored C3 shape does not."""
    import ctypes
    import ncf_amd._lib as L
    lib = L.hip()
    small = L.layout(6041, 3707, 8, 2, "MLP")
    assert lib.ncf_layout_tune(ctypes.byref(small), 256) == L.NCF_OK
    assert lib.ncf_ais_supported(ctypes.byref(small)) == 1
    c3 = L.layout(6041, 3707, 16, 3, "NeuMF-end")
    assert lib.ncf_layout_tune(ctypes.byref(c3), 65536) == L.NCF_OK
    assert lib.ncf_ais_supported(ctypes.byref(c3)) == 0


def test_integration_section2_binding_loads_on_cpu():
    """INTEGRATION.md section 2's code blocks exec as written on the CPU (the library
    loads, every argtypes line names a real export); the GPU tests call them."""
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = open(os.path.join(root, "INTEGRATION.md")).read()
    sec = text.split("## 2.", 1)[1].split("\n## 3.", 1)[0]
    blocks = re.findall(r"```python\n(.*?)```", sec, re.S)
    lib = os.path.join(root, "ncf_amd", "libncf_hip.so")
    ns = {}
    for b in blocks:
        exec(compile(b.replace("/path/to/ncf_amd/libncf_hip.so", lib), "INTEGRATION.md", "exec"), ns)
    for fn in ("train_step", "train_steps_ais", "ais_buffers", "distill_step", "train_step_lazy", "flush"):
        assert callable(ns[fn]), fn
    assert len(ns["_lib"].ncf_train_step_ais.argtypes) == 24
