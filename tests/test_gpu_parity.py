"""GPU parity: the HIP path (libncf_hip.so through its C ABI) against the CPU
oracle (oracle/ncf_oracle.py, itself pinned to the reference in test_oracle.py)
and the reference's golden vectors.

Tolerances (north star: "within 1e-5 relative for fp32 loss/logits"):
  * logits / loss: rtol 1e-5 (atol 1e-7 for near-zero logits)
  * one-step gradients: rtol 1e-4 + atol 1e-6*max|g| (summation order differs:
    atomics and MFMA K-order vs ATen's CPU kernels)
  * Adam trajectories: per-step loss rtol 1e-5 over 100 steps; parameters
    rtol 1e-4, atol 1e-6 after 100 steps on the golden (50 x 80) id space;
    at full id spaces (ml-1m multitile, C4 ml-20m): free-running, rtol 1e-4 +
    atol 1e-6*max|p| for >= 90% of every tensor and every element within 4*T*lr
    -- 90% for a free-running 20-step C4 run: two fp32 trajectories drift apart --
    and every step teacher-forced from the
    oracle's state to rtol 1e-5 + atol 5e-3*lr.
  * HR / NDCG: exact.
"""
import numpy as np
import pytest
import torch

from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu

MODEL_TYPES = ["GMF", "MLP", "NeuMF-end", "NeuMF-pre"]
SHAPES = [(8, 3), (16, 3), (8, 1)]
DEV = "cuda:0"


def _models(mt, f, L, U=50, I=80, seed=1, dropout=0.0):
    from ncf_amd.models import NCF
    torch.manual_seed(seed)
    ref = O.OracleNCF(U, I, f, L, dropout, mt)
    torch.manual_seed(seed)
    m = NCF(U, I, f, L, dropout, mt)
    for (k1, v1), (k2, v2) in zip(ref.state_dict().items(), m.state_dict().items()):
        assert k1 == k2 and torch.equal(v1, v2)
    return ref, m.to(DEV)


def _close_grad_rows(got, exp, name, terms, max_rows):
    """_close_grad for an embedding table at large batches, except for at most
    `max_rows` rows: a row whose layer pre-activation sits within fp32 rounding of 0
    takes the other side of a ReLU in one of the two computations (as the fp32 oracle
    itself does against a float64 one -- scripts/diag_fact_rows.py at NCF(64,4),
    65,536 rows: 3 user rows off on each side, disjoint), so its whole gradient row
    differs by that row's contribution -- in a weight gradient, the flipped unit's
    output row."""
    scale = max(float(np.abs(exp).max()), 1e-30)
    atol = (1e-6 if terms is None else max(1e-6, 2e-8 * float(np.sqrt(terms)))) * scale
    bad = np.abs(got - exp) > atol + 1e-4 * np.abs(exp)
    rows = np.unique(np.nonzero(bad.reshape(got.shape[0], -1))[0])
    assert len(rows) <= max_rows, f"{name}: {len(rows)} rows beyond tolerance"
    keep = np.setdiff1d(np.arange(got.shape[0]), rows)
    _close_grad(got[keep], exp[keep], name, terms=terms)


def _close_grad(got, exp, name, terms=None):
    """rtol 1e-4, atol 1e-6 of the largest gradient -- or, for embedding tables whose
    rows sum `terms` per-row contributions in float-atomic (arrival) order, an atol
    growing like the fp32 rounding of such a sum: 2e-8 * sqrt(terms) * max|g|
    (zipf-hot items take ~30K rows of one batch: 3.5e-6 * max|g|)."""
    scale = max(float(np.abs(exp).max()), 1e-30)
    atol = 1e-6 * scale if terms is None else max(1e-6, 2e-8 * float(np.sqrt(terms))) * scale
    np.testing.assert_allclose(got, exp, rtol=1e-4, atol=atol, err_msg=name)


@pytest.mark.parametrize("mt", MODEL_TYPES)
@pytest.mark.parametrize("f,L", SHAPES)
def test_module_forward_backward_vs_golden(golden, mt, f, L):
    g = golden("G4_fwd_bwd")
    tag = f"{mt}_f{f}_L{L}"
    _, m = _models(mt, f, L)
    u = torch.from_numpy(g["users"]).to(DEV)
    i = torch.from_numpy(g["items"]).to(DEV)
    y = torch.from_numpy(g["labels"]).float().to(DEV)
    pred = m(u, i)
    np.testing.assert_allclose(pred.detach().cpu().numpy(), g[f"{tag}_logits"], rtol=1e-5, atol=1e-7)
    loss = torch.nn.BCEWithLogitsLoss()(pred, y)
    np.testing.assert_allclose(loss.item(), float(g[f"{tag}_loss"]), rtol=1e-5)
    loss.backward()
    for k, p in m.named_parameters():
        key = f"{tag}::grad::{k}"
        if key in g.files:
            assert p.grad is not None, k
            _close_grad(p.grad.cpu().numpy(), g[key], k)
        else:
            assert p.grad is None, f"{k} must keep grad None in {mt} mode"


def test_forward_edge_sizes():
    ref, m = _models("NeuMF-end", 16, 3, U=300, I=500, seed=4)
    for n in (1, 15, 127, 128, 129, 1000, 4097):
        rng = np.random.default_rng(n)
        u = rng.integers(0, 300, n)
        i = rng.integers(0, 500, n)
        with torch.no_grad():
            exp = ref(torch.from_numpy(u), torch.from_numpy(i)).numpy()
            got = m(torch.from_numpy(u).to(DEV), torch.from_numpy(i).to(DEV)).cpu().numpy()
        np.testing.assert_allclose(got, exp, rtol=1e-5, atol=1e-7)


def _engine_for(mt, f, L, U, I, seed, optimizer="adam", lr=1e-3, dropout=0.0):
    from ncf_amd.engine import TrainEngine
    ref, m = _models(mt, f, L, U=U, I=I, seed=seed, dropout=dropout)
    eng = TrainEngine(m, lr=lr, optimizer=optimizer)
    return ref, m, eng


def _stream(eng, users, items, labels, bs):
    u = torch.as_tensor(np.asarray(users).reshape(-1), dtype=torch.int32, device=DEV).contiguous()
    i = torch.as_tensor(np.asarray(items).reshape(-1), dtype=torch.int32, device=DEV).contiguous()
    y = torch.as_tensor(np.asarray(labels).reshape(-1), dtype=torch.float32, device=DEV).contiguous()
    from ncf_amd import ops
    eng.set_epoch_stream(ops.pack_rows(u, i, y), bs)


@pytest.mark.parametrize("mt,opt", [("NeuMF-end", "adam"), ("GMF", "adam"), ("MLP", "adam"), ("NeuMF-end", "sgd")])
@pytest.mark.parametrize("use_graph", [False, True])
def test_engine_trajectory_vs_golden(golden, mt, opt, use_graph):
    g = golden("G5_steps")
    T = 100 if opt == "adam" else 10
    ref, m, eng = _engine_for(mt, 8, 3, 50, 80, 3, optimizer=opt, lr=1e-3 if opt == "adam" else 1e-2)
    _stream(eng, g["users"][:T], g["items"][:T], g["labels"][:T], 256)
    eng.run(T, use_graph=use_graph)
    torch.cuda.synchronize()
    np.testing.assert_allclose(eng.epoch_losses()[:T], g[f"{mt}_{opt}_losses"][:T], rtol=1e-5)
    sd = m.state_dict()
    for k, v in sd.items():
        np.testing.assert_allclose(v.cpu().numpy(), g[f"{mt}_{opt}_t{T}::{k}"], rtol=1e-4, atol=1e-6, err_msg=k)
    assert eng.state_step() == T


ONE_STEP = {  # name: (model_type, f, L, B, expected path)
    "C2": ("NeuMF-end", 8, 3, 1024, 1), "C3": ("NeuMF-end", 16, 3, 8192, 1),
    "default": ("NeuMF-end", 32, 2, 4096, 1),
    # > 256 tiles of 128 rows: every workgroup of the fused kernel runs 2-3 tiles
    # (alternating staging halves, no tile-end barrier, prefetch across tiles)
    "C3-multitile": ("NeuMF-end", 16, 3, 65536 + 3000, 1), "C2-multitile": ("NeuMF-end", 8, 3, 40000, 1),
    "mlp-multitile": ("MLP", 16, 2, 50000, 1), "gmf-multitile": ("GMF", 16, 1, 70000, 1),
    # layered path: tower too large for LDS, or factor_num without a fused kernel
    "cli-default-32x3": ("NeuMF-end", 32, 3, 4096, 2), "stress-64x4": ("NeuMF-end", 64, 4, 1000, 2),
    "odd-f6": ("NeuMF-end", 6, 3, 3001, 2), "mlp-f11": ("MLP", 11, 2, 777, 2),
    "gmf-f5": ("GMF", 5, 1, 2000, 2), "pre-f12": ("NeuMF-pre", 12, 2, 513, 2),
    "mlp-f1": ("MLP", 1, 1, 300, 2),
}


def _fact_mode(lay):
    from ncf_amd import ops
    return ops.fact_mode(lay)


def _one_step(mt, f, Lyr, B, U, I, seed=11, zipf=1.3, flags=0, order=False, data_seed=3):
    """Logits, loss and every gradient of one fused step vs the oracle.  flags: OR-ed
    into a copy of the layout (e.g. NCF_LAYOUT_PER_ROW_L0); order: pass the batch's
    ncf_user_order to the step."""
    import ncf_amd._lib as L
    from ncf_amd import ops
    ref, m = _models(mt, f, Lyr, U=U, I=I, seed=seed)
    rng = np.random.default_rng(data_seed)
    users = rng.integers(0, U, B)
    items = np.minimum(rng.zipf(zipf, B) - 1, I - 1)  # hot items: heavy atomic contention
    labels = (rng.random(B) < 0.2).astype(np.int64)
    users = _untie(ref, users, items, U, rng)  # a draw without ReLU ties
    logits_ref, loss_ref, grads_ref = O.forward_backward(ref, users, items, labels)
    flat, lay = ops.ensure_flat(m)
    if flags:
        lay = type(lay).from_buffer_copy(lay)
        lay.flags |= flags
    gflat = torch.zeros(int(lay.total), device=DEV)
    ws = ops.new_workspace(lay, B, DEV)
    ctl = ops.new_ctl(B, DEV)
    u = torch.as_tensor(users, dtype=torch.int32, device=DEV)
    it = torch.as_tensor(items, dtype=torch.int32, device=DEV)
    y = torch.as_tensor(labels, dtype=torch.float32, device=DEV)
    logits = torch.empty(B, device=DEV)
    st = L.stream_ptr()
    rows = ops.pack_rows(u, it, y)
    uord = None
    if order:
        uord = torch.empty(B + (B + 1) // 2, dtype=torch.int64, device=DEV)  # entries + int32 inverse
        L.check(L.hip().ncf_user_order(rows.data_ptr(), B, B, 1, U, uord.data_ptr(), st), "order")
    L.check(L.hip().ncf_train_step(L.ctypes.byref(lay), flat.data_ptr(), gflat.data_ptr(), rows.data_ptr(),
                                   None if uord is None else uord.data_ptr(), None, ctl.data_ptr(), B, 1, 0,
                                   L.DZ_BCE, ws.data_ptr(), ws.numel() * 4, logits.data_ptr(), st), "train")
    L.check(L.hip().ncf_reduce_slab(L.ctypes.byref(lay), ws.data_ptr(), gflat.data_ptr(), ctl.data_ptr(), st), "reduce")
    torch.cuda.synchronize()
    np.testing.assert_allclose(logits.cpu().numpy(), logits_ref.numpy(), rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(gflat[lay.loss_slot].item(), loss_ref, rtol=1e-5)
    fact = ops.fact_mode(lay)
    for (p, off), (name, _) in zip(ops._segments(m, lay), m.named_parameters()):
        got = gflat[off:off + p.numel()].view_as(p).cpu().numpy()
        if name in grads_ref:
            hot = int(np.bincount(items).max()) if "item" in name else int(np.bincount(users).max())
            if fact and name == "MLP_layers.1.weight":
                # factored layer 0: dW0 = sum_u G_u^T Um[u] (+ items), G_u summed by float
                # atomics in arrival order -- the embedding tables' rounding model
                hot = max(int(np.bincount(items).max()), int(np.bincount(users).max()))
                if B >= 65536:
                    _close_grad_rows(got, grads_ref[name].numpy(), name, hot, max_rows=8)
                else:
                    _close_grad(got, grads_ref[name].numpy(), name, terms=hot)
                continue
            if B >= 65536:  # a bias: its flipped units' entries
                e = grads_ref[name].numpy()
                _close_grad_rows(got.reshape(len(got), -1), e.reshape(len(e), -1), name,
                                 hot if "embed" in name else None, max_rows=8)
                continue
            _close_grad(got, grads_ref[name].numpy(), name, terms=hot if "embed" in name else None)
        else:  # unused in this model type (reference grad None): nothing may be written
            assert not got.any(), name
    return lay


@pytest.mark.parametrize("mt,f,Lyr,B", [("NeuMF-end", 16, 3, 65536),  # C3 (factored layer 0)
                                         ("NeuMF-end", 16, 3, 8192),   # C3 at N = 8
                                         ("NeuMF-end", 8, 3, 1024),    # C2 (per-row layer 0, DM 32)
                                         ("NeuMF-end", 8, 2, 4096),    # per-row, DM 16
                                         ("NeuMF-end", 8, 1, 3000),    # per-row, DM 8
                                         ("NeuMF-end", 32, 2, 8192),   # uw 96: two column chunks
                                         ("NeuMF-end", 64, 1, 20000),  # uw 128
                                         ("MLP", 8, 2, 4096), ("GMF", 16, 1, 3000)])
def test_one_step_user_store_vs_oracle(mt, f, Lyr, B):
    """NCF_LAYOUT_USER_STORE: the step stores every row's user-side gradient (Um and Ug
    parts) into the workspace and user_sum_kernel adds each run of the user order
    (pieces of 32 positions) into the user rows -- every gradient vs the oracle at
    ml-1m ids on the tuned layout with the flag forced on, hot (zipf) items."""
    import ncf_amd._lib as L
    from ncf_amd import ops
    U, I = 6041, 3707
    _, m = _models(mt, f, Lyr, U=U, I=I, seed=11)
    lay = type(ops.ensure_flat(m)[1]).from_buffer_copy(ops.ensure_flat(m)[1])
    L.check(L.hip().ncf_layout_tune(L.ctypes.byref(lay), B), "tune")
    lay = _one_step(mt, f, Lyr, B, U, I, flags=int(lay.flags) | L.LAYOUT_USER_STORE, order=True)
    assert L.hip().ncf_uses_user_order(L.ctypes.byref(lay)) == 1


@pytest.mark.parametrize("B,store", [(4096, 1), (20000, -1), (20000, 0)])
def test_engine_user_store_trajectory_vs_oracle(B, store):
    """The engine with the user store-and-sum (an option, off by default: forced on at
    4,096 rows; by the tune rule at 20,000, and off) over 6 graph-replayed steps of
    NCF(16,3) at ml-1m ids: losses vs the oracle's trajectory, then every step
    teacher-forced."""
    import ncf_amd._lib as L
    assert L.hip().ncf_debug_set_user_store(store) == 0
    try:
        T = 6
        ref, m, eng = _engine_for("NeuMF-end", 16, 3, 6041, 3707, 23)
        rng = np.random.default_rng(47)
        users = rng.integers(0, 6041, (T, B))
        items = np.minimum(rng.zipf(1.3, (T, B)) - 1, 3706)
        labels = (rng.random((T, B)) < 0.2).astype(np.int64)
        _stream(eng, users, items, labels, B)
        assert bool(eng.lay.flags & L.LAYOUT_USER_STORE) == (store != 0)
        assert eng.user_order_ptr() is not None or store == 0
        ref0 = {k: v.clone() for k, v in ref.state_dict().items()}
        eng.run(T, use_graph=True)
        torch.cuda.synchronize()
        got_losses = eng.epoch_losses()[:T].copy()
        opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
        np.testing.assert_allclose(got_losses, O.train_steps(ref, opt, users, items, labels), rtol=1e-5)
        ref.load_state_dict(ref0)
        _teacher_forced_steps(ref, m, eng, users, items, labels)
    finally:
        L.hip().ncf_debug_set_user_store(0)


@pytest.mark.parametrize("waves", [8, 4, 2, 1])
@pytest.mark.parametrize("mt,f,Lyr,B,U,I", [("NeuMF-end", 8, 3, 1024, 6041, 3707),     # C2 (per-row layer 0)
                                            ("NeuMF-end", 16, 3, 8192, 6041, 3707),    # C3 at N = 8 (factored)
                                            ("MLP", 8, 2, 256, 6041, 3707),            # C5 student
                                            ("GMF", 16, 1, 3000, 6041, 3707),
                                            ("NeuMF-end", 16, 3, 20000, 138494, 26745)])  # C4 ids, per-row
def test_one_step_tuned_geometry_vs_oracle(mt, f, Lyr, B, U, I, waves, geometry):
    """One step on the layout ncf_layout_tune shapes for B rows, with 8-, 4-, 2- and
    1-wave workgroups forced (the NCF_LAYOUT_GEO field: 128 / 64 / 32 / 16-row tiles;
    where the shape has no narrow kernel -- per-row layer 0 with more than 8 dW0
    tiles -- the 8-wave one runs)."""
    import ncf_amd._lib as L
    from ncf_amd import ops
    geometry(waves)
    _, m = _models(mt, f, Lyr, U=U, I=I, seed=11)
    lay = type(ops.ensure_flat(m)[1]).from_buffer_copy(ops.ensure_flat(m)[1])
    L.check(L.hip().ncf_layout_tune(L.ctypes.byref(lay), B), "tune")
    _one_step(mt, f, Lyr, B, U, I, flags=int(lay.flags))


@pytest.mark.parametrize("cfg", list(ONE_STEP))
def test_one_step_grads_vs_oracle(cfg):
    """Full-size id spaces (ml-1m): logits, loss and every gradient of one step."""
    import ncf_amd._lib as L
    mt, f, Lyr, B, path = ONE_STEP[cfg]
    assert L.supported(mt, f, Lyr) == path
    _one_step(mt, f, Lyr, B, 6041, 3707)


# C4 (ml-20m-shaped 138,494 x 26,745): U + I > FACT_MAX_ROWS, so the fused
# kernel forms the layer-0 gradients per row (ncf_step_kernel<..., FACT = false>).
C4_U, C4_I = 138494, 26745


@pytest.mark.parametrize("mt,B", [("NeuMF-end", 8192), ("NeuMF-end", 65536), ("MLP", 8192)])
def test_one_step_c4_id_space_per_row_layer0(mt, B):
    lay = _one_step(mt, 16, 3, B, C4_U, C4_I, seed=13, zipf=1.2)
    assert not _fact_mode(lay)


@pytest.mark.parametrize("U,I,fact", [(16384, 16384, True), (16384, 16385, False)])
def test_one_step_fact_boundary(U, I, fact):
    """Both sides of fact_mode (U + I <= 32768, ncf_ops.hip): the factored and the
    per-row layer-0 kernels give the same gradients."""
    lay = _one_step("NeuMF-end", 16, 3, 8192, U, I, seed=14)
    assert _fact_mode(lay) == fact


@pytest.mark.parametrize("mt,f,Lyr,B", [("NeuMF-end", 32, 3, 65536), ("NeuMF-end", 32, 3, 8192),
                                        ("MLP", 32, 3, 8192), ("NeuMF-end", 16, 4, 8192),
                                        # forward-chain instantiations dm 16 / L 3, dm 8 / L 2, dm 128 / L 1
                                        ("NeuMF-end", 4, 3, 8192), ("MLP", 4, 2, 8192),
                                        ("NeuMF-end", 128, 1, 8192),
                                        # dm 512 / 256: expansion by GEMMs (lyr_fact_dx / dw0), W0 via the slab
                                        ("NeuMF-end", 64, 4, 8192), ("MLP", 32, 4, 8192),
                                        # 128-row block tiles of the per-layer GEMMs (R >= 65,536)
                                        ("NeuMF-end", 64, 4, 65536)])
def test_one_step_layered_factored_layer0(mt, f, Lyr, B):
    """Layered path with the factored layer 0 (ABI 10: table projections through W0,
    per-row gather, D0 row sums expanded by fact_expand_kernel; dm = 128 for
    NCF(32,3) and NCF(16,4)) at ml-1m ids, with and without the user order (ABI 12:
    user runs summed before the atomics), and the same shape forced per-row
    (NCF_LAYOUT_PER_ROW_L0): all vs the oracle."""
    import ncf_amd._lib as L
    assert L.supported(mt, f, Lyr) == L.PATH_LAYERED
    # Below 65,536 rows the comparison allows no ReLU-flip row (a unit whose
    # pre-activation is within fp32 rounding of 0 landing on the other side, which
    # moves that row's whole gradient): _one_step redraws the samples with a
    # pre-activation within 1e-6 of a kink (_untie), since at 8,192 rows the f32-MFMA
    # and the bf16-split GEMM cores flip on as many (seed, data) draws -- NCF(64,4)
    # 5 / 12 each, MLP(32,4) 3 / 12 and 4 / 12 (profiles/r03x6/flip_sweep.json,
    # scripts/diag_fact_rows.py).
    sd, dd = (23, 7) if (mt, f, Lyr) == ("MLP", 32, 4) else (19, 3)
    lay = _one_step(mt, f, Lyr, B, 6041, 3707, seed=sd, data_seed=dd)
    assert _fact_mode(lay)
    assert L.hip().ncf_uses_user_order(L.ctypes.byref(lay)) == 1
    _one_step(mt, f, Lyr, B, 6041, 3707, seed=sd, order=True, data_seed=dd)
    lay = _one_step(mt, f, Lyr, min(B, 8192), 6041, 3707, seed=sd, flags=L.LAYOUT_PER_ROW_L0, data_seed=dd)
    assert not _fact_mode(lay)


@pytest.mark.parametrize("f,Lyr,T", [(32, 3, 6), (64, 4, 4)])
def test_engine_layered_factored_trajectory_vs_oracle(f, Lyr, T):
    """NCF(32,3) (the CLI default shape: step chain, LDS expansion) and NCF(64,4) (the
    stress shape: dm 512, GEMM expansion, W0 reduced from the slab by
    ncf_reduce_adam_step) on the factored layered path at ml-1m ids: T engine Adam
    steps of 8,192 rows (hipGraph) free-running (_assert_trajectory_close), then every
    step teacher-forced."""
    B = 8192
    ref, m, eng = _engine_for("NeuMF-end", f, Lyr, 6041, 3707, 23)
    rng = np.random.default_rng(47)
    users = rng.integers(0, 6041, (T, B))
    items = np.minimum(rng.zipf(1.3, (T, B)) - 1, 3706)
    labels = (rng.random((T, B)) < 0.2).astype(np.int64)
    _stream(eng, users, items, labels, B)
    assert _fact_mode(eng.lay)
    ref0 = {k: v.clone() for k, v in ref.state_dict().items()}
    eng.run(T, use_graph=True)
    torch.cuda.synchronize()
    got_losses = eng.epoch_losses()[:T].copy()
    got = {k: v.cpu().numpy().copy() for k, v in m.state_dict().items()}
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    np.testing.assert_allclose(got_losses, O.train_steps(ref, opt, users, items, labels), rtol=1e-5)
    for k, r in ref.state_dict().items():
        _assert_trajectory_close(got[k], r.numpy(), T, 1e-3, k)
    ref.load_state_dict(ref0)
    _teacher_forced_steps(ref, m, eng, users, items, labels)


def _assert_trajectory_close(got, exp, T, lr, name, off_max=0.10):
    """Parameters after T free-running Adam steps.  Two correct fp32 trajectories
    drift apart: Adam turns the summation-order noise of a near-zero gradient into
    up to ~lr of movement, and the drifted parameters later flip ReLU mask bits of
    pre-activations near the kink, which moves a whole embedding row differently.
    So: every element within 4 * T * lr, at most 10% of a tensor outside rtol 1e-4 +
    atol 1e-6 * max|p| (C4, 20 steps: up to ~4% of the first tower weight drifts
    past that); the step-by-step check that catches a wrong update is
    _teacher_forced_steps."""
    got = np.asarray(got, dtype=np.float64)
    exp = np.asarray(exp, dtype=np.float64)
    dev = np.abs(got - exp)
    tol = 1e-4 * np.abs(exp) + 1e-6 * max(float(np.abs(exp).max()), 1e-30)
    off = dev > tol
    info = f"{name}: max dev {dev.max(initial=0.0):.3g}, {off.mean():.5f} of elements off"
    assert float(dev.max(initial=0.0)) <= 4 * T * lr, info
    assert off.mean() <= off_max, info


def _untie(ref, users, items, U, rng, tau=1e-6, rounds=20):
    """users with every sample whose tower pre-activation lies within `tau` of a ReLU
    kink (_tie_mask) redrawn until none does.  At such a sample two correct fp32
    computations (MFMA K order vs ATen's CPU GEMM, ~1e-8 apart) may take different
    mask bits, which moves that sample's whole gradient -- in a deeper layer every row
    of the layer-0 weight gradient; whether a draw has one is chance and depends on the
    GEMM core (NCF(64,4) at 8,192 rows: 5 / 12 draws flip, profiles/r03x6/flip_sweep.json).
    Away from the kinks the step is continuous, so the comparison stays element-wise."""
    users = np.array(users, copy=True)
    for _ in range(rounds):
        near = _tie_mask(ref, users, items, tau)
        if not near.any():
            return users
        users[near] = rng.integers(0, U, int(near.sum()))
    raise AssertionError("no tie-free draw")


def _tie_mask(ref, users, items, tau):
    pres = []
    hs = [mm.register_forward_hook(lambda mod, i, o: pres.append(o.detach())) for mm in ref.MLP_layers
          if isinstance(mm, torch.nn.Linear)]
    with torch.no_grad():
        ref(torch.as_tensor(users), torch.as_tensor(items))
    for h in hs:
        h.remove()
    if not pres:
        return np.zeros(len(users), dtype=bool)
    return (torch.stack([p.abs().min(dim=1).values for p in pres]).min(dim=0).values < tau).numpy()


def _relu_ties(ref, users, items, tau=1e-7):
    """Samples of a batch with a tower pre-activation within `tau` of the ReLU kink
    at the oracle's current parameters: there the two summation orders (MFMA
    K-order vs ATen's CPU GEMM, ~1e-8 apart at these scales) may pick different
    mask bits -- both correct to fp32 -- and that sample's gradient changes
    discontinuously.  Returns (users, items) of those samples."""
    pres = []
    hs = [mm.register_forward_hook(lambda mod, i, o: pres.append(o.detach())) for mm in ref.MLP_layers
          if isinstance(mm, torch.nn.Linear)]
    with torch.no_grad():
        ref(torch.as_tensor(users), torch.as_tensor(items))
    for h in hs:
        h.remove()
    if not pres:
        return set(), set()
    near = (torch.stack([p.abs().min(dim=1).values for p in pres]).min(dim=0).values < tau).numpy()
    return set(np.asarray(users)[near].tolist()), set(np.asarray(items)[near].tolist())


def _teacher_forced_steps(ref, m, eng, users, items, labels, lr=1e-3):
    """Every step of an Adam trajectory, checked from the oracle's own state: before
    step t the engine gets the oracle's parameters and Adam moments (and step count),
    runs one fused step (graph off) on batch t, and the loss must match to rtol
    1e-5 and the parameters the oracle's after step t to rtol 1e-5 + atol 5e-3 * lr
    (one Adam step from the same state: only the summation order differs).  The
    exceptions are the discontinuities of ReLU ties (_relu_ties): embedding rows of
    the tied samples' users / items, and at most 1% of a tower tensor (their
    rank-one share of the tower gradients) when the step has a tie -- each element
    within 2 * lr, one Adam step's largest change.  A wrong-row update, stale
    staging or a bad moment fails at the step it happens."""
    from ncf_amd import ops
    opt = torch.optim.Adam(ref.parameters(), lr=lr)
    segs = ops._segments(m, eng.lay)
    params = dict(ref.named_parameters())
    ties = 0
    for t in range(len(users)):
        with torch.no_grad():
            for (p, off), (k, rp) in zip(segs, params.items()):
                n = rp.numel()
                eng.flat[off:off + n].copy_(rp.detach().reshape(-1))
                st = opt.state.get(rp, {})
                eng.exp_avg[off:off + n].copy_(st["exp_avg"].reshape(-1) if st else torch.zeros(n))
                eng.exp_avg_sq[off:off + n].copy_(st["exp_avg_sq"].reshape(-1) if st else torch.zeros(n))
        tie_u, tie_i = _relu_ties(ref, users[t], items[t])
        ties += len(tie_u)
        eng.ctl[0] = t
        eng.ctl[1] = t
        eng.optimizer_state_set()  # deferred Adam: every row current as of step t
        eng.run(1, use_graph=False)
        losses = O.train_steps(ref, opt, [users[t]], [items[t]], [labels[t]])
        torch.cuda.synchronize()
        np.testing.assert_allclose(eng.epoch_losses()[t], losses[0], rtol=1e-5, err_msg=f"loss step {t}")
        for (p, off), (k, rp) in zip(segs, params.items()):
            got = eng.flat[off:off + p.numel()].view_as(p).cpu().numpy().astype(np.float64)
            exp = rp.detach().numpy().astype(np.float64)
            dev = np.abs(got - exp)
            off_ = dev > 1e-5 * np.abs(exp) + 5e-3 * lr
            if not off_.any():
                continue
            where = f"{k} after step {t}: {int(off_.sum())} elements off, max {dev.max():.3g}"
            assert dev.max() <= 2 * lr, where
            if k.startswith("embed"):
                rows = set(np.flatnonzero(off_.any(axis=1)).tolist())
                unexplained = sorted(rows - (tie_u if "user" in k else tie_i))
                assert not unexplained, f"{where}; rows with no ReLU tie: {unexplained[:10]}"
            else:
                assert (tie_u or tie_i) and off_.mean() <= 0.01, where
    return ties


def test_engine_trajectory_c4_id_space():
    """20 engine Adam steps (hipGraph) at the C4 id space vs torch.optim.Adam on the
    oracle: free-running per-step loss rtol 1e-5 and parameters per
    _assert_trajectory_close, then every step teacher-forced (_teacher_forced_steps)."""
    T, B = 20, 16384
    ref, m, eng = _engine_for("NeuMF-end", 16, 3, C4_U, C4_I, 15)
    rng = np.random.default_rng(41)
    users = rng.integers(0, C4_U, (T, B))
    items = np.minimum(rng.zipf(1.2, (T, B)) - 1, C4_I - 1)
    labels = (rng.random((T, B)) < 0.2).astype(np.int64)
    _stream(eng, users, items, labels, B)
    assert not _fact_mode(eng.lay)
    eng.run(T, use_graph=True)
    torch.cuda.synchronize()
    got_losses = eng.epoch_losses()[:T].copy()
    got = {k: v.cpu().numpy().copy() for k, v in m.state_dict().items()}
    ref0 = {k: v.clone() for k, v in ref.state_dict().items()}
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    losses = O.train_steps(ref, opt, users, items, labels)
    np.testing.assert_allclose(got_losses, losses, rtol=1e-5)
    for k, r in ref.state_dict().items():
        _assert_trajectory_close(got[k], r.numpy(), T, 1e-3, k)
    ref.load_state_dict(ref0)
    _teacher_forced_steps(ref, m, eng, users, items, labels)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("f,Lyr", [(16, 3), (32, 3)])
def test_rank_shards_sum_to_full_batch(world, f, Lyr):
    """DP decomposition: sum over ranks of shard grads == single-device grads."""
    import ncf_amd._lib as L
    from ncf_amd import ops
    U, I, B = 6041, 3707, 3000
    _, m = _models("NeuMF-end", f, Lyr, U=U, I=I, seed=5)
    flat, lay = ops.ensure_flat(m)
    rng = np.random.default_rng(9)
    u = torch.as_tensor(rng.integers(0, U, B), dtype=torch.int32, device=DEV)
    it = torch.as_tensor(rng.integers(0, I, B), dtype=torch.int32, device=DEV)
    y = torch.as_tensor((rng.random(B) < 0.2), dtype=torch.float32, device=DEV)
    st = L.stream_ptr()
    rows = ops.pack_rows(u, it, y)

    def run(world, rank):
        gflat = torch.zeros(int(lay.total), device=DEV)
        ws = ops.new_workspace(lay, (B + world - 1) // world, DEV)
        ctl = ops.new_ctl(B, DEV)
        # the rank slices' user order (used where ncf_uses_user_order: NCF(32,3))
        uord = torch.empty(B + (B + 1) // 2, dtype=torch.int64, device=DEV)  # entries + int32 inverse
        L.check(L.hip().ncf_user_order(rows.data_ptr(), B, B, world, U, uord.data_ptr(), st), "order")
        L.check(L.hip().ncf_train_step(L.ctypes.byref(lay), flat.data_ptr(), gflat.data_ptr(), rows.data_ptr(),
                                       uord.data_ptr(), None, ctl.data_ptr(), B, world, rank, L.DZ_BCE,
                                       ws.data_ptr(), ws.numel() * 4, None, st), "train")
        L.check(L.hip().ncf_reduce_slab(L.ctypes.byref(lay), ws.data_ptr(), gflat.data_ptr(), ctl.data_ptr(), st), "reduce")
        return gflat
    full = run(1, 0)
    parts = sum(run(world, r) for r in range(world))
    torch.cuda.synchronize()
    d = (parts - full).abs().max().item()
    assert d <= 1e-6 * full.abs().max().item() + 1e-9, d


@pytest.mark.parametrize("bs,k", [(100, 10), (100, 1), (100, 5), (25, 10)])
def test_hr_ndcg_vs_golden(golden, bs, k):
    import ncf_amd._lib as L
    g = golden("G6_metrics")
    logits = torch.as_tensor(g["logits"], device=DEV)
    items = torch.as_tensor(g["test_pairs"][:, 1], dtype=torch.int32, device=DEV)
    n = items.numel()
    nb = (n + bs - 1) // bs
    hr = torch.empty(nb, dtype=torch.int32, device=DEV)
    nd = torch.empty(nb, dtype=torch.float32, device=DEV)
    L.check(L.hip().ncf_hr_ndcg(logits.data_ptr(), items.data_ptr(), n, bs, k, hr.data_ptr(), nd.data_ptr(),
                                L.stream_ptr()), "hr")
    torch.cuda.synchronize()
    assert hr.cpu().tolist() == g[f"bs{bs}_k{k}_HR"].tolist()
    np.testing.assert_allclose(nd.cpu().numpy(), g[f"bs{bs}_k{k}_NDCG"], rtol=1e-6)


def test_metrics_unequal_and_large_loader_batches():
    """metrics() on loaders the ranking kernel does not take -- a batch_sampler of
    unequal batches, and 2,000-row batches -- equals the reference's per-batch loop
    (metrics.py:4-25) run on the same model's per-batch forward."""
    from ncf_amd.metrics import _metrics_cpu, metrics
    from ncf_amd.models import NCF
    torch.manual_seed(5)
    gpu = NCF(300, 500, 8, 2, 0.0, "NeuMF-end").to(DEV)

    class PerBatch(torch.nn.Module):  # the reference loop's model(user, item), on the device
        def forward(self, u, i):
            return gpu(u.to(DEV), i.to(DEV)).cpu()
    cpu = PerBatch()
    rng = np.random.default_rng(2)
    n = 6000
    ds = torch.utils.data.TensorDataset(torch.as_tensor(rng.integers(0, 300, n)), torch.as_tensor(rng.integers(0, 500, n)),
                                        torch.zeros(n, dtype=torch.int64))
    cuts = np.cumsum([0] + [int(x) for x in rng.integers(20, 140, 200)])
    cuts = cuts[cuts < n].tolist() + [n]
    ragged = [list(range(a, b)) for a, b in zip(cuts, cuts[1:])]
    for loader in (torch.utils.data.DataLoader(ds, batch_sampler=ragged),
                   torch.utils.data.DataLoader(ds, batch_size=2000, shuffle=False)):
        hr, nd = metrics(gpu, loader, 10)
        hr_ref, nd_ref = _metrics_cpu(cpu, loader, 10)
        assert hr == hr_ref
        np.testing.assert_allclose(nd, nd_ref, rtol=1e-12)


def test_hr_ndcg_short_batch_raises(golden):
    import ncf_amd._lib as L
    g = golden("G6_metrics")
    logits = torch.as_tensor(g["logits"], device=DEV)
    items = torch.as_tensor(g["test_pairs"][:, 1], dtype=torch.int32, device=DEV)
    hr = torch.empty(10000, dtype=torch.int32, device=DEV)
    nd = torch.empty(10000, dtype=torch.float32, device=DEV)
    assert L.hip().ncf_hr_ndcg(logits.data_ptr(), items.data_ptr(), items.numel(), 7, 10, hr.data_ptr(),
                               nd.data_ptr(), L.stream_ptr()) == L.NCF_E_ARG


def _rand_rows(rng, n, n_users, n_items, pos_frac=0.3, hot=None):
    from ncf_amd import ops
    u = rng.integers(0, n_users, n)
    i = rng.integers(0, n_items, n)
    if hot is not None:  # fraction of rows on item 0: one item group larger than a part
        i[rng.random(n) < hot] = 0
    y = rng.random(n) < pos_frac
    return torch.as_tensor(ops.pack_rows_host(u, i, y), device=DEV)


def test_pack_rows_matches_host_packing():
    from ncf_amd import ops
    rng = np.random.default_rng(1)
    n = 4099
    u, i = rng.integers(0, 2**31 - 1, n), rng.integers(0, 2**31 - 1, n)
    y = (rng.random(n) < 0.5).astype(np.float32)
    got = ops.pack_rows(torch.as_tensor(u, dtype=torch.int32, device=DEV),
                        torch.as_tensor(i, dtype=torch.int32, device=DEV),
                        torch.as_tensor(y, device=DEV)).cpu().numpy()
    assert np.array_equal(got, ops.pack_rows_host(u, i, y))


def test_gather_epoch():
    import ncf_amd._lib as L
    n = 10007
    rows = _rand_rows(np.random.default_rng(0), n, 100, 100)
    perm = torch.randperm(n, device=DEV)
    out = torch.empty_like(rows)
    L.check(L.hip().ncf_gather_epoch(rows.data_ptr(), perm.data_ptr(), n, out.data_ptr(), L.stream_ptr()), "gather")
    assert torch.equal(out, rows[perm])


# (rows, batch, items, hot-item fraction): one part (B <= 8192), 8 and 16 parts with
# XCD-grouped blocks, a partial last batch, item ranges above the LDS offset table
# (global offsets), an item group above the LDS staging buffer (direct writes),
# the reference's batch_size=256, odd batch sizes, one item.
PREP_CASES = [(10007, 1000, 37, None), (65536 * 2 + 123, 65536, 3707, None), (5000, 5000, 1, None),
              (131072 + 77, 131072, 3707, None), (70001, 65536, 100000, None), (70001, 65536, 3707, 0.4),
              (20000, 256, 3707, None), (99999, 33333, 999, 0.05)]


def _canon_keys(r):
    r = r.astype(np.uint64)
    return (((r >> np.uint64(32)) & np.uint64(0x7FFFFFFF)) << np.uint64(33)) | \
        ((r & np.uint64(0xFFFFFFFF)) << np.uint64(1)) | (r >> np.uint64(63))


@pytest.mark.parametrize("canonical", [False, True])
@pytest.mark.parametrize("n,bs,n_items,hot", PREP_CASES)
def test_prepare_epoch_batches_grouped_by_item(n, bs, n_items, hot, canonical):
    """Per batch: same rows as the plain shuffle (DataLoader membership), grouped by
    item; canonical (NCF_PREP_CANONICAL, data parallelism): exactly the batch's rows
    sorted by (item, user, label) -- staged parts and a hot item's part beyond the LDS
    stage (hot 0.4) alike -- so every rank building the stream gets the same one."""
    from ncf_amd import ops
    rng = np.random.default_rng(n + bs)
    rows = _rand_rows(rng, n, 500, n_items, hot=hot)
    perm = torch.randperm(n, device=DEV)
    prep = ops.EpochPrep(DEV, canonical=canonical)
    out = prep(rows, perm, bs, n_items)
    torch.cuda.synchronize()
    exp = rows[perm].cpu().numpy()
    got = out.cpu().numpy()
    for b0 in range(0, n, bs):
        sl = slice(b0, min(n, b0 + bs))
        gi = (got[sl] >> 32) & 0x7FFFFFFF
        if bs >= 4096:  # smaller batches are shuffled only (include/ncf_hip.h)
            assert (np.diff(gi) >= 0).all(), "batch not grouped by item"
            if canonical:
                e = exp[sl]
                assert np.array_equal(got[sl], e[np.argsort(_canon_keys(e), kind="stable")]), "not canonical"
        else:
            assert np.array_equal(got[sl], exp[sl])
        assert np.array_equal(np.sort(exp[sl]), np.sort(got[sl])), "batch membership changed"
    # second epoch through the same workspace: identical multiset per batch again
    perm2 = torch.randperm(n, device=DEV)
    out2 = prep(rows, perm2, bs, n_items).cpu().numpy()
    exp2 = rows[perm2].cpu().numpy()
    for b0 in range(0, n, bs):
        sl = slice(b0, min(n, b0 + bs))
        assert np.array_equal(np.sort(exp2[sl]), np.sort(out2[sl]))


@pytest.mark.parametrize("n,bs,world,users", [(65536 * 2 + 123, 65536, 1, 6040), (70001, 65536, 3, 6040),
                                              (10007, 1000, 2, 1), (5000, 4096, 4, 32767), (99, 7, 5, 50)])
def test_user_order_sorts_each_rank_slice(n, bs, world, users):
    """ncf_user_order: in every rank slice of every batch (the partial last batch
    split by its own ceil(cnt / world), as the step selects rows), the entries'
    offsets are a permutation of the slice's by ascending user, padding rows (-1)
    last, and each entry's user field is its row's user."""
    import ncf_amd._lib as L
    rng = np.random.default_rng(n + world)
    rows = _rand_rows(rng, n, users, 3707, hot=0.2)
    pad = torch.as_tensor(rng.random(n) < 0.01, device=DEV)
    rows = torch.where(pad, rows | 0xFFFFFFFF, rows)  # user -1
    order = torch.full((n + (n + 1) // 2,), -7, dtype=torch.int64, device=DEV)  # entries + int32 inverse
    L.check(L.hip().ncf_user_order(rows.data_ptr(), n, bs, world, users, order.data_ptr(), L.stream_ptr()),
            "ncf_user_order")
    torch.cuda.synchronize()
    r, e = rows.cpu().numpy(), order[:n].cpu().numpy()
    inv = order.cpu().numpy().view(np.int32)[2 * n:3 * n]
    o, ou = e & 0xFFFFFFFF, e >> 32  # entry: user << 32 | offset (user -1: padding)
    slices = 0
    for b0 in range(0, n, bs):
        cnt = min(bs, n - b0)
        per = -(-cnt // world)
        for lo in range(0, cnt, per):
            s0, ln = b0 + lo, min(per, cnt - lo)
            oo = o[s0:s0 + ln]
            assert np.array_equal(np.sort(oo), np.arange(ln)), "not a permutation of the slice"
            assert np.array_equal(inv[s0:s0 + ln][oo], np.arange(ln)), "inverse positions"
            u = (r[s0:s0 + ln][oo] & 0xFFFFFFFF).astype(np.int64)
            assert np.array_equal(ou[s0:s0 + ln], np.where(u == 0xFFFFFFFF, -1, u)), "entry user field"
            key = np.where(u == 0xFFFFFFFF, users, u)
            assert (np.diff(key) >= 0).all(), "slice not sorted by user"
            slices += 1
    assert slices >= world


LAYERED = [("NeuMF-end", 32, 3), ("MLP", 6, 2), ("GMF", 5, 1), ("NeuMF-pre", 64, 4)]


@pytest.mark.parametrize("mt,f,Lyr", LAYERED)
def test_layered_module_autograd_and_forward(mt, f, Lyr):
    """NCF.forward / autograd on the layered path vs the oracle, incl. edge sizes."""
    import ncf_amd._lib as L
    assert L.supported(mt, f, Lyr) == L.PATH_LAYERED
    ref, m = _models(mt, f, Lyr, U=300, I=500, seed=8)
    for n in (1, 63, 64, 65, 1000):
        rng = np.random.default_rng(n)
        u = rng.integers(0, 300, n)
        i = rng.integers(0, 500, n)
        y = (rng.random(n) < 0.3).astype(np.int64)
        lg_ref, loss_ref, g_ref = O.forward_backward(ref, u, i, y)
        m.zero_grad(set_to_none=True)
        pred = m(torch.from_numpy(u).to(DEV), torch.from_numpy(i).to(DEV))
        np.testing.assert_allclose(pred.detach().cpu().numpy(), lg_ref.numpy(), rtol=1e-5, atol=1e-7)
        loss = torch.nn.BCEWithLogitsLoss()(pred, torch.from_numpy(y).float().to(DEV))
        np.testing.assert_allclose(loss.item(), loss_ref, rtol=1e-5)
        loss.backward()
        for k, p in m.named_parameters():
            if k in g_ref:
                _close_grad(p.grad.cpu().numpy(), g_ref[k].numpy(), f"{k} n={n}")
            else:
                assert p.grad is None, k


@pytest.mark.parametrize("mt,f,Lyr", [("NeuMF-end", 32, 3), ("GMF", 5, 1)])
@pytest.mark.parametrize("use_graph", [False, True])
def test_layered_engine_trajectory_vs_oracle(mt, f, Lyr, use_graph):
    """30 fused-engine Adam steps on the layered path vs torch.optim.Adam on the oracle."""
    T, B = 30, 512
    ref, m, eng = _engine_for(mt, f, Lyr, 200, 300, 6)
    rng = np.random.default_rng(12)
    users = rng.integers(0, 200, (T, B))
    items = rng.integers(0, 300, (T, B))
    labels = (rng.random((T, B)) < 0.2).astype(np.int64)
    _stream(eng, users, items, labels, B)
    eng.run(T, use_graph=use_graph)
    torch.cuda.synchronize()
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    losses = O.train_steps(ref, opt, users, items, labels)
    np.testing.assert_allclose(eng.epoch_losses()[:T], losses, rtol=1e-5)
    for (k, v), (k2, v2) in zip(m.state_dict().items(), ref.state_dict().items()):
        np.testing.assert_allclose(v.cpu().numpy(), v2.numpy(), rtol=1e-4, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("mt,f,Lyr", [("NeuMF-end", 16, 3), ("GMF", 8, 1), ("NeuMF-end", 32, 3)])
def test_fused_reduce_adam_bitwise_equals_separate_kernels(monkeypatch, mt, f, Lyr):
    """ncf_reduce_adam_step == ncf_reduce_slab + ncf_adam_step (same slab summation
    order, same Adam arithmetic).  Not bit for bit: the embedding gradients are f32
    atomics whose order differs between any two runs; Adam turns a near-zero
    gradient's order-dependent sign into up to ~lr of movement, so parameters are
    held per _assert_trajectory_close, losses to rtol 1e-5, the step counters exactly."""
    T, B = 15, 700
    rng = np.random.default_rng(21)
    users = rng.integers(0, 200, (T, B))
    items = rng.integers(0, 300, (T, B))
    labels = (rng.random((T, B)) < 0.2).astype(np.int64)
    out = []
    for fused in ("1", "0"):
        monkeypatch.setenv("NCF_FUSED_ADAM", fused)
        _, m, eng = _engine_for(mt, f, Lyr, 200, 300, 6)
        assert eng._fused_optimizer == (fused == "1")
        _stream(eng, users, items, labels, B)
        eng.run(T, use_graph=True)
        torch.cuda.synchronize()
        out.append(([v.cpu().numpy().copy() for v in m.state_dict().values()], eng.epoch_losses()[:T].copy(),
                    eng.ctl.cpu().numpy()[:2].copy()))
    for k, (a, b) in enumerate(zip(out[0][0], out[1][0])):
        _assert_trajectory_close(a, b, T, 1e-3, f"param {k}")
    np.testing.assert_allclose(out[0][1], out[1][1], rtol=1e-5)
    assert np.array_equal(out[0][2], out[1][2]) and out[0][2][1] == T


@pytest.mark.parametrize("mt,f,Lyr", [("NeuMF-end", 16, 3), ("NeuMF-end", 8, 2)])
def test_engine_multitile_trajectory_vs_oracle(mt, f, Lyr):
    """Batches of 40,000 rows (every workgroup runs 2 tiles per step): 6 engine
    Adam steps vs torch.optim.Adam on the oracle, free-running
    (_assert_trajectory_close) and teacher-forced step by step (_teacher_forced_steps:
    a wrong tile, e.g. stale staging, fails at the step it happens)."""
    T, B = 6, 40000
    ref, m, eng = _engine_for(mt, f, Lyr, 3000, 2000, 9)
    rng = np.random.default_rng(31)
    users = rng.integers(0, 3000, (T, B))
    items = np.minimum(rng.zipf(1.3, (T, B)) - 1, 1999)
    labels = (rng.random((T, B)) < 0.2).astype(np.int64)
    _stream(eng, users, items, labels, B)
    eng.run(T, use_graph=True)
    torch.cuda.synchronize()
    got_losses = eng.epoch_losses()[:T].copy()
    got = {k: v.cpu().numpy().copy() for k, v in m.state_dict().items()}
    ref0 = {k: v.clone() for k, v in ref.state_dict().items()}
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    losses = O.train_steps(ref, opt, users, items, labels)
    np.testing.assert_allclose(got_losses, losses, rtol=1e-5)
    for k, r in ref.state_dict().items():
        _assert_trajectory_close(got[k], r.numpy(), T, 1e-3, k)
    ref.load_state_dict(ref0)
    _teacher_forced_steps(ref, m, eng, users, items, labels)


@pytest.fixture
def geometry():
    """Force the fused step's workgroup geometry (ncf_debug_set_geometry) for the test."""
    import ncf_amd._lib as L
    yield lambda waves: L.check(L.hip().ncf_debug_set_geometry(waves), "geometry")
    L.hip().ncf_debug_set_geometry(0)


@pytest.mark.parametrize("waves", [0, 8, 4, 2, 1])
@pytest.mark.parametrize("B,per_row", [(1024, True), (4096, True), (8192, False), (300, True), (20000, False)])
def test_engine_tuned_launch_shape_vs_oracle(B, per_row, waves, geometry):
    """ncf_layout_tune: the engine launches ceil(B / (16 x waves)) workgroups (the
    reductions read that many slab rows) -- by default (waves 0) 8 waves where the batch
    has 256 128-row tiles, else 4, or forced 8 / 4 / 2 / 1 -- and takes per-row layer 0
    when 2B < U + I (config C2: NCF(8,3), bs 1024, ml-1m ids).  Every step
    teacher-forced from the oracle.  (NCF(8,3) has every geometry: OWN0 below 8 waves
    and at 8, the factored kernel at B >= U + I / 2.)"""
    import ncf_amd._lib as L
    geometry(waves)
    T = 6
    ref, m, eng = _engine_for("NeuMF-end", 8, 3, 6041, 3707, 17)
    rng = np.random.default_rng(43)
    users = rng.integers(0, 6041, (T, B))
    items = np.minimum(rng.zipf(1.3, (T, B)) - 1, 3706)
    labels = (rng.random((T, B)) < 0.2).astype(np.int64)
    _stream(eng, users, items, labels, B)
    assert _fact_mode(eng.lay) == (not per_row)
    w = waves or (8 if (B + 127) // 128 >= 256 else 4)
    assert (8, 4, 2, 1)[(eng.lay.flags >> L.LAYOUT_GEO_SHIFT) & L.LAYOUT_GEO_MASK] == w
    tiles = (B + 16 * w - 1) // (16 * w)
    assert (eng.lay.flags >> 8) & 0xFFF == (tiles if tiles < 256 else 0)
    ref0 = {k: v.clone() for k, v in ref.state_dict().items()}
    eng.run(T, use_graph=True)
    torch.cuda.synchronize()
    got_losses = eng.epoch_losses()[:T].copy()
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    np.testing.assert_allclose(got_losses, O.train_steps(ref, opt, users, items, labels), rtol=1e-5)
    ref.load_state_dict(ref0)
    _teacher_forced_steps(ref, m, eng, users, items, labels)


# --------------------------------------------------------------------------- dropout
# nn.Dropout(p) before every tower Linear (models.py:23): training steps with p > 0
# run the layered path with hashed keep masks (include/ncf_hip.h ncf_dropout_hash);
# the oracle applies the same masks (forward_masked), so everything but the mask
# bits (torch's Philox stream, not reproduced: parity unpinned) is checked exactly.
def _masked_step_ref(ref, users, items, labels, masks):
    ref.zero_grad(set_to_none=True)
    u = torch.as_tensor(np.asarray(users), dtype=torch.int64)
    i = torch.as_tensor(np.asarray(items), dtype=torch.int64)
    logits = O.forward_masked(ref, u, i, masks)
    loss = O.bce_mean(logits, torch.as_tensor(np.asarray(labels)))
    loss.backward()
    return logits.detach(), float(loss.item()), {k: p.grad.detach().clone() for k, p in ref.named_parameters()
                                                 if p.grad is not None}


@pytest.mark.parametrize("mt,f,Lyr,p", [("NeuMF-end", 16, 3, 0.3), ("MLP", 8, 2, 0.5), ("NeuMF-end", 32, 3, 0.1)])
def test_one_step_dropout_vs_masked_oracle(mt, f, Lyr, p):
    """One training step with dropout p at ml-1m ids (B = 8,192; the fused shape
    NCF(16,3) is routed to the layered path) vs the oracle under the same masks."""
    import ncf_amd._lib as L
    from ncf_amd import ops
    U, I, B = 6041, 3707, 8192
    ref, m = _models(mt, f, Lyr, U=U, I=I, seed=29, dropout=p)
    rng = np.random.default_rng(5)
    users = rng.integers(0, U, B)
    items = np.minimum(rng.zipf(1.3, B) - 1, I - 1)
    labels = (rng.random(B) < 0.2).astype(np.int64)
    flat, lay0 = ops.ensure_flat(m)
    lay = type(lay0).from_buffer_copy(lay0)
    ops.set_dropout(lay, m)
    assert lay.dropout > 0 and not ops.fact_mode(lay)
    masks = O.dropout_masks(ref, int(lay.dropout_seed), 0, np.arange(B), p)
    kept = float(np.mean([mk.numpy().astype(bool).mean() for mk in masks]))
    assert abs(kept - (1 - p)) < 0.01
    logits_ref, loss_ref, grads_ref = _masked_step_ref(ref, users, items, labels, masks)
    gflat = torch.zeros(int(lay.total), device=DEV)
    ws = ops.new_workspace(lay, B, DEV)
    ctl = ops.new_ctl(B, DEV)
    u = torch.as_tensor(users, dtype=torch.int32, device=DEV)
    it = torch.as_tensor(items, dtype=torch.int32, device=DEV)
    y = torch.as_tensor(labels, dtype=torch.float32, device=DEV)
    rows = ops.pack_rows(u, it, y)
    logits = torch.empty(B, device=DEV)
    st = L.stream_ptr()
    L.check(L.hip().ncf_train_step(L.ctypes.byref(lay), flat.data_ptr(), gflat.data_ptr(), rows.data_ptr(), None,
                                   None, ctl.data_ptr(), B, 1, 0, L.DZ_BCE, ws.data_ptr(), ws.numel() * 4,
                                   logits.data_ptr(), st), "train")
    L.check(L.hip().ncf_reduce_slab(L.ctypes.byref(lay), ws.data_ptr(), gflat.data_ptr(), ctl.data_ptr(), st),
            "reduce")
    torch.cuda.synchronize()
    np.testing.assert_allclose(logits.cpu().numpy(), logits_ref.numpy(), rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(gflat[lay.loss_slot].item(), loss_ref, rtol=1e-5)
    for (q, off), (name, _) in zip(ops._segments(m, lay), m.named_parameters()):
        got = gflat[off:off + q.numel()].view_as(q).cpu().numpy()
        if name in grads_ref:
            hot = int(np.bincount(items).max()) if "item" in name else int(np.bincount(users).max())
            _close_grad(got, grads_ref[name].numpy(), name, terms=hot if "embed" in name else None)


def test_engine_dropout_trajectory_vs_masked_oracle():
    """TrainEngine (hipGraph) with dropout 0.2 on NCF(16,3): step t masks the rows
    t*B .. of the epoch stream at Adam step t; 6 steps vs torch.optim.Adam on the
    oracle under the same masks (losses rtol 1e-5, parameters per
    _assert_trajectory_close)."""
    from ncf_amd import ops
    T, B, p = 6, 4096, 0.2
    ref, m, eng = _engine_for("NeuMF-end", 16, 3, 6041, 3707, 31, dropout=p)
    assert eng.lay.dropout == np.float32(p) and not ops.fact_mode(eng.lay)
    rng = np.random.default_rng(53)
    users = rng.integers(0, 6041, (T, B))
    items = np.minimum(rng.zipf(1.3, (T, B)) - 1, 3706)
    labels = (rng.random((T, B)) < 0.2).astype(np.int64)
    _stream(eng, users, items, labels, B)
    eng.run(T, use_graph=True)
    torch.cuda.synchronize()
    got_losses = eng.epoch_losses()[:T].copy()
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    losses = []
    for t in range(T):
        masks = O.dropout_masks(ref, int(eng.lay.dropout_seed), t, t * B + np.arange(B), p)
        opt.zero_grad()
        loss = O.bce_mean(O.forward_masked(ref, torch.as_tensor(users[t]), torch.as_tensor(items[t]), masks),
                          torch.as_tensor(labels[t]))
        loss.backward()
        opt.step()
        losses.append(loss.item())
    np.testing.assert_allclose(got_losses, losses, rtol=1e-5)
    for k, r in ref.state_dict().items():
        _assert_trajectory_close(m.state_dict()[k].cpu().numpy(), r.numpy(), T, 1e-3, k)


def test_module_forward_dropout_train_and_eval():
    """NCF.forward on the device with dropout 0.4: train mode applies the masks of
    its own step index in forward and backward (= the oracle under those masks); a
    fresh mask per call; eval mode is the plain forward."""
    from ncf_amd import ops
    p, n = 0.4, 3000
    ref, m = _models("NeuMF-end", 16, 3, U=400, I=700, seed=37, dropout=p)
    rng = np.random.default_rng(9)
    users, items = rng.integers(0, 400, n), rng.integers(0, 700, n)
    labels = (rng.random(n) < 0.3).astype(np.int64)
    m.train()
    pred = m(torch.as_tensor(users, device=DEV), torch.as_tensor(items, device=DEV))
    t = m._ncf_drop_t
    masks = O.dropout_masks(ref, ops.dropout_seed(DEV), t, np.arange(n), p)
    lg_ref, loss_ref, g_ref = _masked_step_ref(ref, users, items, labels, masks)
    np.testing.assert_allclose(pred.detach().cpu().numpy(), lg_ref.numpy(), rtol=1e-5, atol=1e-7)
    loss = torch.nn.BCEWithLogitsLoss()(pred, torch.as_tensor(labels, dtype=torch.float32, device=DEV))
    np.testing.assert_allclose(loss.item(), loss_ref, rtol=1e-5)
    loss.backward()
    for k, q in m.named_parameters():
        if k in g_ref:
            _close_grad(q.grad.cpu().numpy(), g_ref[k].numpy(), k)
    with torch.no_grad():
        again = m(torch.as_tensor(users, device=DEV), torch.as_tensor(items, device=DEV))
    assert m._ncf_drop_t == t + 1 and not torch.equal(again, pred.detach())
    m.eval()
    ref.eval()
    with torch.no_grad():
        ev = m(torch.as_tensor(users, device=DEV), torch.as_tensor(items, device=DEV))
        ev_ref = ref(torch.as_tensor(users), torch.as_tensor(items))
    np.testing.assert_allclose(ev.cpu().numpy(), ev_ref.numpy(), rtol=1e-5, atol=1e-7)


def test_engine_loss_history_beyond_65536_batches():
    """An epoch of 70,001 batches (2 rows each): the loss history grows to the
    epoch's batch count (the kernels write loss_hist[b % num_batches]) -- the last
    batch's loss lands in its own slot, nothing past the buffer."""
    T, B = 3, 2
    ref, m, eng = _engine_for("NeuMF-end", 8, 3, 50, 80, 41)
    n = 140001
    rng = np.random.default_rng(61)
    users, items = rng.integers(0, 50, n), rng.integers(0, 80, n)
    labels = (rng.random(n) < 0.3).astype(np.int64)
    _stream(eng, users, items, labels, B)
    assert eng.num_batches == 70001 and eng.loss_hist.numel() >= 70001
    eng.run(T, use_graph=True)
    eng.ctl[0] = eng.num_batches - 1  # the partial last batch (1 row)
    eng.run(1, use_graph=False)
    torch.cuda.synchronize()
    h = eng.epoch_losses()
    assert h.shape[0] == 70001 and np.isfinite(h).all()
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    exp = O.train_steps(ref, opt, users[:T * B].reshape(T, B), items[:T * B].reshape(T, B),
                        labels[:T * B].reshape(T, B))
    exp.append(O.train_steps(ref, opt, [users[-1:]], [items[-1:]], [labels[-1:]])[0])
    np.testing.assert_allclose(h[:T], exp[:T], rtol=1e-5)
    np.testing.assert_allclose(h[-1], exp[-1], rtol=1e-5)
