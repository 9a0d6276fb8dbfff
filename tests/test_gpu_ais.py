"""In-step Adam (ABI 18, ncf_train_step_ais): the previous step's dense Adam inside the
next training launch -- on the fly for what the launch reads, written for every float
by its extra workgroups -- against the two-launch form (ncf_train_step +
ncf_reduce_adam_step) and the oracle.

The two forms run the same Adam on the same gradients; the tower gradient is summed
by float atomics instead of the slab's fixed order, so trajectories agree to the
step's usual last-bit noise (test_gpu_parity's criterion), the losses to 1e-6."""
import os

import numpy as np
import pytest
import torch

from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _run(on, U, I, f, nl, mt, B, T, graph=True, chunks=1, seed=0):
    from ncf_amd import ops
    from ncf_amd.engine import TrainEngine
    from ncf_amd.models import NCF
    rng = np.random.default_rng(seed)
    u = rng.integers(0, U, T * B)
    i = np.minimum(rng.zipf(1.3, T * B) - 1, I - 1)
    y = (rng.random(T * B) < 0.2).astype(np.float32)
    torch.manual_seed(1)
    m = NCF(U, I, f, nl, 0.0, mt).to(DEV)
    old = TrainEngine.ADAM_IN_STEP
    TrainEngine.ADAM_IN_STEP = on
    try:
        eng = TrainEngine(m, lr=1e-3)
        eng.set_epoch_stream(torch.as_tensor(ops.pack_rows_host(u, i, y), device=DEV), B)
        assert eng._ais_active == on
        per = T // chunks
        for c in range(chunks):
            eng.run(per if c < chunks - 1 else T - per * (chunks - 1), use_graph=graph)
        torch.cuda.synchronize()
        ctl = eng.ctl.cpu().numpy()
        assert int(ctl[0]) == T and int(ctl[1]) == T, ctl  # batch, adam_t
        assert not getattr(eng, "_ais_live", False)
        return ({k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()},
                eng.epoch_losses()[:T].copy(), (u, i, y),
                (eng.exp_avg.cpu().numpy().copy(), eng.exp_avg_sq.cpu().numpy().copy()))
    finally:
        TrainEngine.ADAM_IN_STEP = old


@pytest.mark.parametrize("mt,f,nl", [("NeuMF-end", 8, 3), ("MLP", 8, 2), ("GMF", 8, 1), ("NeuMF-end", 16, 2)])
@pytest.mark.parametrize("graph", [True, False])
def test_in_step_adam_equals_two_launch_form(mt, f, nl, graph):
    from test_gpu_parity import _assert_trajectory_close
    U, I, B, T = 6041, 3707, 1024, 24
    a, la, _, sa = _run(True, U, I, f, nl, mt, B, T, graph)
    b, lb, _, sb = _run(False, U, I, f, nl, mt, B, T, graph)
    assert np.all(la > 0)  # every step's loss recorded (the last by ncf_ais_flush)
    np.testing.assert_allclose(la, lb, rtol=1e-6)
    for k in a:
        _assert_trajectory_close(a[k], b[k], T, 1e-3, k)
    for x, y in zip(sa, sb):  # the moments come back into the engine's buffers too
        np.testing.assert_allclose(x, y, rtol=1e-4, atol=1e-9)


def test_in_step_adam_across_runs_and_chunks():
    """Three run() calls (flush / begin between them) and graph chunks of 32 with
    remainders: the same trajectory as one run."""
    U, I, B, T = 6041, 3707, 1024, 70
    a, la, _, _ = _run(True, U, I, 8, 3, "NeuMF-end", B, T, True, chunks=3)
    b, lb, _, _ = _run(True, U, I, 8, 3, "NeuMF-end", B, T, True, chunks=1)
    np.testing.assert_allclose(la, lb, rtol=1e-6)
    from test_gpu_parity import _assert_trajectory_close
    for k in a:
        _assert_trajectory_close(a[k], b[k], T, 1e-3, k)


def test_in_step_adam_vs_oracle():
    U, I, B, T = 6041, 3707, 1024, 30
    a, la, (u, i, y), _ = _run(True, U, I, 8, 3, "NeuMF-end", B, T)
    torch.manual_seed(1)
    ref = O.OracleNCF(U, I, 8, 3, 0.0, "NeuMF-end")
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    lo = O.train_steps(ref, opt, u.reshape(T, B), i.reshape(T, B), y.astype(np.int64).reshape(T, B))
    np.testing.assert_allclose(la, lo, rtol=1e-5)
    from test_gpu_parity import _assert_trajectory_close
    for k, v in ref.state_dict().items():
        _assert_trajectory_close(a[k], v.detach().numpy(), T, 1e-3, k)


def test_in_step_adam_single_steps_and_state():
    """step() leaves no update pending; the optimizer state round-trips."""
    from ncf_amd import ops
    from ncf_amd.engine import TrainEngine
    from ncf_amd.models import NCF
    U, I, B = 600, 400, 1024
    rng = np.random.default_rng(3)
    u, i = rng.integers(0, U, 4 * B), rng.integers(0, I, 4 * B)
    y = (rng.random(4 * B) < 0.2).astype(np.float32)
    out = []
    for on in (True, False):
        old = TrainEngine.ADAM_IN_STEP
        TrainEngine.ADAM_IN_STEP = on
        try:
            torch.manual_seed(2)
            m = NCF(U, I, 8, 3, 0.0, "NeuMF-end").to(DEV)
            eng = TrainEngine(m, lr=1e-3)
            eng.set_epoch_stream(torch.as_tensor(ops.pack_rows_host(u, i, y), device=DEV), B)
            for _ in range(3):
                eng.step()
            torch.cuda.synchronize()
            out.append((torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy(),
                        eng.ctl.cpu().numpy().copy()))
        finally:
            TrainEngine.ADAM_IN_STEP = old
    assert list(out[0][1][:2]) == list(out[1][1][:2]) == [3, 3]
    np.testing.assert_allclose(out[0][0], out[1][0], rtol=1e-4, atol=1e-6)
