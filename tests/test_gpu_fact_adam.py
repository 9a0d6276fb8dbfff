"""NCF_LAYOUT_FACT_IN_ADAM: the factored layer-0 expansion (dUm, dIm, dW0 from the
per-entity sums) inside the optimizer launch (ncf_fact_adam.inc), against the
two-launch form (fact_expand_kernel, then reduce_adam_kernel) and the oracle.

One step from the same state: the same loss, every parameter within one Adam step's
reordering noise (the step kernel's float atomics already make two runs of the same
form differ in the last bits of the embedding gradients, and W0's block partials are
summed in groups of 8, then the groups, instead of by 16 row groups).  Twenty steps: the losses to 1e-6 relative.  The loop at C3's shape against
the oracle is test_gpu_fullsize.test_full_epoch_vs_oracle[c3] (the default path)."""
import os

import numpy as np
import pytest
import torch

from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _run(on, U, I, f, nl, B, T, seed=0):
    from ncf_amd import ops
    from ncf_amd.engine import TrainEngine
    from ncf_amd.models import NCF
    import ncf_amd._lib as L
    os.environ["NCF_FACT_IN_ADAM"] = "1" if on else "0"
    try:
        rng = np.random.default_rng(seed)
        u = rng.integers(0, U, T * B)
        i = np.minimum(rng.zipf(1.3, T * B) - 1, I - 1)
        y = (rng.random(T * B) < 0.2).astype(np.float32)
        torch.manual_seed(1)
        m = NCF(U, I, f, nl, 0.0, "NeuMF-end").to(DEV)
        eng = TrainEngine(m, lr=1e-3)
        eng.set_epoch_stream(torch.as_tensor(ops.pack_rows_host(u, i, y), device=DEV), B)
        assert bool(eng.lay.flags & L.LAYOUT_FACT_IN_ADAM) == on
        assert ops.fact_mode(eng.lay)
        eng.run(T)
        torch.cuda.synchronize()
        return ({k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()},
                eng.epoch_losses()[:T].copy(), (u, i, y))
    finally:
        os.environ.pop("NCF_FACT_IN_ADAM", None)


@pytest.mark.parametrize("f,nl", [(16, 3), (8, 3), (16, 1)])
def test_one_step_equals_two_launch_form(f, nl):
    """dm 64, 32 and 16 (the kernel's three instantiations)."""
    U, I, B = 6041, 3707, 65536
    a, la, _ = _run(True, U, I, f, nl, B, 1)
    b, lb, _ = _run(False, U, I, f, nl, B, 1)
    from test_gpu_parity import _assert_trajectory_close
    assert np.array_equal(la, lb)
    for k in a:  # the step's float atomics make even the two-launch form vary in the last bits
        _assert_trajectory_close(a[k], b[k], 1, 1e-3, k)
        np.testing.assert_allclose(a[k], b[k], rtol=1e-4, atol=2e-5, err_msg=k)


def test_twenty_steps_track_two_launch_form_and_oracle():
    U, I, B, T = 6041, 3707, 65536, 20
    a, la, (u, i, y) = _run(True, U, I, 16, 3, B, T)
    b, lb, _ = _run(False, U, I, 16, 3, B, T)
    np.testing.assert_allclose(la, lb, rtol=1e-6)
    torch.manual_seed(1)
    ref = O.OracleNCF(U, I, 16, 3, 0.0, "NeuMF-end")
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    lo = O.train_steps(ref, opt, u.reshape(T, B), i.reshape(T, B), y.astype(np.int64).reshape(T, B))
    np.testing.assert_allclose(la, lo, rtol=1e-5)
