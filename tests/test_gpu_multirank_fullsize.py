"""Multi-rank parity at the reference's full shapes ("C3 (1 vs 2/4/8
GPUs)", first steps at <= 1e-5 relative; scripts/train_neumf.py:55,86,90,106-118).

World 2 and 4 ranks are spawned processes sharing cuda:0 over gloo (the one-GPU test
box cannot hold one RCCL rank per process; gloo moves the same device buffers through
the host, so everything but the transport is the bench's N > 1 path):

  * C3 -- NCF(16,3) NeuMF-end, the ml-1m-shaped data set, global batch 65,536, the
    default exchange (dp_mode "auto", which resolves to "allreduce" here: a 65,536-row
    ml-1m batch touches every row), one whole fresh epoch through Trainer.fit (the
    epoch pipeline: fresh negatives and permutation, the fused factored step on each
    rank's 32,768 / 16,384-row shard, hipGraph replay);
  * C4 -- NCF(16,3) at the ml-20m id space (138,494 x 26,745), global batch 65,536,
    100 steps on the engine: world 2 with the default exchange ("auto", which resolves
    to "owner" at C4), world 4 and world 8 -- BASELINE config 4's own rank count --
    with "owner" explicitly.

Checks: ranks bitwise equal to each other (losses and every parameter); every step's
loss within rtol 1e-5 of the single-rank engine on the same stream; the losses
against the oracle (oracle/ncf_oracle.py, the reference loop restated on torch CPU
ops + torch.optim.Adam with the same negatives and permutation): C3 the first 20
steps at rtol 1e-5; C4 the first 10 at 1e-5 and 20 at 1e-4 (the single-rank C4 run
itself parts from the fp32 oracle to ~3.6e-5 from step ~12, test_gpu_fullsize.py);
the parameters after the run against the single-rank run by the trajectory criterion
of the single-rank tests (test_gpu_parity._assert_trajectory_close: the shard sums
are the whole-batch sums in another fp32 order, which Adam turns into drift).

Round 5 adds the owner-sharded exchange (dp_mode "owner": gradient rows to their
owners, dense Adam per owner, the next batch's rows back) at the configs' own rank
counts: C4 at world 2, 4 and 8 over 100 steps, C3 at world 8 (8,192-row shards, one whole
fresh epoch through Trainer.fit), and the bench's weak-scaling leg -- world 2 at a
global batch of 131,072 -- against the oracle at batch_size 131,072.  Past the first
steps at C4 the late tolerance is 1e-4: the reference's own fp32 loop, perturbed by
one ulp per step, parts by ~1e-5 to 4e-5 within 100 steps at this shape
(test_oracle.test_c4_fp32_trajectory_sensitivity).

Every rank builds the same epoch stream: the grouping is canonical for world > 1
(ncf_prepare_epoch2 NCF_PREP_CANONICAL; without it the rows of an item run sit in
arrival order, which differs between the processes, and a shard boundary inside a run
gave some rows to two ranks and others to none: per-step losses off by up to 8e-5).
zero1 on the factored path expands the shard's G rows with the W0 the step ran with
(a snapshot in the workspace; reading W0 in place raced with its own update)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import ncf_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
B = 65536


def _data(shape):
    from ncf_amd import synthetic
    from ncf_amd.data import NCFData
    ds = synthetic.make_dataset(shape, seed=0)
    I = ds["item_num"]
    train = NCFData(np.stack([ds["train_users"], ds["train_items"]], 1), I, None, 4, True)
    tu = np.repeat(ds["test_users"], 100)
    ti = np.concatenate([ds["test_items"][:, None], ds["test_negatives"]], 1).reshape(-1)
    test = NCFData(np.stack([tu, ti], 1), I, None, 0, False)
    return ds, train, test


def _flat(model):
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy()


def _c3_run(world, rank, group, batch=B):
    """Trainer.fit(1) at C3 (train_neumf.py:98-131), seeds 0 as the scripts set them."""
    from torch.utils.data import DataLoader
    from ncf_amd.models import NCF
    from ncf_amd.trainer import Trainer
    ds, train, test = _data("ml-1m")
    np.random.seed(0)
    torch.manual_seed(0)
    model = NCF(ds["user_num"], ds["item_num"], 16, 3, 0.0, "NeuMF-end").to(DEV)
    tr = Trainer(model, train, DataLoader(test, batch_size=100, shuffle=False), batch_size=batch, lr=1e-3, top_k=10,
                 verbose=False, world_size=world, rank=rank, process_group=group)
    tr.fit(1)
    torch.cuda.synchronize()
    eng = tr.engine
    losses = eng.epoch_losses()[:eng.num_batches].astype(np.float64).copy()
    if eng.dp_mode == "zero1":
        assert eng._fact_shard  # the sharded factored expansion ran
    return _flat(model), losses, eng.dp_mode


def _c3w_run(world, rank, group):
    """The bench's weak-scaling leg: the per-GPU batch held at 65,536 (global B x world)."""
    return _c3_run(world, rank, group, batch=B * world)


def _c3n_run(world, rank, group):
    """C3 with no process group handed to Trainer (its default): the engine must run its
    owner all-gather and stream check over the default group (without it the
    replicas kept stale rows after fit)."""
    return _c3_run(world, rank, None)


def _c4_stream(train, item_num, dev):
    """One epoch stream as the host path of Trainer._epoch_stream builds it:
    ng_sample (NumPy global stream), the DataLoader's permutation (torch global
    generator), packed rows grouped by item per global batch."""
    from ncf_amd import ops
    from ncf_amd.data import epoch_permutation
    train.ng_sample()
    u, i, y = train.arrays()
    perm = epoch_permutation(len(u)).to(dev)
    rows = torch.from_numpy(ops.pack_rows_host(u, i, y)).to(dev)
    return ops.EpochPrep(torch.device(dev), canonical=True)(rows, perm, B, int(item_num))


C4_STEPS = 20


def _c4_run(world, rank, group, steps=C4_STEPS):
    from ncf_amd.engine import TrainEngine
    from ncf_amd.models import NCF
    ds, train, _ = _data("ml-20m")
    np.random.seed(0)
    torch.manual_seed(0)
    model = NCF(ds["user_num"], ds["item_num"], 16, 3, 0.0, "NeuMF-end").to(DEV)
    eng = TrainEngine(model, lr=1e-3, world_size=world, rank=rank, process_group=group)
    stream = _c4_stream(train, ds["item_num"], DEV)
    eng.set_epoch_stream(stream, B, checked=True)
    eng.run(steps)
    torch.cuda.synchronize()
    losses = eng.epoch_losses()[:steps].astype(np.float64).copy()
    # the next global batch of the same stream (untrained): the held-out check of c4l
    nxt = stream[steps * B:(steps + 1) * B].cpu().numpy().view(np.uint64)
    held = ((nxt & 0xFFFFFFFF), (nxt >> 32) & 0x7FFFFFFF, (nxt >> 63) & 1)
    return _flat(model), losses, eng.dp_mode, held


def _c4l_run(world, rank, group):
    """C4 over 100 steps."""
    return _c4_run(world, rank, group, steps=100)


# what dp_mode "auto" resolves to (TrainEngine.auto_dp_mode)
AUTO_EXPECT = {("c3", 2): "allreduce", ("c3", 4): "owner", ("c3", 8): "owner", ("c4", 2): "owner",
               ("c4l", 2): "owner"}

RUNS = {"c3": _c3_run, "c4": _c4_run, "c4l": _c4l_run, "c3w": _c3w_run, "c3n": _c3n_run}


def _worker(rank, world, port, name, q, dp_mode=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if dp_mode is not None:  # TrainEngine's default exchange for world > 1 (Trainer takes none)
        os.environ["NCF_DP_MODE"] = dp_mode
    # the ranks share the box's CPUs: one sampler pool each, sized for the group
    os.environ.setdefault("LOCAL_WORLD_SIZE", str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        res = RUNS[name](world, rank, dist.group.WORLD)
    except Exception:  # report instead of leaving the other ranks waiting in a collective
        import traceback
        q.put((rank, None, traceback.format_exc()))
        os._exit(1)
    q.put((rank, res, None))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(name, world, dp_mode=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q, dp_mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, out, err = q.get(timeout=600)
            if out is None:
                raise AssertionError(f"rank {r} failed:\n{err}")
            res[r] = out
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return res


_single = {}


def _single_rank(name):
    """The single-rank run of the same config (the weak-scaling leg: at world 2's global
    batch)."""
    if name not in _single:
        _single[name] = _c3_run(1, 0, None, batch=2 * B) if name == "c3w" else RUNS[name](1, 0, None)
    return _single[name]


_ORACLE = {}


def _oracle_losses(name, steps, batch=B):
    """The reference loop's first `steps` losses from the same seeds (oracle; once per
    data shape, steps and batch in a session)."""
    key = (name.startswith("c4"), steps, batch)
    if key not in _ORACLE:
        _ORACLE[key] = _oracle_losses_run(name, steps, batch)
    return _ORACLE[key]


def _oracle_losses_run(name, steps, batch):
    ds, _, _ = _data("ml-20m" if name.startswith("c4") else "ml-1m")
    U, I = ds["user_num"], ds["item_num"]
    pu, pi = ds["train_users"], ds["train_items"]
    torch.set_num_threads(min(16, torch.get_num_threads()))
    torch.manual_seed(0)
    ref = O.OracleNCF(U, I, 16, 3, 0.0, "NeuMF-end")
    neg = O.ng_sample(pu, pi, I, 4, 0)
    users = np.concatenate([pu, np.repeat(pu, 4)]).astype(np.int64)
    items = np.concatenate([pi, neg]).astype(np.int64)
    labels = np.concatenate([np.ones(len(pu), np.int64), np.zeros(len(neg), np.int64)])
    perm = O.epoch_order(len(users))
    sl = [perm[b * batch:(b + 1) * batch] for b in range(steps)]
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    return np.asarray(O.train_steps(ref, opt, [users[s] for s in sl], [items[s] for s in sl],
                                    [labels[s] for s in sl]), dtype=np.float64)


@pytest.mark.parametrize("name,world,dp_mode", [("c3", 2, None), ("c3", 4, None), ("c4l", 2, None),
                                                 ("c3", 4, "zero1"), ("c4l", 4, "owner"), ("c4l", 8, "owner"),
                                                 ("c3", 8, "owner"), ("c3", 8, None), ("c3w", 2, "owner"),
                                                 ("c3n", 2, "owner")])
def test_full_shape_ranks_match_single_rank_and_oracle(name, world, dp_mode):
    """dp_mode None: the default ("auto"); "zero1" at C3: reduce-scatter, each rank
    expands the factored layer 0 of its own shard inside its Adam launch
    (ncf_adam_step_fact), all-gather; "owner": the owner-sharded exchange."""
    res = _spawn(name, world, dp_mode)
    flat0, loss0, mode0 = res[0][:3]
    for r in range(1, world):
        assert np.array_equal(res[r][1], loss0), f"rank {r} losses differ from rank 0"
        assert np.array_equal(res[r][0], flat0), f"rank {r} parameters differ from rank 0"
        assert res[r][2] == mode0
    want = dp_mode or AUTO_EXPECT[(name, world)]
    assert mode0 == want, mode0
    flat1, loss1, mode1 = _single_rank(name)[:3]
    assert mode1 == "single"
    nb = {"c3": 76, "c4": 20, "c4l": 100, "c3w": 38, "c3n": 76}[name]
    assert len(loss0) == len(loss1) == nb
    batch = 2 * B if name == "c3w" else B
    ref = _oracle_losses(name, 20, batch)
    rel1 = np.abs(loss0 - loss1) / np.abs(loss1)
    relo = np.abs(loss0[:20] - ref) / np.abs(ref)
    rel1o = np.abs(loss1[:20] - ref) / np.abs(ref)
    info = (f"{name} world {world} {mode0}: max rel vs 1 rank {rel1.max():.2e} (first step > 1e-5: "
            f"{int(np.argmax(rel1 > 1e-5)) if (rel1 > 1e-5).any() else None}); vs oracle (20) {relo.max():.2e}; "
            f"1 rank vs oracle (20) {rel1o.max():.2e}; per step vs 1 rank {np.round(rel1 * 1e6, 2).tolist()} (1e-6)")
    print(info)
    if name.startswith("c3"):
        assert relo.max() <= 1e-5, info
        assert rel1.max() <= 1e-5, info
    else:
        assert relo[:10].max() <= 1e-5 and relo.max() <= 1e-4, info
        # the steps the single rank holds to the oracle at 1e-5: held to the single rank at 1e-5
        held = rel1o <= 1e-5
        assert rel1[:20][held].max(initial=0.0) <= 1e-5, info
        assert rel1.max() <= 1e-4, info
    # parameters after the free-running steps: two fp32 trajectories (shard sums vs
    # whole-batch sums) -- the criterion of the single-rank trajectory tests
    from test_gpu_parity import _assert_trajectory_close
    if nb < 100:
        _assert_trajectory_close(flat0, flat1, nb, 1e-3, f"{name} world {world}: params vs 1 rank")
        return
    # 100 free-running steps at C4: the element-wise criterion stops meaning much -- the
    # reference's own loop perturbed by one ulp per step leaves 9% of the elements
    # outside it (0.27% at 50 steps, 0.01% at 20; test_oracle.py), two GPU runs 11-30%
    # (Adam turns near-zero gradients of rarely touched rows into +-lr moves).  Checked
    # instead: every element within 4 T lr, and the two parameter sets give the same
    # loss on the stream's next (untrained) global batch -- the oracle model on the CPU --
    # within the late tolerance of the per-step losses, 1e-4 relative
    dev = np.abs(flat0.astype(np.float64) - flat1.astype(np.float64))
    assert dev.max() <= 4 * nb * 1e-3, dev.max()
    ds, _, _ = _data("ml-20m")
    hu, hi, hy = (np.asarray(x, dtype=np.int64) for x in res[0][3])
    assert all(np.array_equal(a, b) for a, b in zip(res[0][3], _single_rank(name)[3]))
    held = []
    for flat in (flat0, flat1):
        m = O.OracleNCF(ds["user_num"], ds["item_num"], 16, 3, 0.0, "NeuMF-end")
        off = 0
        with torch.no_grad():
            for p in m.parameters():
                p.copy_(torch.from_numpy(flat[off:off + p.numel()].reshape(p.shape)))
                off += p.numel()
            held.append(float(O.bce_mean(m(torch.from_numpy(hu), torch.from_numpy(hi)), torch.from_numpy(hy))))
    print(f"{name} world {world}: held-out loss {held[0]:.8f} vs 1 rank {held[1]:.8f}; "
          f"{(dev > 1e-4 * np.abs(flat1) + 1e-6 * np.abs(flat1).max()).mean():.3f} of elements off element-wise")
    assert abs(held[0] - held[1]) <= 1e-4 * abs(held[1]), held
