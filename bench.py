#!/usr/bin/env python3
"""Headline benchmark: NeuMF training interactions/sec on MI355X.

Workload (BASELINE.json metric "training interactions/sec + HR@10, NeuMF
factors=64 ml-1m"): NCF(6041, 3707, factor_num=16,
num_layers=3, 'NeuMF-end') -- 64-wide MLP embeddings, tower [128,64,32,16] --
on ml-1m-shaped synthetic data (994,169 positives, 4 sampled negatives each),
global batch 65,536 (8,192 per GPU at 8 GPUs), Adam lr 1e-3.

A "step" = fused fwd+loss+bwd kernel (+ the factored layer-0 expansion), tower-grad
reduction, (RCCL gradient exchange when N > 1), dense Adam -- the whole optimizer
step of scripts/train_neumf.py:111-115, captured into hipGraphs and replayed.
The timed region is whole epochs (--steps rounded up): every epoch in it is a
fresh epoch of the reference loop -- new negatives (NCFData.ng_sample, bit-exact;
the parallel host sampler, prefetched while the previous epoch trains) and a new
DataLoader permutation (bit-exact torch.randperm, on the device), packed,
shuffled and grouped on the device (ncf_amd.pipeline).  The data set itself is
resident in HBM before the timed region.  The global batch is the reference's
batch size at every N (strong scaling); value = rows of the timed epochs /
max-over-ranks time.  At N > 1 `weak_scaling` also times the per-GPU batch held
at the single-GPU size.

Also reported: `e2e` -- Trainer.fit (the scripts' loop: epochs + metrics() per
epoch) at the same config, rows per epoch / epoch wall time; `cpu_baseline` -- the
oracle (reference model restated on torch CPU ops) on the host cores, in a child
process.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 either under
torch.distributed.run (one process per GPU, RCCL) or directly, in which case the
script spawns its N ranks itself before any GPU call.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (dataset shape, factor_num, num_layers, global batch = the reference's batch_size)
    "c3": ("ml-1m", 16, 3, 65536),     # headline: NeuMF-64 (MLP [128,64,32,16])
    "c2": ("ml-1m", 8, 3, 1024),       # NeuMF [64,32,16,8], bs 1024
    "c4": ("ml-20m", 16, 3, 65536),    # ml-20m shape
    "cli": ("ml-1m", 32, 3, 65536),    # train_neumf.py --num_layers 3 with the config's factor_num 32 (layered path)
    "stress": ("ml-1m", 64, 4, 65536), # NCF(64,4): MLP [1024,512,256,128,64] (layered path)
    "c5": ("ml-1m", 8, 2, 256),        # distillation: student NCF(8,2,'MLP') of teacher NCF(16,3,'NeuMF-end')
}
# model type of the trained model per config (NeuMF-end unless listed); C5 trains the
# student of scripts/train_student.py's default response distillation
MODEL = {"c5": "MLP"}
C5_TEACHER = (16, 3, "NeuMF-end")


def build_model(cfg, U, I, dev):
    """(trained model, distillation module or None) of config `cfg`, random init from
    the current torch seed (teacher first for C5, as train_student.py builds them)."""
    from ncf_amd.models import NCF
    _, f, nl, _ = CONFIGS[cfg]
    if cfg != "c5":
        return NCF(U, I, f, nl, 0.0, MODEL.get(cfg, "NeuMF-end")).to(dev), None
    from ncf_amd.distill import ResponseDistillation
    tf, tl, tm = C5_TEACHER
    teacher = NCF(U, I, tf, tl, 0.0, tm).to(dev)
    teacher.eval()
    student = NCF(U, I, f, nl, 0.0, MODEL["c5"]).to(dev)
    dist = ResponseDistillation(teacher, student)  # train_student.py default: response, T 2.0, alpha 0.5
    dist.to(dev)
    return student, dist


def tower_flops_per_row(f, L, model="NeuMF-end"):
    dm = f * 2 ** (L - 1)
    s = [(2 * dm) >> k for k in range(L + 1)]
    fl = 6 * sum(s[k] * s[k + 1] for k in range(L))
    p = 2 * f if model.startswith("NeuMF") else f
    return fl + 6 * p


def executed_flops(f, L, model, rows, tables, fact, fused):
    """Flops the kernels execute per step (2 per MAC), beside the algorithmic
    SURVEY 8(d) count of tower_flops_per_row: with the factored layer 0
     the per-row layer-0 dgrad + wgrad (and, on the layered path,
    its forward) become per-entity GEMMs over the U + I table rows (`tables`):
    projection 2 (U + I) dm^2 (layered only), dX and dW0 4 (U + I) dm^2."""
    dm = f * 2 ** (L - 1)
    s = [(2 * dm) >> k for k in range(L + 1)]
    p = 2 * f if model.startswith("NeuMF") else f
    if not fact:
        return tower_flops_per_row(f, L, model) * rows
    upper = 6 * sum(s[k] * s[k + 1] for k in range(1, L))  # layers k >= 1: fwd, dgrad, wgrad
    per_row = upper + 6 * p + (2 * s[0] * s[1] if fused else 0)  # the fused kernel's layer-0 forward per row
    per_step = (4 if fused else 6) * tables * dm * dm
    return per_row * rows + per_step


def gather_scatter_bytes_per_row(f, L):
    """Algorithmic HBM bytes per row of the fused kernel: the 8-byte packed row
    (user, item, label), the four embedding rows read, and the same four rows'
    gradient added (f32 atomics: read-modify-write at the memory side)."""
    dm = f * 2 ** (L - 1)
    rows = 2 * (f + dm) * 4
    return 8 + rows + rows


def cache_probe(eng, rows_n, reps=50):
    """ncf_probe_gather_scatter (include/ncf_hip.h) on the engine's own tables and the
    first `rows_n` rows of its current epoch stream: the step's gather + float-atomic
    scatter pattern with no arithmetic, `reps` launches back to back between one HIP
    event pair on the launch stream per mode.  GB/s in the same algorithmic bytes as
    roofline_hbm (gather_scatter_bytes_per_row; gather only: the row + reads, scatter
    only: the row + adds)."""
    import ncf_amd._lib as L
    lay = eng.lay
    if eng.model.model_type != "NeuMF-end" or eng.model.factor_num % 4:
        return None
    f, nl = eng.model.factor_num, eng.model.num_layers
    dev = eng.device
    st = torch.cuda.current_stream(dev)
    sp = L.stream_ptr(dev)
    scratch = torch.zeros_like(eng.grads)
    sink = torch.empty(L.PROBE_BLOCKS * 256, dtype=torch.float32, device=dev)
    full = gather_scatter_bytes_per_row(f, nl)
    half = (full - 8) // 2
    out = {}
    for mode, name, per_row in ((1, "gather", 8 + half), (2, "scatter", 8 + half), (3, "gather_scatter", full)):
        def launch():
            L.check(L.hip().ncf_probe_gather_scatter(ctypes.byref(lay), eng.flat.data_ptr(), scratch.data_ptr(),
                                                     sink.data_ptr(), eng.rows.data_ptr(), rows_n, mode, sp), "probe")
        launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            launch()
        e1.record(st)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / reps
        out[name] = {"GBps": per_row * rows_n / (ms * 1e-3) / 1e9, "us_per_launch": ms * 1e3}
    del scratch, sink
    return out


def adam_info(kt, eng, model):
    """The optimizer launch and the bytes it moves.  Dense Adam over the embedding
    tables: 32 B/param (read p, g, m, v; write p, m, v, g = 0).  ncf_reduce_adam_step
    also reads the tower slab (ncf_reduce_rows rows: the fused step's workgroups, or
    the layered path's atomic-spreading rows) and, on the factored path, the
    expansion's dW0 partials (ncf_fact_partials_bytes), and runs Adam
    on the tower straight from those sums (24 B/param: read p, m, v; write p, m, v)."""
    import ncf_amd._lib as L
    from ncf_amd import ops
    lay = eng.lay
    lib = L.hip()
    emb = sum(p.numel() for p, act in zip(list(model.ordered_params())[:4], ops.active_mask(model)[:4]) if act)
    tower = sum(p.numel() for p in list(model.ordered_params())[4:])
    stride = int(lib.ncf_slab_stride(L.ctypes.byref(lay)))
    slab_rows = int(lib.ncf_reduce_rows(L.ctypes.byref(lay)))
    partial = int(lib.ncf_fact_partials_bytes(L.ctypes.byref(lay)))
    slab_cols = stride
    if ops.fact_mode(lay):
        slab_cols = stride - (int(lay.b[0]) - int(lay.w[0]))  # W0's columns come from the partials
    if "ncf_train_step_ais" in kt:  # in-step Adam: no optimizer launch of its own
        return {"kernel": "in-step Adam inside ncf_train_step_ais (the previous step's update, on the fly for "
                          "the launch's reads, written by its extra workgroups)", "params": emb + tower,
                "bytes": 32 * (emb + tower), "ms": None,
                "note": "no separate launch: the step's launch time is kernel_ms.ncf_train_step_ais"}
    if "ncf_reduce_adam_step" in kt:
        b = 32 * emb + 24 * tower + slab_rows * slab_cols * 4 + partial
        ms = kt["ncf_reduce_adam_step"]
        out = {"kernel": "ncf_reduce_adam_step (slab reduce + Adam)", "params": emb + tower, "bytes": b,
               "bytes_detail": {"embedding_adam": 32 * emb, "tower_adam": 24 * tower,
                                "slab_read": slab_rows * slab_cols * 4, "w0_partials_read": partial},
               "ms": ms, "GB/s": b / (ms * 1e-3) / 1e9}
        return out
    if "ncf_lazy_adam_step" in kt or "ncf_lazy_adam_step_packed" in kt:
        # deferred Adam: the rows of lists A, B, C per step (include/ncf_hip.h
        # ncf_batch_touched), from the epoch's touched lists
        key = "ncf_lazy_adam_step" if "ncf_lazy_adam_step" in kt else "ncf_lazy_adam_step_packed"
        ms = kt[key]
        from ncf_amd.engine import touched_segments
        U, I = model.user_num, model.item_num
        nb = eng.num_batches
        lists = touched_segments(eng._touched_buf(eng.rows).cpu().numpy(), nb)
        wu = sum(p.numel() // U for p, a in zip(list(model.ordered_params())[:4], ops.active_mask(model)[:4])
                 if a and p.shape[0] == U)
        wi = sum(p.numel() // I for p, a in zip(list(model.ordered_params())[:4], ops.active_mask(model)[:4])
                 if a and p.shape[0] == I)
        rows_u = sum(len(lists[b][k]) for b in range(nb) for k in (0, 2, 4))
        rows_i = sum(len(lists[b][k]) for b in range(nb) for k in (1, 3, 5))
        grad_rows = sum(len(lists[b][0]) * wu + len(lists[b][1]) * wi for b in range(nb))
        moved = (rows_u * wu + rows_i * wi) / nb  # embedding floats read and written per step
        b = 24 * moved + 8 * grad_rows / nb + 24 * tower + slab_rows * slab_cols * 4 + partial
        return {"kernel": f"{key} (tower slab reduce + Adam, deferred embedding Adam)", "params": emb + tower,
                "embedding_floats_moved_per_step": moved, "dense_embedding_floats": emb,
                "bytes": b, "bytes_note": "p, m, v read + written (24 B) per embedding float of the rows "
                                          "of lists A, B, C (every row on the epoch's last batch), the gradient read "
                                          "+ cleared (8 B) for list A's rows, the tower as ncf_reduce_adam_step",
                "ms": ms, "GB/s": b / (ms * 1e-3) / 1e9}
    if "ncf_owner_adam" in kt:
        # dp_mode "owner": dense Adam on this rank's 1/W of the embedding rows (p, m, v read +
        # written), the W received contributions read and the next slices' rows written
        # (the two all-to-all buffers), the tower replicated
        ms = kt["ncf_owner_adam"]
        W = max(1, eng.world_size)
        P = eng._ow_plan
        xfer = 4 * W * (int(P.send_floats) + int(P.param_floats))
        b = 24 * emb / W + xfer + 24 * tower
        return {"kernel": "ncf_owner_adam (owned rows' dense Adam, tower Adam, next rows packed)",
                "params": emb / W + tower, "bytes": b,
                "bytes_detail": {"owned_adam": 24 * emb / W, "exchange_buffers": xfer, "tower_adam": 24 * tower},
                "ms": ms, "GB/s": b / (ms * 1e-3) / 1e9}
    b = 32 * (emb + tower)
    ms = kt.get("optimizer")
    if ms is None:  # an optimizer this accounting does not know: report the launch groups only
        return {"kernel": "optimizer", "params": emb + tower, "launch_groups_ms": dict(kt)}
    return {"kernel": "ncf_adam_step", "params": emb + tower, "bytes": b, "ms": ms, "GB/s": b / (ms * 1e-3) / 1e9}


def _kname(n):
    """Kernel name as the summaries key it: the fused step's template gained a trailing
    AIS flag in round 5 (`..., NW, false>`), older summaries lack it -- both match."""
    n = str(n)
    return n[:-len(", false>")] + ">" if n.endswith(", false>") and "ncf_step_kernel<" in n else n


def pmc_traffic(config, names):
    """HBM bytes per launch of `names` from the newest committed rocprofv3 PMC summary
    of THIS config (profiles/r*_prof_summary.json with "config" == config, written by
    scripts/profile.sh + scripts/prof_summary.py from separate FETCH_SIZE and
    WRITE_SIZE passes: bytes = (2 * FETCH_SIZE + WRITE_SIZE) KB * 1024, the gfx950
    correction of the MI355X guide).  (None, None) if there is none."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_prof_summary.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("config") != config:
            continue
        got = {_kname(k.get("kernel")): k.get("hbm_bytes_corrected") for k in d.get("kernels", [])}
        if all(got.get(_kname(n)) for n in names):
            return float(sum(got[_kname(n)] for n in names)), os.path.relpath(path, ROOT)
    return None, None


def host_facts():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return {"nproc": os.cpu_count(), "cpus_available": avail, "cpu_model": model}


class _RefLikeDataset:
    """Per-sample view of an epoch like the reference NCFData (datasets.py:71-83):
    __getitem__ returns python ints, batched by the stock DataLoader's collate."""

    def __init__(self, users, items, labels):
        self.u, self.i, self.y = users, items, labels

    def __len__(self):
        return len(self.u)

    def __getitem__(self, idx):
        return int(self.u[idx]), int(self.i[idx]), int(self.y[idx])


def _oracle_steps(cfg, U, I, batch, seconds, threads, users=None, items=None, labels=None, seed=0):
    """Adam steps of the oracle model (the reference NCF restated on stock torch CPU
    ops + torch.optim.Adam) on `batch`-row batches for ~`seconds`: rows/s.  Batches
    come from the given epoch stream, or are random ids in the model's id space."""
    from oracle import ncf_oracle as O
    shape, f, L, _ = CONFIGS[cfg]
    torch.set_num_threads(threads)
    torch.manual_seed(seed)
    m = O.OracleNCF(U, I, f, L, 0.0, MODEL.get(cfg, "NeuMF-end"))
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    rng = np.random.default_rng(seed)
    if users is None:
        n = batch * 8
        users, items = rng.integers(1, U, n), rng.integers(1, I, n)
        labels = (rng.random(n) < 0.2).astype(np.int64)
    nb = max(1, len(users) // batch)
    bat = lambda b: (users[b * batch:(b + 1) * batch], items[b * batch:(b + 1) * batch],  # noqa: E731
                     labels[b * batch:(b + 1) * batch])
    O.train_steps(m, opt, *[[x] for x in bat(0)])  # warm-up
    steps, t0 = 0, time.perf_counter()
    while True:
        u, i, y = bat((1 + steps) % nb)
        O.train_steps(m, opt, [u], [i], [y])
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": steps * batch / el, "steps": steps, "seconds": round(el, 2), "threads": threads,
            "ms_per_step": el / steps * 1e3}


SWEEP_THREADS = (8, 16, 32, 64, 128)


def cpu_baseline(cfg, seconds, script_epoch=True):
    """BASELINE.md section 3 on the host cores (run in a child process that never
    touches the GPU): the oracle -- the reference model restated on stock PyTorch CPU
    ops + torch.optim.Adam, `kind` "port" -- timed
      * step-only on the config's epoch stream at each of SWEEP_THREADS torch threads
        (the best is `value`, its count `cores`) and at os.cpu_count() threads;
      * step-only at C2 and C4 shapes (random ids) at the best count;
      * a script-equivalent epoch (train_neumf.py:98-131): ng_sample (the oracle's
        C restatement), the stock DataLoader(shuffle=True, num_workers=4) over a
        per-sample dataset, zero_grad/forward/BCE/backward/Adam per batch, and the
        metrics() pass (forward over the test candidates + HR/NDCG), at the best count."""
    from oracle import ncf_oracle as O
    shape, f, L, batch = CONFIGS[cfg]
    ds, _ = make_train_data(cfg)
    U, I = ds["user_num"], ds["item_num"]
    pu, pi = ds["train_users"], ds["train_items"]
    facts = host_facts()
    t0 = time.perf_counter()
    neg = O.ng_sample(pu, pi, I, 4, 0)
    t_sample = time.perf_counter() - t0
    users = np.concatenate([pu, np.repeat(pu, 4)]).astype(np.int64)
    items = np.concatenate([pi, neg]).astype(np.int64)
    labels = np.concatenate([np.ones(len(pu), np.int64), np.zeros(len(neg), np.int64)])
    perm = O.epoch_order(len(users), torch.Generator().manual_seed(0))
    su, si, sy = users[perm], items[perm], labels[perm]
    threads_all = facts["nproc"]
    # thread sweep: the best count is `value` (and `cores`); a sweep point takes
    # ~seconds / 2 of steps after one warm-up step
    sweep = {}
    for t in SWEEP_THREADS:
        sweep[t] = _oracle_steps(cfg, U, I, batch, seconds / 2, t, su, si, sy)
    best = max(sweep, key=lambda t: sweep[t]["value"])
    out = {"unit": "interactions/s", "kind": "port", "cores": best,
           "sample": f"{cfg.upper()} step-only: {batch}-row Adam steps of the oracle NCF({U},{I},{f},{L}) on the "
                     f"shuffled epoch stream, ~{seconds / 2:.0f} s at each of {list(SWEEP_THREADS)} torch threads "
                     f"(value: the best, {best}) and at os.cpu_count() threads; C2/C4-shape step-only and one "
                     f"script-equivalent epoch at the best count beside it",
           **facts}
    out["value"] = sweep[best]["value"]
    out["threads_best"] = best
    out["thread_sweep"] = {str(t): r for t, r in sweep.items()}
    out["step_only_all_threads"] = _oracle_steps(cfg, U, I, batch, seconds / 2, threads_all, su, si, sy)
    out["c2_step_only"] = _oracle_steps("c2", 6041, 3707, 1024, seconds / 3, best)
    out["c4_step_only"] = _oracle_steps("c4", 138494, 26745, 65536, seconds / 3, best)
    if script_epoch:
        from torch.utils.data import DataLoader
        torch.set_num_threads(best)
        torch.manual_seed(0)
        m = O.OracleNCF(U, I, f, L, 0.0, MODEL.get(cfg, "NeuMF-end"))
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        t0 = time.perf_counter()
        neg = O.ng_sample(pu, pi, I, 4, 1)
        items_e = np.concatenate([pi, neg]).astype(np.int64)
        loader = DataLoader(_RefLikeDataset(users, items_e, labels), batch_size=batch, shuffle=True, num_workers=4)
        t_loop = time.perf_counter()
        nb = 0
        for u, i, y in loader:
            opt.zero_grad()
            loss = O.bce_mean(m(u, i), y)
            loss.backward()
            opt.step()
            nb += 1
        t_eval = time.perf_counter()
        tu = np.repeat(ds["test_users"], 100).astype(np.int64)
        ti = np.concatenate([ds["test_items"][:, None], ds["test_negatives"]], 1).reshape(-1).astype(np.int64)
        with torch.no_grad():
            lg = m(torch.from_numpy(tu), torch.from_numpy(ti)).numpy()
        HR, _ = O.metrics_np(lg, ti, 100, 10)
        t1 = time.perf_counter()
        out["script_epoch"] = {"seconds": t1 - t0, "interactions_per_s": len(users) / (t1 - t0),
                               "ng_sample_s": t_loop - t0, "train_loop_s": t_eval - t_loop, "metrics_s": t1 - t_eval,
                               "batches": nb, "HR@10": float(np.mean(HR)), "threads": best, "num_workers": 4}
    out["ng_sample_s"] = t_sample
    return out


def cpu_baseline_child(cfg, seconds, script_epoch=True):
    """Run cpu_baseline in a child process (no HIP context: the DataLoader's worker
    processes fork from it) and return its JSON."""
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", "--config", cfg,
           "--cpu-seconds", str(seconds)] + ([] if script_epoch else ["--no-script-epoch"])
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=900)
    if r.returncode != 0:
        return {"error": r.stderr[-2000:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


def make_train_data(cfg, seed=0):
    from ncf_amd import synthetic
    from ncf_amd.data import NCFData
    shape = CONFIGS[cfg][0]
    ds = synthetic.make_dataset(shape, seed=seed)
    train = NCFData(np.stack([ds["train_users"], ds["train_items"]], 1), ds["item_num"], None, 4, True)
    return ds, train


def engine_for(cfg, dev, global_batch, world=1, rank=0, group=None):
    """(engine, model, pipeline) of config `cfg` at `global_batch` (diagnostic scripts)."""
    ds, train = make_train_data(cfg)
    return setup_engine(cfg, ds, train, world, rank, dev, group, global_batch)


def setup_engine(cfg, ds, train, world, rank, dev, group, global_batch, seed=0):
    """Bit-exact epoch pipeline over the resident data set -> NCF + TrainEngine.
    Identical on every rank (seeded)."""
    from ncf_amd.engine import TrainEngine
    from ncf_amd.pipeline import EpochPipeline
    U, I = ds["user_num"], ds["item_num"]
    np.random.seed(seed)
    torch.manual_seed(seed)
    model, dist = build_model(cfg, U, I, dev)
    pipe = EpochPipeline(train, dev, global_batch, I, user_num=U, prefetch=True, canonical=world > 1)
    eng = TrainEngine(model, lr=1e-3, world_size=world, rank=rank, process_group=group,
                      distill=None if dist is None else dist.device_plan())
    eng.stream_buffers = pipe.buffers  # the pipeline alternates two: graphs captured for both up front
    pipe.on_built = eng.owner_prebuild  # dp_mode "owner": each epoch's bucket lists built with the epoch
    eng.set_epoch_stream(pipe.next_epoch(peek_eval_draw=False), global_batch, checked=True)

    def next_epoch():  # fresh negatives + permutation (no metrics() pass between bench epochs)
        eng.set_epoch_stream(pipe.next_epoch(peek_eval_draw=False), global_batch, checked=True)
    eng.next_epoch = next_epoch
    return eng, model, pipe


# Where the boundary's host work goes (NCF_BENCH_BOUNDARY=early|top|auto, default auto):
# early for epochs of at most EARLY_MAX_STEPS steps, else at the top of the next epoch.
# Measured on the box (profiles/r03_evidence/ab_boundary.json, same session A/B):
# C3 (76 steps per epoch) 57-62 us/step early against 71-75 top -- the host is not
# ahead of a 4.5 ms epoch at its start; C2 (4,855) 24.2-25.0 early against 22.3 top,
# C5 (19,418) 14.7 against 14.0 -- a host running whole long epochs ahead slows the
# small steps (the frozen rate is the same in both).
BOUNDARY = os.environ.get("NCF_BENCH_BOUNDARY", "auto")
WARM_S = float(os.environ.get("NCF_BENCH_WARM_S", "0.5"))
EARLY_MAX_STEPS = 1024
# fresh epochs of the `sustained` figure (epochs above EARLY_MAX_STEPS steps: one)
SUSTAINED_EPOCHS = int(os.environ.get("NCF_BENCH_SUSTAINED_EPOCHS", "8"))


def _early_boundary(eng):
    return BOUNDARY == "early" or (BOUNDARY == "auto" and eng.num_batches <= EARLY_MAX_STEPS)


def run_steps(eng, n_steps, use_graph):
    """n_steps optimizer steps; a new epoch (fresh negatives and permutation)
    starts at every epoch boundary inside the timed region.  The boundary's host
    work (the pipeline join, the reference's RNG draws, the stream switch) is done
    as soon as an epoch's steps are enqueued, while the device still runs them, for
    short epochs (_early_boundary); a timed region of E whole epochs holds E such
    boundaries (the last one for the epoch after it), the warm-up's last boundary
    prepared the first.  Long epochs take it at the top of the next epoch.  The
    draws happen in the reference's order either way."""
    done = 0
    while done < n_steps:
        pos = eng.batches_done % eng.num_batches
        if pos == 0 and eng.batches_done > 0 and not getattr(eng, "boundary_ready", False):
            eng.next_epoch()
        eng.boundary_ready = False
        k = min(n_steps - done, eng.num_batches - pos)
        eng.run(k, use_graph=use_graph)
        eng.batches_done += k
        done += k
        if eng.batches_done % eng.num_batches == 0 and _early_boundary(eng):
            eng.next_epoch()
            eng.boundary_ready = True


def e2e_fit(cfg, ds, dev, epochs):
    """Trainer.fit -- the loop scripts/train_neumf.py runs (per epoch: ng_sample,
    DataLoader order, the steps, metrics() over the leave-one-out test set) --
    at this config on a fresh model; epoch wall times as the scripts print them."""
    from torch.utils.data import DataLoader
    from ncf_amd.data import NCFData
    from ncf_amd.trainer import Trainer
    shape, f, nl, batch = CONFIGS[cfg]
    U, I = ds["user_num"], ds["item_num"]
    np.random.seed(1)
    torch.manual_seed(1)
    model, dist = build_model(cfg, U, I, dev)
    train = NCFData(np.stack([ds["train_users"], ds["train_items"]], 1), I, None, 4, True)
    tu = np.repeat(ds["test_users"], 100)
    ti = np.concatenate([ds["test_items"][:, None], ds["test_negatives"]], 1).reshape(-1)
    test = NCFData(np.stack([tu, ti], 1), I, None, 0, False)
    tr = Trainer(model, train, DataLoader(test, batch_size=100, shuffle=False), batch_size=batch, lr=1e-3,
                 top_k=10, device=dev, verbose=False, distill=dist)
    tr.fit(1)  # graph capture, prefetch start-up
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    tr.fit(epochs)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    n = len(train)
    return {"value": epochs * n / wall, "unit": "interactions/s", "wall_s": wall,
            "epoch_device_s": [h["device_time"] for h in tr.history[1:]], "rows_per_epoch": n, "epochs": epochs,
            "HR@10": [round(h["hr"], 4) for h in tr.history],
            "note": "wall clock of Trainer.fit(epochs) (per epoch: fresh negatives and permutation, the "
                    "steps, metrics() over the leave-one-out test set, the printed-line readback), after "
                    "one warm-up fit(1)",
            "prefetch_hits": tr._pipe.stats["prefetch_hits"] if tr._pipe is not None else None,
            "pipeline_depth": tr._pipe.depth if tr._pipe is not None else None,
            "boundary_join_ms": [round(x[0], 2) for x in tr._pipe.stats.get("boundary_ms", [])[1:]]
            if tr._pipe is not None else None}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(argv, n):
    """`bench.py --gpus N` without a launcher: N child processes of this script, one
    per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR 127.0.0.1 / MASTER_PORT),
    started before this process touches any GPU; rank 0's stdout is the JSON line.
    If a rank fails the others are stopped.  Returns the worst exit code."""
    import signal
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL, start_new_session=True))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or code
                for q in live:  # a failed rank: the others would wait in a collective forever
                    try:
                        os.killpg(q.pid, signal.SIGTERM)
                    except OSError:
                        pass
        time.sleep(0.05)
    return rc


def _max_over_ranks(x, group, dev):
    if group is None:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def _barrier(group, dev):
    if group is not None:
        import torch.distributed as dist
        if dev.type == "cuda":
            dist.barrier(group=group, device_ids=[dev.index])
        else:
            dist.barrier(group=group)


def snapshot_state(eng):
    """Copies of the engine's trained state (parameters, Adam moments, control block,
    loss history, deferred-Adam row steps)."""
    names = ("flat", "exp_avg", "exp_avg_sq", "ctl", "loss_hist", "_last")
    return {k: getattr(eng, k).clone() for k in names if getattr(eng, k, None) is not None}


def restore_state(eng, snap):
    """Back to snapshot_state's copies, in place (captured graphs keep their pointers)."""
    for k, v in snap.items():
        getattr(eng, k).copy_(v)
    torch.cuda.synchronize(eng.device)


def measure(cfg, ds, train, world, rank, dev, group, global_batch, steps, warmup, use_graph, whole_epochs=True):
    """Warm-up, then whole fresh epochs timed (>= `steps` optimizer steps, rounded up
    to whole epochs of `global_batch`-row global batches: every epoch in the timed
    region draws new negatives and a new permutation), then the same number of steps
    on the last epoch stream reused (`frozen`).  Max over ranks, barrier +
    synchronize on both sides of each timed region.  whole_epochs=False (--profile-run:
    rocprofv3 passes serialise every launch): exactly `warmup` and `steps` steps."""
    eng, model, pipe = setup_engine(cfg, ds, train, world, rank, dev, group, global_batch)
    nb = eng.num_batches
    n_rows = eng.n_total
    # warm-up: whole epochs, at least `warmup` steps and, with whole epochs, at least
    # WARM_S seconds -- the first process on a fresh box ran its first timed C3 epoch
    # at 61 us/step after one or two warm-up epochs (~10 ms) against 57 in the next
    # processes on the same box, with the same host boundary times (a device-side
    # ramp; the frozen rate right after it was 56.7)
    warm = max(1, -(-max(1, warmup) // nb)) * nb if whole_epochs else max(1, warmup)
    eng.batches_done = 0
    t_w = time.perf_counter()
    run_steps(eng, warm, use_graph)
    torch.cuda.synchronize(dev)
    # every rank must run the same number of steps (each step is a collective at N > 1):
    # another epoch while any rank is short of WARM_S.  Those extra epochs only warm the
    # device: the trained state goes back to the one the requested warm-up left (the
    # quality figures stay those of a few epochs of training, as in the reference's runs)
    snap0 = None
    extra = 0
    while whole_epochs and _max_over_ranks(float(time.perf_counter() - t_w < WARM_S), group, dev) > 0:
        if snap0 is None:
            snap0 = snapshot_state(eng)
        run_steps(eng, nb, use_graph)
        extra += nb
        torch.cuda.synchronize(dev)
    warm_s = time.perf_counter() - t_w
    if snap0 is not None:
        restore_state(eng, snap0)
        eng.batches_done -= extra  # the control block's batch / step went back with the state
    epochs = max(1, -(-steps // nb)) if whole_epochs else steps / nb
    k = int(round(epochs * nb))
    _barrier(group, dev)
    torch.cuda.synchronize(dev)
    e0 = pipe.stats["epochs"]
    t0 = time.perf_counter()
    run_steps(eng, k, use_graph)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    _barrier(group, dev)
    dt = _max_over_ranks(dt, group, dev)
    fresh = pipe.stats["epochs"] - e0
    losses = eng.epoch_losses()
    final_loss = float(losses[(eng.state_step() - 1) % nb])
    # the trained state as the timed epochs left it: the quality figures are taken from
    # it, after the frozen run and the kernel timings below (restore_state)
    snap = snapshot_state(eng)
    # the same steps on the current epoch stream, reused (the step kernel wraps to the
    # epoch's first batch): the device + exchange rate beside `value`
    _barrier(group, dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    eng.run(k, use_graph=use_graph)
    torch.cuda.synchronize(dev)
    dtf = time.perf_counter() - t0
    _barrier(group, dev)
    dtf = _max_over_ranks(dtf, group, dev)
    ne = max(1, int(np.ceil(epochs)))
    hm = pipe.stats.get("host_ms", [])[-ne:]
    host = {k2: float(np.mean([h[k2] for h in hm if k2 in h])) for k2 in ("sample", "words", "stage")
            if any(k2 in h for h in hm)}
    bm = pipe.stats.get("boundary_ms", [])[-ne:]
    if bm:
        host["boundary_join"] = float(np.mean([x[0] for x in bm]))
        host["boundary_rest"] = float(np.mean([x[1] for x in bm]))
    host["sampler_threads"] = pipe.ds._get_sampler().threads if pipe.S else 0
    host["words_threads"] = pipe._wordgen.threads
    # sustained: SUSTAINED_EPOCHS more fresh epochs from the timed state -- each epoch's
    # negatives, permutation and grouping built while earlier epochs train (the
    # pipeline's side-stream build shares the device with the steps), as a long
    # training run pays it; `value`'s short timed region starts with two epochs
    # already built during the warm-up
    sustained = None
    ns = SUSTAINED_EPOCHS if nb <= EARLY_MAX_STEPS else min(1, SUSTAINED_EPOCHS)
    if whole_epochs and ns > 0:
        restore_state(eng, snap)
        _barrier(group, dev)
        torch.cuda.synchronize(dev)
        e1 = pipe.stats["epochs"]
        t0 = time.perf_counter()
        run_steps(eng, ns * nb, use_graph)
        torch.cuda.synchronize(dev)
        dts = time.perf_counter() - t0
        _barrier(group, dev)
        dts = _max_over_ranks(dts, group, dev)
        hs = pipe.stats.get("host_ms", [])[-ns:]
        sustained = {"value": ns * n_rows / dts, "ms_per_step": dts / (ns * nb) * 1e3, "epochs": ns,
                     "fresh_epochs": pipe.stats["epochs"] - e1,
                     "device_build_ms_per_epoch": None,
                     "host_stage_ms": float(np.mean([h["stage"] for h in hs if "stage" in h])) if hs else None,
                     "note": "consecutive fresh epochs after the timed ones, every epoch's host sampling and device "
                             "build (rows, permutation, grouping on a side stream) inside the region; `value` times "
                             "the driver's epochs, whose streams the warm-up prefetched"}
        ev = pipe.device_ms()
        if ev is not None:
            sustained["device_build_ms_per_epoch"] = float(ev[0] + ev[1])
    return {"eng": eng, "model": model, "pipe": pipe, "snap": snap, "value": epochs * n_rows / dt, "dt": dt, "steps": k,
            "sustained": sustained,
            "epochs": epochs, "fresh_epochs": fresh, "rows_per_epoch": n_rows, "batches_per_epoch": nb,
            "warmup_run": {"steps": warm + extra, "seconds": round(warm_s, 3), "trained_steps_kept": warm,
                           "note": f"untimed: whole epochs, >= --warmup steps and >= {WARM_S} s (device ramp on a fresh box); "
                                   "the trained state of the steps past --warmup is discarded"},
            "final_loss": final_loss, "frozen_value": k * n_rows / nb / dtf, "frozen_ms_per_step": dtf / k * 1e3,
            "epoch_host_ms": host}


def harness_main(args, world, rank):
    """--cpu-harness (tests only): the launch / rendezvous / timing / JSON contract of
    this script on the CPU over gloo, with no device work -- each rank draws the
    config's epochs through the product host sampler and takes its shard of every
    global batch.  The line says so; it is not a measurement of the hot path."""
    import torch.distributed as dist
    from ncf_amd.distributed import shard_range
    group = None
    if world > 1:
        dist.init_process_group("gloo")
        group = dist.group.WORLD
    if os.environ.get("NCF_BENCH_FAIL_RANK") == str(rank):  # tests: a rank dying after rendezvous
        raise SystemExit(3)
    shape, f, nl, global_batch = CONFIGS[args.config]
    per_gpu = -(-global_batch // world)
    ds, train = make_train_data(args.config)
    dev = torch.device("cpu")
    _barrier(group, dev)
    t0 = time.perf_counter()
    np.random.seed(0)
    n = 0
    for _ in range(max(1, args.harness_epochs)):
        train.ng_sample()
        m = len(train)
        for b0 in range(0, m, global_batch):
            lo, hi = shard_range(min(global_batch, m - b0), world, rank)
            n += hi - lo
    dt = _max_over_ranks(time.perf_counter() - t0, group, dev)
    rows = torch.tensor([n], dtype=torch.int64)
    if group is not None:
        dist.all_reduce(rows, group=group)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": int(rows.item()) / dt, "unit": "interactions/s", "n_gpus": world,
                          "harness": "cpu-gloo: host sampler + shard arithmetic only, no device work",
                          "config": {"workload": args.config.upper(), "global_batch": global_batch,
                                     "per_gpu_batch": per_gpu, "parallelism": f"dp{world}"}}), flush=True)
    if group is not None:
        dist.barrier(group=group)
        dist.destroy_process_group()


METRIC = "training interactions/sec + HR@10, NeuMF factors=64 ml-1m, 1/2/4/8 MI355X"


def newest_profile(config, kernel_names):
    """(mfma_busy_frac of the first kernel, source) from the newest SQ pass of this
    config in profiles/ (scripts/profile.sh), or (None, None)."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_prof_summary.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("config") != config:
            continue
        for k in d.get("kernels", []):
            if _kname(k.get("kernel")) == _kname(kernel_names[0]) and k.get("mfma_busy_frac") is not None:
                return float(k["mfma_busy_frac"]), os.path.relpath(path, ROOT)
    return None, None


LAYERED_STEP_PREFIXES = ("ncf::lyr_", "ncf::fact_expand_kernel")


def layered_profile(config):
    """(HBM bytes per step, MFMA-busy fraction, source) of the layered path's step from
    the newest committed rocprofv3 summary of this config: every kernel of
    ncf_train_step (LAYERED_STEP_PREFIXES), each weighted by its launches per step
    (calls / the calls of lyr_proj_kernel, the step's first launch); the busy fraction
    time-weighted over those kernels.  (None, None, None) if there is none."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_prof_summary.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("config") != config:
            continue
        ks = [k for k in d.get("kernels", []) if str(k.get("kernel", "")).startswith(LAYERED_STEP_PREFIXES)]
        steps = max((k.get("calls") or 0 for k in ks if k["kernel"].startswith("ncf::lyr_proj_kernel")), default=0)
        if not steps or not all(k.get("hbm_bytes_corrected") for k in ks):
            continue
        traffic = sum(k["hbm_bytes_corrected"] * k["calls"] / steps for k in ks)
        t = [(k["avg_us"] * k["calls"] / steps, k.get("mfma_busy_frac")) for k in ks]
        busy = (sum(a * b for a, b in t) / sum(a for a, _ in t)) if all(b is not None for _, b in t) else None
        return float(traffic), busy, os.path.relpath(path, ROOT)
    return None, None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200, help="timed steps, rounded up to whole epochs")
    ap.add_argument("--warmup", type=int, default=20, help="warm-up steps, rounded up to whole epochs")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--kernel-steps", type=int, default=20, help="eager steps timed per kernel with HIP events")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--skip-cpu-baseline", action="store_true")
    ap.add_argument("--no-script-epoch", action="store_true")
    ap.add_argument("--skip-eval", action="store_true")
    ap.add_argument("--no-weak", action="store_true", help="N > 1: skip the weak-scaling (global batch x N) field")
    ap.add_argument("--e2e-epochs", type=int, default=16, help="Trainer.fit epochs for the e2e figure (0: skip)")
    ap.add_argument("--profile-run", action="store_true",
                    help="exactly --warmup/--steps steps (not whole epochs): for rocprofv3 passes, not a bench line")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-harness", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--harness-epochs", type=int, default=1, help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.cpu_baseline_only:  # child of cpu_baseline_child: no GPU
        print(json.dumps(cpu_baseline(args.config, args.cpu_seconds, not args.no_script_epoch)), flush=True)
        return None
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # spawn the ranks ourselves, before anything touches a GPU
        sys.exit(spawn_ranks(sys.argv[1:], args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.cpu_harness:
        return harness_main(args, world, rank)
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    # rehearsal of the N > 1 flow on a one-GPU box (not a measurement): every rank on
    # cuda:0 (NCF_BENCH_SAME_DEVICE=1) over gloo (NCF_BENCH_BACKEND=gloo; RCCL refuses
    # two ranks on one device)
    rehearsal = os.environ.get("NCF_BENCH_SAME_DEVICE") == "1"
    dev = torch.device("cuda", 0 if rehearsal else local)
    torch.cuda.set_device(dev)
    group = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("NCF_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        group = dist.group.WORLD

    shape, f, nl, global_batch = CONFIGS[args.config]
    per_gpu = -(-global_batch // world)
    mtype = MODEL.get(args.config, "NeuMF-end")
    use_graph = not args.no_graph
    t_data = time.perf_counter()
    ds, train = make_train_data(args.config)
    U, I = ds["user_num"], ds["item_num"]
    t_data = time.perf_counter() - t_data

    # ---- headline: the reference's global batch split over the N ranks (strong
    # scaling), whole fresh epochs
    m = measure(args.config, ds, train, world, rank, dev, group, global_batch, args.steps, args.warmup, use_graph,
                whole_epochs=not args.profile_run)
    eng, model, pipe = m["eng"], m["model"], m["pipe"]

    # ---- per-kernel live timing (HIP events on the launch stream) -------------
    kt = eng.time_kernels(args.kernel_steps)
    pipe_ms = []
    for _ in range(3):  # the epoch pipeline's device part: rows + randperm (side stream), grouping
        eng.next_epoch()
        eng.run(min(eng.num_batches, 100), use_graph=use_graph)
        pipe_ms.append(pipe.device_ms())
    kt["epoch_rows_randperm_side_stream"] = float(np.mean([x[0] for x in pipe_ms]))
    kt["epoch_grouping_side_stream"] = float(np.mean([x[1] for x in pipe_ms]))
    kt["epoch_host_ms"] = m["epoch_host_ms"]
    kt["ncf_train_step_per_launch_b2b"] = eng.time_train_kernel(50)
    from ncf_amd import ops
    import ncf_amd._lib as L
    fact = ops.fact_mode(eng.lay)
    path = L.supported(mtype, f, nl)
    dm = f * 2 ** (nl - 1)
    rows_per_launch = per_gpu
    ms = kt["ncf_train_step_per_launch_b2b"]
    alg_flops = tower_flops_per_row(f, nl, mtype) * rows_per_launch
    alg_tf = alg_flops / (ms * 1e-3) / 1e12
    xflops = executed_flops(f, nl, mtype, rows_per_launch, U + I, fact, path == L.PATH_FUSED)
    executed_tf = xflops / (ms * 1e-3) / 1e12
    bytes_launch = gather_scatter_bytes_per_row(f, nl) * rows_per_launch
    achieved_gbs = bytes_launch / (ms * 1e-3) / 1e9
    if path == L.PATH_FUSED:
        mode = {"GMF": 0, "MLP": 1}.get(mtype, 2)
        waves = (8, 4, 2, 1)[(int(eng.lay.flags) >> L.LAYOUT_GEO_SHIFT) & L.LAYOUT_GEO_MASK]
        names = [f"ncf::ncf_step_kernel<{f}, {nl}, {mode}, false, {'true' if fact else 'false'}, {waves}>"]
        if fact:
            names.append(f"ncf::fact_expand_kernel<{dm}>")
        kname = (f"ncf_step_kernel<{f},{nl},{mtype.split('-')[0]},FACT={str(fact).lower()}>"
                 + (f" + fact_expand_kernel<{dm}> (factored layer 0)" if fact else " (per-row layer 0)")
                 + "; launch group timed back to back")
        traffic, traffic_src = pmc_traffic(args.config, names) if world == 1 else (None, None)
        busy, busy_src = newest_profile(args.config, names) if world == 1 else (None, None)
    else:
        names = []
        traffic, busy, traffic_src = layered_profile(args.config) if world == 1 else (None, None, None)
        busy_src = traffic_src
        kname = ("layered path: all kernels of ncf_train_step (fwd/predict/bwd GEMMs); the fp32 GEMMs with "
                 "16-byte loads run as exact three-plane bf16 splits on v_mfma_f32_16x16x32_bf16 (six bf16 "
                 "products per fp32 product; peak kept at the fp32 MFMA figure)")

    # ---- the gather / scatter rate against a measured cache ceiling: the same
    # access pattern alone (ncf_probe_gather_scatter) on the same tables and rows
    roofline_cache = None
    if path == L.PATH_FUSED and world == 1:
        probe = cache_probe(eng, rows_per_launch)
        if probe is not None:
            ceil = probe["gather_scatter"]["GBps"]
            tables_mb = 4 * (U + I) * (f + dm) / 1e6
            state_mb = 4 * 4 * int(eng.lay.total) / 1e6  # params, grads, two Adam moments
            roofline_cache = {
                "achieved": achieved_gbs, "reference_rate": ceil, "unit": "GB/s", "ratio": achieved_gbs / ceil,
                "probe": probe, "tables_MB": round(tables_mb, 2), "model_state_MB": round(state_mb, 2),
                "resident": ("L2/MALL (tables fit the 4 MB L2 per XCD and the 256 MB MALL)" if tables_mb <= 4 else
                             "MALL-assisted (tables and optimizer state fit the 256 MB MALL)" if state_mb <= 256 else
                             "HBM (model state above the 256 MB MALL)"),
                "note": "achieved = the step launch group's gather+scatter algorithmic bytes (roofline_hbm) / its "
                        "time; reference_rate = ncf_probe_gather_scatter: the same 16-byte row gathers and "
                        "row-contiguous float-atomic adds, same rows and tables, no arithmetic, launches back to "
                        "back.  Not a ceiling: the probe issues one atomic per gathered float, the step sums item "
                        "runs first (and the factored layer 0 scatters D0 rows), so ratio > 1 is possible"}

    # ---- weak scaling (extra field): global batch x N, per-GPU batch fixed -----
    weak = None
    if world > 1 and not args.no_weak:
        pipe.close()
        w = measure(args.config, ds, train, world, rank, dev, group, global_batch * world, args.steps,
                    args.warmup, use_graph)
        weak = {"value": w["value"], "ms_per_step": w["dt"] / w["steps"] * 1e3, "steps": w["steps"],
                "global_batch": global_batch * world, "per_gpu_batch": global_batch,
                "note": "the per-GPU batch held at the single-GPU batch (a different training trajectory "
                        "from the reference's batch size); `value` is the reference's global batch"}
        w["pipe"].close()

    # ---- quality: HR@10 / NDCG@10 on the leave-one-out test set ---------------
    hr10 = ndcg10 = None
    restore_state(eng, m["snap"])  # quality of the state the timed epochs trained, nothing after
    if not args.skip_eval and rank == 0:
        from ncf_amd.metrics import evaluate_arrays
        tu = np.repeat(ds["test_users"], 100)
        ti = np.concatenate([ds["test_items"][:, None], ds["test_negatives"]], 1).reshape(-1)
        HR, NDCG = evaluate_arrays(model, tu, ti, 100, 10)
        hr10, ndcg10 = float(np.mean(HR)), float(np.mean(NDCG))
    if weak is None:
        pipe.close()

    out = None
    if rank == 0:
        e2e = None
        if args.e2e_epochs > 0 and world == 1:
            e2e = e2e_fit(args.config, ds, dev, args.e2e_epochs)
        cpu = None
        if not args.skip_cpu_baseline and world == 1:
            cpu = cpu_baseline_child(args.config, args.cpu_seconds, not args.no_script_epoch)
        dt, k = m["dt"], m["steps"]
        out = {
            "metric": METRIC,
            "value": m["value"],
            "unit": "interactions/s",
            "n_gpus": world,
            "steps": k,
            "warmup": args.warmup,
            "warmup_run": m["warmup_run"],
            "ms_per_step": dt / k * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": (f"synthetic {shape}-shaped ({U - 1:,} users x {I - 1:,} items, {len(ds['train_users']):,} "
                     f"train positives, 4 bit-exact sampled negatives each); {m['epochs']} whole epochs timed "
                     f"({k} steps, requested {args.steps}, rounded up), each with fresh negatives and permutation "
                     f"({m['fresh_epochs']} epoch boundaries in the timed region); seed 0"),
            "config": {"workload": f"{args.config.upper()}: NCF(user_num={U}, item_num={I}, factor_num={f}, "
                                   f"num_layers={nl}, {mtype}), Adam lr 1e-3"
                                   + (f"; response distillation (T 2.0, alpha 0.5) from a random-init teacher "
                                      f"NCF({C5_TEACHER[0]}, {C5_TEACHER[1]}, {C5_TEACHER[2]}) whose logits of "
                                      f"each epoch stream are one forward launch at the epoch boundary"
                                      if args.config == "c5" else ""),
                       "global_batch": global_batch, "per_gpu_batch": per_gpu, "parallelism": f"dp{world}",
                       "mlp_layers": [int(2 * f * 2 ** (nl - 1)) >> j for j in range(nl + 1)],
                       "dp_exchange": eng.dp_mode, "hip_graph": use_graph,
                       "rows_per_epoch": m["rows_per_epoch"], "steps_per_epoch": m["batches_per_epoch"]},
            "roofline": {"bound": "mfma", "achieved": executed_tf, "peak": 157.3, "unit": "TFLOP/s",
                         "frac": executed_tf / 157.3, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": kname, "kernel_ms": ms, "flops_per_launch": xflops,
                         "flops_note": "fp32 flops the kernels execute per launch (2 per MAC): per-row tower "
                                       "layers >= 1 and predict, the fused kernel's per-row layer-0 forward, the "
                                       "factored layer 0's per-entity GEMMs over the U + I table rows",
                         "hw_mfma_busy": busy, "hw_mfma_busy_source": busy_src,
                         "algorithmic": {"flops_per_launch": alg_flops, "achieved": alg_tf,
                                         "note": "SURVEY 8(d) per-row tower flops (6 sum s_k s_k+1 + predict) x rows; "
                                                 "the factored layer 0 does not execute the per-row layer-0 "
                                                 "backward it counts, so this rate is not a roofline fraction"}},
            "roofline_hbm": {"bound": "hbm", "achieved": achieved_gbs, "peak": 8000.0, "unit": "GB/s",
                             "frac": achieved_gbs / 8000.0, "bytes_per_launch": bytes_launch,
                             "traffic_GBps": (traffic / (ms * 1e-3) / 1e9) if traffic else None,
                             "note": ("gather+scatter algorithmic bytes of the same launch group" if path == L.PATH_FUSED
                                      else "gather+scatter algorithmic bytes over all layered-path kernels")},
            "roofline_cache": roofline_cache,
            "kernel_ms": kt,
            "adam": adam_info(kt, eng, model),
            "quality": {"HR@10": hr10, "NDCG@10": ndcg10, "epochs_trained": round(eng.state_step() / eng.num_batches, 2),
                        "last_batch_loss": m["final_loss"]},
            "e2e": e2e,
            "sustained": m["sustained"],
            "frozen_epoch": {"value": m["frozen_value"], "ms_per_step": m["frozen_ms_per_step"],
                             "note": "the same steps with the last epoch stream reused (no new negatives or "
                                     "permutation): device + exchange rate"},
            "weak_scaling": weak,
            "cpu_baseline": cpu,
            "setup_s": {"data": round(t_data, 2)},
        }
        if path != L.PATH_FUSED and f % 4 == 0:
            # the layered GEMMs run on v_mfma_f32_16x16x32_bf16 (six bf16 products per fp32
            # product): the ceiling of those instructions in fp32-equivalent flops is the
            # dense bf16 peak / 6
            out["roofline"]["bf16_split_ceiling"] = {
                "peak": 2500.0 / 6, "unit": "TFLOP/s (fp32-equivalent)", "frac": executed_tf / (2500.0 / 6),
                "note": "the same executed flops against the bf16-split GEMM core's own ceiling (2.5 PF dense bf16 / 6); "
                        "`frac` above is against the fp32 MFMA peak"}
        if rehearsal:
            out["rehearsal"] = (f"{world} ranks on one device over {os.environ.get('NCF_BENCH_BACKEND', 'nccl')}: "
                                "a check of the N > 1 flow, not a measurement")
        print(json.dumps(out), flush=True)
    if world > 1:
        _barrier(group, dev)
        torch.distributed.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
