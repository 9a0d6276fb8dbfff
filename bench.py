#!/usr/bin/env python3
"""Headline benchmark: NeuMF training interactions/sec on MI355X.

Workload (BASELINE.json metric "training interactions/sec + HR@10, NeuMF
factors=64 ml-1m"): NCF(6041, 3707, factor_num=16,
num_layers=3, 'NeuMF-end') -- 64-wide MLP embeddings, tower [128,64,32,16] --
on ml-1m-shaped synthetic data (994,169 positives, 4 sampled negatives each),
65,536 rows per GPU per step, Adam lr 1e-3.

A "step" = fused fwd+loss+bwd kernel (+ the factored layer-0 expansion), tower-grad
reduction, (RCCL gradient exchange when N > 1), dense Adam -- the whole optimizer
step of scripts/train_neumf.py:111-115, captured into hipGraphs and replayed.
Every epoch inside the timed region is a fresh epoch of the reference loop: new
negatives (NCFData.ng_sample, bit-exact; host sampler, prefetched on a host thread
while the previous epoch trains) and a new DataLoader permutation (bit-exact
torch.randperm, on the device), packed, shuffled and grouped on the device
(ncf_amd.pipeline).  The data set itself is resident in HBM before the timed
region.  Per-GPU work is fixed (65,536 rows/GPU/step), so scaling is weak and
value = all ranks' rows / max-over-ranks time.

Also reported: `e2e` -- Trainer.fit (the scripts' loop: epochs + metrics() per
epoch) at the same config, rows per epoch / epoch wall time; `cpu_baseline` -- the
oracle (reference model restated on torch CPU ops) on the host cores.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, RCCL).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (dataset shape, factor_num, num_layers, rows per GPU per step)
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
    if "ncf_reduce_adam_step" in kt:
        b = 32 * emb + 24 * tower + slab_rows * slab_cols * 4 + partial
        ms = kt["ncf_reduce_adam_step"]
        return {"kernel": "ncf_reduce_adam_step (slab reduce + Adam)", "params": emb + tower, "bytes": b,
                "bytes_detail": {"embedding_adam": 32 * emb, "tower_adam": 24 * tower,
                                 "slab_read": slab_rows * slab_cols * 4, "w0_partials_read": partial},
                "ms": ms, "GB/s": b / (ms * 1e-3) / 1e9}
    b = 32 * (emb + tower)
    ms = kt["optimizer"]
    return {"kernel": "ncf_adam_step", "params": emb + tower, "bytes": b, "ms": ms, "GB/s": b / (ms * 1e-3) / 1e9}


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
        got = {k.get("kernel"): k.get("hbm_bytes_corrected") for k in d.get("kernels", [])}
        if all(got.get(n) for n in names):
            return float(sum(got[n] for n in names)), os.path.relpath(path, ROOT)
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


def cpu_baseline(cfg, ds, batch, seconds, threads):
    """The oracle (oracle/ncf_oracle.py: the reference model restated on stock
    PyTorch CPU ops + torch.optim.Adam) timed on the host cores: (i) steady-state
    Adam steps on `batch`-row batches of the real epoch stream for ~`seconds`, and
    (ii) a script-equivalent epoch -- ng_sample (the oracle's C restatement),
    the DataLoader permutation, packing, then every step of the epoch -- timed on
    the first batches and extrapolated to the epoch's batch count."""
    from oracle import ncf_oracle as O
    shape, f, L, _ = CONFIGS[cfg]
    U, I = ds["user_num"], ds["item_num"]
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    m = O.OracleNCF(U, I, f, L, 0.0, "NeuMF-end")
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    pu, pi = ds["train_users"], ds["train_items"]
    t0 = time.perf_counter()
    neg = O.ng_sample(pu, pi, I, 4, 0)
    t_sample = time.perf_counter() - t0
    users = np.concatenate([pu, np.repeat(pu, 4)])
    items = np.concatenate([pi, neg])
    labels = np.concatenate([np.ones(len(pu), np.int64), np.zeros(len(neg), np.int64)])
    t0 = time.perf_counter()
    perm = O.epoch_order(len(users), torch.Generator().manual_seed(0))
    t_perm = time.perf_counter() - t0
    nb = (len(users) + batch - 1) // batch
    bat = lambda b: (users[perm[b * batch:(b + 1) * batch]], items[perm[b * batch:(b + 1) * batch]],  # noqa: E731
                     labels[perm[b * batch:(b + 1) * batch]])
    O.train_steps(m, opt, *[[x] for x in bat(0)])  # warm-up
    steps, t0 = 0, time.perf_counter()
    while True:
        u, i, y = bat(1 + steps % (nb - 1)) if nb > 1 else bat(0)
        O.train_steps(m, opt, [u], [i], [y])
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    step_s = el / steps
    epoch_s = t_sample + t_perm + nb * step_s
    return {"value": steps * batch / el, "unit": "interactions/s", "cores": threads, "kind": "port",
            "sample": f"{steps} x {batch}-row Adam steps of the oracle on the epoch stream of {cfg.upper()} "
                      f"(reference NCF restated on torch CPU ops, NCF({U},{I},{f},{L})), {el:.1f} s on "
                      f"{threads} threads",
            "script_epoch_s": epoch_s,
            "script_epoch_note": f"ng_sample {t_sample:.2f} s + DataLoader permutation {t_perm:.2f} s + "
                                 f"{nb} steps x {step_s * 1e3:.1f} ms (steps timed on {steps}, extrapolated)",
            "script_epoch_interactions_per_s": len(users) / epoch_s,
            **host_facts(), "torch_threads": threads}


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
    pipe = EpochPipeline(train, dev, global_batch, I, user_num=U, prefetch=True)
    eng = TrainEngine(model, lr=1e-3, world_size=world, rank=rank, process_group=group,
                      distill=None if dist is None else dist.device_plan())
    eng.stream_buffers = pipe.buffers  # the pipeline alternates two: graphs captured for both up front
    eng.set_epoch_stream(pipe.next_epoch(peek_eval_draw=False), global_batch, checked=True)

    def next_epoch():  # fresh negatives + permutation (no metrics() pass between bench epochs)
        eng.set_epoch_stream(pipe.next_epoch(peek_eval_draw=False), global_batch, checked=True)
    eng.next_epoch = next_epoch
    return eng, model, pipe


def run_steps(eng, n_steps, use_graph):
    """n_steps optimizer steps; a new epoch (fresh negatives and permutation)
    starts at every epoch boundary inside the timed region."""
    done = 0
    while done < n_steps:
        pos = eng.batches_done % eng.num_batches
        if pos == 0 and eng.batches_done > 0:
            eng.next_epoch()
        k = min(n_steps - done, eng.num_batches - pos)
        eng.run(k, use_graph=use_graph)
        eng.batches_done += k
        done += k


def e2e_fit(cfg, ds, dev, epochs):
    """Trainer.fit -- the loop scripts/train_neumf.py runs (per epoch: ng_sample,
    DataLoader order, the steps, metrics() over the leave-one-out test set) --
    at this config on a fresh model; epoch wall times as the scripts print them."""
    from torch.utils.data import DataLoader
    from ncf_amd.data import NCFData
    from ncf_amd.trainer import Trainer
    shape, f, nl, per_gpu = CONFIGS[cfg]
    U, I = ds["user_num"], ds["item_num"]
    np.random.seed(1)
    torch.manual_seed(1)
    model, dist = build_model(cfg, U, I, dev)
    train = NCFData(np.stack([ds["train_users"], ds["train_items"]], 1), I, None, 4, True)
    tu = np.repeat(ds["test_users"], 100)
    ti = np.concatenate([ds["test_items"][:, None], ds["test_negatives"]], 1).reshape(-1)
    test = NCFData(np.stack([tu, ti], 1), I, None, 0, False)
    tr = Trainer(model, train, DataLoader(test, batch_size=100, shuffle=False), batch_size=per_gpu, lr=1e-3,
                 top_k=10, device=dev, verbose=False, distill=dist)
    tr.fit(1)  # graph capture, prefetch start-up
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    tr.fit(epochs)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    n = len(train)
    return {"value": epochs * n / wall, "unit": "interactions/s", "wall_s": wall,
            "epoch_device_s": [h["time"] for h in tr.history[1:]], "rows_per_epoch": n, "epochs": epochs,
            "HR@10": [round(h["hr"], 4) for h in tr.history],
            "note": "wall clock of Trainer.fit(epochs) (per epoch: fresh negatives and permutation, the "
                    "steps, metrics() over the leave-one-out test set, the printed-line readback), after "
                    "one warm-up fit(1)",
            "prefetch_hits": tr._pipe.stats["prefetch_hits"] if tr._pipe is not None else None,
            "pipeline_depth": tr._pipe.depth if tr._pipe is not None else None,
            "boundary_join_ms": [round(x[0], 2) for x in tr._pipe.stats.get("boundary_ms", [])[1:]]
            if tr._pipe is not None else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--kernel-steps", type=int, default=20, help="eager steps timed per kernel with HIP events")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--skip-cpu-baseline", action="store_true")
    ap.add_argument("--skip-eval", action="store_true")
    ap.add_argument("--e2e-epochs", type=int, default=16, help="Trainer.fit epochs for the e2e figure (0: skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run --nproc-per-node N")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    group = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)
        group = dist.group.WORLD

    shape, f, nl, per_gpu = CONFIGS[args.config]
    global_batch = per_gpu * world
    t_data = time.perf_counter()
    ds, train = make_train_data(args.config)
    U, I = ds["user_num"], ds["item_num"]
    eng, model, pipe = setup_engine(args.config, ds, train, world, rank, dev, group, global_batch)
    torch.cuda.synchronize(dev)
    t_data = time.perf_counter() - t_data

    # ---- warmup (first step eager, then capture) -----------------------------
    use_graph = not args.no_graph
    eng.batches_done = 0
    run_steps(eng, max(1, args.warmup), use_graph)
    torch.cuda.synchronize(dev)

    # ---- timed region ----------------------------------------------------------
    if world > 1:
        torch.distributed.barrier(group=group, device_ids=[local])
    torch.cuda.synchronize(dev)
    epochs0 = pipe.stats["epochs"]
    t0 = time.perf_counter()
    run_steps(eng, args.steps, use_graph)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    epochs_in_timed = pipe.stats["epochs"] - epochs0
    if world > 1:
        torch.distributed.barrier(group=group, device_ids=[local])
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=group)
        dt = float(t.item())
    rows = args.steps * global_batch
    value = rows / dt
    losses = eng.epoch_losses()
    final_loss = float(losses[(eng.state_step() - 1) % eng.num_batches])

    # ---- the same number of steps on the current epoch stream, reused (no fresh
    # negatives / permutation: the step kernel wraps to the epoch's first batch): the
    # device + exchange rate beside `value`, which the sequential host sampler bounds
    # once an epoch is only a few steps long (N >= 4 at 65,536 rows per GPU)
    if world > 1:
        torch.distributed.barrier(group=group, device_ids=[local])
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    eng.run(args.steps, use_graph=use_graph)
    torch.cuda.synchronize(dev)
    dt_frozen = time.perf_counter() - t0
    if world > 1:
        torch.distributed.barrier(group=group, device_ids=[local])
        t = torch.tensor([dt_frozen], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=group)
        dt_frozen = float(t.item())
    frozen = {"value": rows / dt_frozen, "ms_per_step": dt_frozen / args.steps * 1e3,
              "note": "the same steps with the last epoch stream reused (no new negatives or permutation): "
                      "device + exchange rate; `value` times fresh epochs, whose host sampler (sequential in "
                      "the reference's NumPy stream, ~3 ms per ml-1m epoch) bounds it once an epoch is only a "
                      "few global steps long"}

    # ---- per-kernel live timing (HIP events on the launch stream) -------------
    kt = eng.time_kernels(args.kernel_steps)
    pipe_ms = []
    for _ in range(3):  # the epoch pipeline's device part: rows + randperm (side stream), grouping
        eng.next_epoch()
        eng.run(min(eng.num_batches, 100), use_graph=use_graph)
        pipe_ms.append(pipe.device_ms())
    kt["epoch_rows_randperm_side_stream"] = float(np.mean([x[0] for x in pipe_ms]))
    kt["epoch_grouping_side_stream"] = float(np.mean([x[1] for x in pipe_ms]))
    hm = pipe.stats.get("host_ms", [])[-3:]
    kt["epoch_host_ms"] = {k: float(np.mean([h[k] for h in hm if k in h])) for k in ("sample", "words", "stage")
                           if any(k in h for h in hm)}
    bm = pipe.stats.get("boundary_ms", [])[1:]
    if bm:
        kt["epoch_host_ms"]["boundary_join"] = float(np.mean([x[0] for x in bm]))
        kt["epoch_host_ms"]["boundary_rest"] = float(np.mean([x[1] for x in bm]))
    kt["ncf_train_step_per_launch_b2b"] = eng.time_train_kernel(50)
    from ncf_amd import ops
    import ncf_amd._lib as L
    mtype = MODEL.get(args.config, "NeuMF-end")
    fact = ops.fact_mode(eng.lay)
    path = L.supported(mtype, f, nl)
    dm = f * 2 ** (nl - 1)
    rows_per_launch = per_gpu
    flops = tower_flops_per_row(f, nl, mtype) * rows_per_launch
    ms = kt["ncf_train_step_per_launch_b2b"]
    achieved_tf = flops / (ms * 1e-3) / 1e12
    xflops = executed_flops(f, nl, mtype, rows_per_launch, U + I, fact, path == L.PATH_FUSED)
    executed_tf = xflops / (ms * 1e-3) / 1e12
    bytes_launch = gather_scatter_bytes_per_row(f, nl) * rows_per_launch
    achieved_gbs = bytes_launch / (ms * 1e-3) / 1e9
    if path == L.PATH_FUSED:
        mode = {"GMF": 0, "MLP": 1}.get(mtype, 2)
        names = [f"ncf::ncf_step_kernel<{f}, {nl}, {mode}, false, {'true' if fact else 'false'}>"]
        if fact:
            names.append(f"ncf::fact_expand_kernel<{dm}>")
        kname = (f"ncf_step_kernel<{f},{nl},{mtype.split('-')[0]},FACT={str(fact).lower()}>"
                 + (f" + fact_expand_kernel<{dm}> (factored layer 0)" if fact else " (per-row layer 0)")
                 + "; launch group timed back to back")
        traffic, traffic_src = pmc_traffic(args.config, names)
    else:
        names, traffic, traffic_src = [], None, None
        kname = "layered path: all kernels of ncf_train_step (fwd/predict/bwd GEMMs)"

    # ---- quality: HR@10 / NDCG@10 on the leave-one-out test set ---------------
    hr10 = ndcg10 = None
    if not args.skip_eval and rank == 0:
        from ncf_amd.metrics import evaluate_arrays
        tu = np.repeat(ds["test_users"], 100)
        ti = np.concatenate([ds["test_items"][:, None], ds["test_negatives"]], 1).reshape(-1)
        HR, NDCG = evaluate_arrays(model, tu, ti, 100, 10)
        hr10, ndcg10 = float(np.mean(HR)), float(np.mean(NDCG))
    pipe.close()

    out = None
    if rank == 0:
        e2e = None
        if args.e2e_epochs > 0 and world == 1:
            e2e = e2e_fit(args.config, ds, dev, args.e2e_epochs)
        cpu = None
        if not args.skip_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.config, ds, per_gpu, args.cpu_seconds, threads=min(16, host_facts()["cpus_available"]))
        out = {
            "metric": "training interactions/sec + HR@10, NeuMF factors=64 ml-1m, 1/2/4/8 MI355X",
            "value": value,
            "unit": "interactions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": (f"synthetic {shape}-shaped ({U - 1:,} users x {I - 1:,} items, {len(ds['train_users']):,} "
                     f"train positives, 4 bit-exact sampled negatives each, fresh negatives and permutation "
                     f"every epoch: {epochs_in_timed} epoch boundaries in the timed region; seed 0)"),
            "config": {"workload": f"{args.config.upper()}: NCF(user_num={U}, item_num={I}, factor_num={f}, "
                                   f"num_layers={nl}, {mtype}), Adam lr 1e-3"
                                   + (f"; response distillation (T 2.0, alpha 0.5) from a random-init teacher "
                                      f"NCF({C5_TEACHER[0]}, {C5_TEACHER[1]}, {C5_TEACHER[2]}) whose logits of "
                                      f"each epoch stream are one forward launch at the epoch boundary"
                                      if args.config == "c5" else ""),
                       "global_batch": global_batch, "per_gpu_batch": per_gpu, "parallelism": f"dp{world}",
                       "mlp_layers": [int(2 * f * 2 ** (nl - 1)) >> k for k in range(nl + 1)],
                       "dp_exchange": eng.dp_mode, "hip_graph": use_graph},
            "roofline": {"bound": "mfma", "achieved": achieved_tf, "peak": 157.3, "unit": "TFLOP/s",
                         "frac": achieved_tf / 157.3, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": kname, "flops_per_launch": flops, "kernel_ms": ms,
                         "executed": {"flops_per_launch": xflops, "achieved": executed_tf,
                                      "frac": executed_tf / 157.3,
                                      "note": "flops the kernels execute; `achieved` counts the SURVEY 8(d) "
                                              "per-row tower flops (6 sum s_k s_k+1 + predict), of which the "
                                              "factored layer 0 replaces the layer-0 per-row GEMMs by "
                                              "per-entity ones over the U + I table rows"
                                              + ("; with it the algorithmic rate exceeds the fp32 MFMA peak"
                                                 if achieved_tf > 157.3 else "")}},
            "roofline_hbm": {"bound": "hbm", "achieved": achieved_gbs, "peak": 8000.0, "unit": "GB/s",
                             "frac": achieved_gbs / 8000.0, "bytes_per_launch": bytes_launch,
                             "note": ("gather+scatter algorithmic bytes of the same launch group" if path == L.PATH_FUSED
                                      else "gather+scatter algorithmic bytes over all layered-path kernels")},
            "kernel_ms": kt,
            "adam": adam_info(kt, eng, model),
            "quality": {"HR@10": hr10, "NDCG@10": ndcg10, "epochs_trained": round(eng.state_step() / eng.num_batches, 2),
                        "last_batch_loss": final_loss},
            "e2e": e2e,
            "frozen_epoch": frozen,
            "cpu_baseline": cpu,
            "setup_s": {"data+first_epoch": round(t_data, 2)},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.barrier(group=group, device_ids=[local])
        torch.distributed.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
