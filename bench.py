#!/usr/bin/env python3
"""Headline benchmark: NeuMF training interactions/sec on MI355X.

Workload (BASELINE.json metric "training interactions/sec + HR@10, NeuMF
factors=64 ml-1m"): NCF(6041, 3707, factor_num=16,
num_layers=3, 'NeuMF-end') -- 64-wide MLP embeddings, tower [128,64,32,16] --
on ml-1m-shaped synthetic data (994,169 positives, 4 sampled negatives each,
bit-exact reference sampler), 65,536 rows per GPU per step, Adam lr 1e-3.

A "step" = fused fwd+loss+bwd kernel, tower-grad reduction, (RCCL all-reduce
of the gradient bucket when N > 1), dense Adam -- the whole optimizer step of
scripts/train_neumf.py:111-115, captured once into a hipGraph and replayed.
The epoch stream (users/items/labels, already shuffled) is resident in HBM
before the timed region.  Per-GPU work is fixed (65,536 rows/GPU/step), so
scaling is weak and value = all ranks' rows / max-over-ranks time.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, RCCL).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
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
}


def tower_flops_per_row(f, L, model="NeuMF-end"):
    dm = f * 2 ** (L - 1)
    s = [(2 * dm) >> k for k in range(L + 1)]
    fl = 6 * sum(s[k] * s[k + 1] for k in range(L))
    p = 2 * f if model.startswith("NeuMF") else f
    return fl + 6 * p


def gather_scatter_bytes_per_row(f, L):
    """Algorithmic HBM bytes per row of the fused kernel: the 8-byte packed row
    (user, item, label), the four embedding rows read, and the same four rows'
    gradient added (f32 atomics: read-modify-write at the memory side)."""
    dm = f * 2 ** (L - 1)
    rows = 2 * (f + dm) * 4
    return 8 + rows + rows


def adam_info(kt, P, adam_bytes, eng):
    """Optimizer launch and its bytes: dense Adam is 32 B/param (read p, g, m, v;
    write p, m, v, g = 0); the fused reduce+Adam also reads the partial slab."""
    if "ncf_reduce_adam_step" in kt:
        slab_bytes = int(eng.ws.numel()) * 4
        ms = kt["ncf_reduce_adam_step"]
        return {"kernel": "ncf_reduce_adam_step (slab reduce + Adam)", "params": P,
                "bytes": adam_bytes + slab_bytes, "ms": ms, "GB/s": (adam_bytes + slab_bytes) / (ms * 1e-3) / 1e9}
    ms = kt["optimizer"]
    return {"kernel": "ncf_adam_step", "params": P, "bytes": adam_bytes, "ms": ms,
            "GB/s": adam_bytes / (ms * 1e-3) / 1e9}


def pmc_traffic(f, L):
    """HBM bytes per launch of the fused step kernel from the newest committed
    rocprofv3 PMC summary (profiles/r*_prof_summary.json, written by
    scripts/profile.sh + scripts/prof_summary.py from separate FETCH_SIZE and
    WRITE_SIZE passes of this bench: bytes = (2 * FETCH_SIZE + WRITE_SIZE) KB * 1024,
    the gfx950 correction of the MI355X guide).  (None, None) if absent."""
    import glob
    dm = f * 2 ** (L - 1)
    names = (f"ncf::ncf_step_kernel<{f}, {L}, 2, false, true>", f"ncf::fact_expand_kernel<{dm}>")
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_prof_summary.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        got = {k.get("kernel"): k.get("hbm_bytes_corrected") for k in d.get("kernels", [])}
        if all(got.get(n) for n in names):
            return float(sum(got[n] for n in names)), os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(f, L, U, I, batch, seconds, threads):
    """The oracle (oracle/ncf_oracle.py: the reference model restated on stock
    PyTorch CPU ops + torch.optim.Adam) timed on a bounded sample of the same
    workload: full 65,536-row steps on random ids of the same id space."""
    from oracle import ncf_oracle as O
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    m = O.OracleNCF(U, I, f, L, 0.0, "NeuMF-end")
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    rng = np.random.default_rng(0)
    mk = lambda: (torch.from_numpy(rng.integers(0, U, batch)), torch.from_numpy(rng.integers(0, I, batch)),
                  torch.from_numpy((rng.random(batch) < 0.2).astype(np.int64)))
    u, i, y = mk()
    O.train_steps(m, opt, [u], [i], [y])  # warm-up
    steps, t0 = 0, time.perf_counter()
    while True:
        O.train_steps(m, opt, [u], [i], [y])
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": steps * batch / el, "unit": "interactions/s", "cores": threads, "kind": "port",
            "sample": f"{steps} x {batch}-row Adam steps of the oracle (reference NCF restated on torch CPU "
                      f"ops), NCF({U},{I},{f},{L}), {el:.1f} s on {threads} threads "
                      f"({platform.processor() or platform.machine()})"}


def setup_engine(config, world, rank, dev, group, global_batch, seed=0):
    """Synthetic dataset -> bit-exact negatives -> shuffled epoch stream in HBM
    -> NCF + TrainEngine.  Identical on every rank (seeded)."""
    from ncf_amd import synthetic
    from ncf_amd.data import HostSampler, epoch_permutation
    from ncf_amd.engine import TrainEngine
    from ncf_amd.models import NCF
    from ncf_amd import ops
    shape, f, nl, _ = CONFIGS[config]
    ds = synthetic.make_dataset(shape, seed=seed)
    U, I = ds["user_num"], ds["item_num"]
    np.random.seed(seed)
    torch.manual_seed(seed)
    sampler = HostSampler(ds["train_users"], ds["train_items"], U, I)
    t_s = time.perf_counter()
    neg = sampler.sample(I, 4)
    t_sample = time.perf_counter() - t_s
    pu, pi = ds["train_users"], ds["train_items"]
    users = np.concatenate([pu, np.repeat(pu, 4)]).astype(np.int32)
    items = np.concatenate([pi, neg]).astype(np.int32)
    labels = np.concatenate([np.ones(len(pu), np.float32), np.zeros(len(neg), np.float32)])
    model = NCF(U, I, f, nl, 0.0, "NeuMF-end").to(dev)
    perm = epoch_permutation(len(users)).to(dev)
    rows_d = torch.from_numpy(ops.pack_rows_host(users, items, labels)).to(dev)  # resident in HBM
    prep = ops.EpochPrep(dev)
    stream = prep(rows_d, perm, global_batch, I)
    eng = TrainEngine(model, lr=1e-3, world_size=world, rank=rank, process_group=group)
    eng.set_epoch_stream(stream, global_batch)

    def prepare():  # per-epoch device work: shuffle + group each batch by item (same output buffer)
        prep(rows_d, perm, global_batch, I)
    eng.prepare_epoch = prepare
    return eng, model, ds, t_sample


def run_steps(eng, n_steps, use_graph):
    """n_steps optimizer steps; the per-epoch device preparation (ncf_prepare_epoch)
    runs at every epoch boundary inside the timed region."""
    done = 0
    while done < n_steps:
        pos = eng.batches_done % eng.num_batches
        if pos == 0 and eng.batches_done > 0:
            eng.prepare_epoch()
        k = min(n_steps - done, eng.num_batches - pos)
        eng.run(k, use_graph=use_graph)
        eng.batches_done += k
        done += k


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
    eng, model, ds, t_sample = setup_engine(args.config, world, rank, dev, group, global_batch)
    U, I = ds["user_num"], ds["item_num"]
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
    t0 = time.perf_counter()
    run_steps(eng, args.steps, use_graph)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    if world > 1:
        torch.distributed.barrier(group=group, device_ids=[local])
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=group)
        dt = float(t.item())
    rows = args.steps * global_batch
    value = rows / dt
    losses = eng.epoch_losses()
    final_loss = float(losses[(eng.state_step() - 1) % eng.num_batches])

    # ---- per-kernel live timing (HIP events on the launch stream) -------------
    kt = eng.time_kernels(args.kernel_steps)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        eng.prepare_epoch()
    e1.record()
    torch.cuda.synchronize(dev)
    kt["prepare_epoch_per_epoch"] = e0.elapsed_time(e1) / 5
    kt["ncf_train_step_per_launch_b2b"] = eng.time_train_kernel(50)
    rows_per_launch = per_gpu
    flops = tower_flops_per_row(f, nl) * rows_per_launch
    ms = kt["ncf_train_step_per_launch_b2b"]
    achieved_tf = flops / (ms * 1e-3) / 1e12
    bytes_launch = gather_scatter_bytes_per_row(f, nl) * rows_per_launch
    achieved_gbs = bytes_launch / (ms * 1e-3) / 1e9
    P = sum(p.numel() for p in model.parameters())
    adam_bytes = 32 * P  # read p,g,m,v; write p,m,v,g(=0)
    traffic, traffic_src = pmc_traffic(f, nl)
    import ncf_amd._lib as L
    path = L.supported("NeuMF-end", f, nl)

    # ---- quality: HR@10 / NDCG@10 on the leave-one-out test set ---------------
    hr10 = ndcg10 = None
    if not args.skip_eval and rank == 0:
        from ncf_amd.metrics import evaluate_arrays
        tu = np.repeat(ds["test_users"], 100)
        ti = np.concatenate([ds["test_items"][:, None], ds["test_negatives"]], 1).reshape(-1)
        HR, NDCG = evaluate_arrays(model, tu, ti, 100, 10)
        hr10, ndcg10 = float(np.mean(HR)), float(np.mean(NDCG))

    out = None
    if rank == 0:
        cpu = None
        if not args.skip_cpu_baseline and world == 1:
            cpu = cpu_baseline(f, nl, U, I, per_gpu, args.cpu_seconds, threads=min(16, os.cpu_count() or 1))
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
            "data": "synthetic ml-1m-shaped (6,040 users x 3,706 items, 994,169 train positives, "
                    "4 bit-exact sampled negatives each; seed 0)",
            "config": {"workload": f"{args.config.upper()}: NCF(user_num={U}, item_num={I}, factor_num={f}, "
                                   f"num_layers={nl}, NeuMF-end), Adam lr 1e-3",
                       "global_batch": global_batch, "per_gpu_batch": per_gpu, "parallelism": f"dp{world}",
                       "mlp_layers": [int(2 * f * 2 ** (nl - 1)) >> k for k in range(nl + 1)],
                       "dp_exchange": eng.dp_mode, "hip_graph": use_graph},
            "roofline": {"bound": "mfma", "achieved": achieved_tf, "peak": 157.3, "unit": "TFLOP/s",
                         "frac": achieved_tf / 157.3, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": (f"ncf_step_kernel<{f},{nl},NeuMF,FACT> + fact_expand_kernel<{f * 2 ** (nl - 1)}> "
                                    "(fused fwd+bwd, factored layer 0; launch group timed back to back)"
                                    if path == 1 else
                                    "layered path: all kernels of ncf_train_step (fwd/predict/bwd GEMMs)"),
                         "flops_per_launch": flops, "kernel_ms": ms},
            "roofline_hbm": {"bound": "hbm", "achieved": achieved_gbs, "peak": 8000.0, "unit": "GB/s",
                             "frac": achieved_gbs / 8000.0, "bytes_per_launch": bytes_launch,
                             "note": "gather+scatter algorithmic bytes of the same fused kernel"},
            "kernel_ms": kt,
            "adam": adam_info(kt, P, adam_bytes, eng),
            "quality": {"HR@10": hr10, "NDCG@10": ndcg10, "epochs_trained": round(eng.state_step() / eng.num_batches, 2),
                        "last_batch_loss": final_loss},
            "cpu_baseline": cpu,
            "setup_s": {"data+upload": round(t_data, 2), "ng_sample_cpp": round(t_sample, 3)},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.barrier(group=group, device_ids=[local])
        torch.distributed.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
