#!/usr/bin/env python3
"""Projected 1/2/4/8-GPU step times from measured per-rank local costs.

The one-GPU pool cannot run the N-rank RCCL transport, so the curve is projected:

    T(N) = local(N) + exchange(N)

* local(N): the graph-replayed per-rank step measured on one MI355X with the engine
  as rank 0 of an emulated world N (scripts/dp_modes.py: its shard of every global
  batch, the real launches, a one-rank group whose collectives move nothing), taken
  from the dp_modes JSON files given on the command line;
* exchange(N): the collectives of the mode on the wire, modelled as ring collectives
  over xGMI -- per collective  alpha + (N - 1) / N * S / B  for a reduce-scatter or an
  all-gather of S bytes, twice that volume for an all-reduce -- with B the per-link
  xGMI bandwidth (7 links x ~153 GB/s per MI355X: a ring is per-link bound; the
  task's stated figure, not measured here) and alpha a per-collective latency
  (RCCL launch + ring steps; an assumption, varied over --alpha).
* dp_mode "owner": two all-to-alls of fixed chunks per peer (the gradient rows with the
  tower tail, then the next batch's rows); on the 8-GPU node every pair of GPUs has its
  own xGMI link, so each all-to-all is  alpha + chunk / B_link  (the W - 1 chunks go out
  on W - 1 links at once); B_link over --link-bw (the task's 153 GB/s per link, and a
  pessimistic figure for RCCL's all-to-all).  The chunk sizes are the ones the engine
  allocated at that world (dp_modes JSON "owner").

Usage: scaling_model.py OUT.json dp_modes_c3_n2.json dp_modes_c3_n4.json ...
(N = 1 is the single-process bench value, --n1-us per config)."""
import argparse
import json


def exchange_us(mode, n, floats, packed_floats, b_gbs, alpha_us, owner=None):
    if n == 1:
        return 0.0
    if mode == "owner":  # two all-to-alls, every peer on its own link
        return 2 * alpha_us + (owner["grad_chunk_bytes"] + owner["param_chunk_bytes"]) / (b_gbs * 1e3)
    s = 4.0 * floats
    ring = (n - 1) / n
    if mode == "allreduce":
        return alpha_us + 2 * ring * s / (b_gbs * 1e3)
    if mode == "touched":
        return alpha_us + 2 * ring * 4.0 * packed_floats / (b_gbs * 1e3)
    if mode == "zero1":  # reduce-scatter + all-gather: one all-reduce's bytes, two collectives
        return 2 * alpha_us + 2 * ring * s / (b_gbs * 1e3)
    raise ValueError(mode)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("inputs", nargs="+")
    ap.add_argument("--bw", type=float, nargs="+", default=[153.0, 450.0],
                    help="ring bus GB/s: one xGMI link (a single ring, per-link bound) and an "
                         "optimistic multi-ring figure over several of the 7 links")
    ap.add_argument("--alpha", type=float, nargs="+", default=[10.0, 25.0], help="us per collective")
    ap.add_argument("--link-bw", type=float, nargs="+", default=[153.0, 64.0],
                    help="all-to-all GB/s per peer link (owner mode): the stated xGMI link figure and a "
                         "pessimistic one")
    ap.add_argument("--n1-us", type=json.loads, default={"c3": 55.9, "c4": 126.0},
                    help="single-process us/step per config (bench lines)")
    ap.add_argument("--floats", type=json.loads, default={"c3": 790737, "c4": 13230017})
    ap.add_argument("--packed", type=json.loads, default={"c3": 790737, "c4": 7400000},
                    help="touched-mode packed floats per step (DESIGN §6 table)")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--local", choices=("events", "graph"), default="events",
                    help="local part: the event-timed launch groups without the collectives (events), or the "
                         "graph-replayed step minus the one-rank collectives' kernel time (graph; per-part event "
                         "pairs add several us each)")
    ap.add_argument("--coll-us", type=json.loads, default={},
                    help='graph mode: {"config/mode": us} of one one-rank collective kernel (rocprofv3 trace of '
                         'the dp_modes run)')
    a = ap.parse_args()
    rows = []
    for path in a.inputs:
        txt = open(path).read().strip().splitlines()
        d = json.loads([line for line in txt if line.startswith("{")][-1])
        cfg, n = d["config"], int(d["world_emulated"])
        for mode, m in d["modes"].items():
            # local part: the per-rank launch groups (HIP events on the launch stream)
            # without the emulated collectives (a one-rank group, or their exact
            # all-reduce forms over it, move nothing between GPUs)
            local = sum(1e3 * v for k, v in m["launch_groups_ms"].items()
                        if k not in ("allreduce", "reduce_scatter", "all_gather", "all_to_all_grads",
                                     "all_to_all_params"))
            if a.local == "graph":
                ncoll = {"allreduce": 1, "touched": 1, "zero1": 2, "owner": 2}[mode]
                local = 1e3 * m["ms_per_step_graph"] - ncoll * float(a.coll_us.get(f"{cfg}/{mode}", 0.0))
            for bw in (a.link_bw if mode == "owner" else a.bw):
                for alpha in a.alpha:
                    x = exchange_us(mode, n, a.floats[cfg], a.packed[cfg], bw, alpha, m.get("owner"))
                    t = local + x
                    rows.append({"config": cfg, "n_gpus": n, "mode": mode, "bw_GBps": bw, "alpha_us": alpha,
                                 "local_us": round(local, 1), "exchange_us": round(x, 1), "step_us": round(t, 1),
                                 "interactions_per_s": a.batch / (t * 1e-6), "vs_1gpu": a.n1_us[cfg] / t})
    for cfg, us in a.n1_us.items():
        rows.append({"config": cfg, "n_gpus": 1, "mode": "single", "bw_GBps": 0, "alpha_us": 0, "local_us": us,
                     "exchange_us": 0, "step_us": us, "interactions_per_s": a.batch / (us * 1e-6), "vs_1gpu": 1.0})
    json.dump({"model": "T(N) = local(N) + ring collectives over xGMI (owner: two all-to-alls over the "
                        "point-to-point links)", "rows": rows}, open(a.out, "w"), indent=1)
    for r in sorted(rows, key=lambda r: (r["config"], r["n_gpus"], r["mode"], r["bw_GBps"], r["alpha_us"])):
        print(f"{r['config']} N={r['n_gpus']} {r['mode']:9s} B={r['bw_GBps']:4.0f} a={r['alpha_us']:3.0f}  "
              f"local {r['local_us']:6.1f}  xchg {r['exchange_us']:6.1f}  step {r['step_us']:6.1f} us  "
              f"{r['interactions_per_s'] / 1e9:6.3f} G/s  x{r['vs_1gpu']:.2f}")


if __name__ == "__main__":
    main()
