#!/usr/bin/env python3
"""A/B timing of ncf_train_step across library variants (diagnosis).

  python scripts/ab_kernel.py [--config c3] default wfree ...
Each variant ("default" = libncf_hip.so, else libncf_hip_<name>.so via
NCF_HIP_LIB) runs in its own process (the library is loaded once per process);
rounds interleave the variants.  Prints one JSON line: median ms per launch
over back-to-back launches (HIP events on the launch stream)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(cfg):
    sys.path.insert(0, ROOT)
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    per = bench.CONFIGS[cfg][3]
    eng, _, _ = bench.engine_for(cfg, dev, per)
    eng.run(3, use_graph=False)
    ts = sorted(eng.time_train_kernel(40) for _ in range(5))
    print("RESULT", ts[len(ts) // 2])


def main():
    args = sys.argv[1:]
    if args and args[0] == "--child":
        return child(args[1])
    cfg = "c3"
    if args and args[0] == "--config":
        cfg, args = args[1], args[2:]
    variants = args or ["default"]
    res = {v: [] for v in variants}
    for _ in range(3):
        for v in variants:
            env = dict(os.environ)
            env.pop("NCF_HIP_LIB", None)
            if v != "default":
                env["NCF_HIP_LIB"] = v
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", cfg], env=env,
                                 capture_output=True, text=True, timeout=600)
            if out.returncode != 0:
                print(out.stdout[-2000:], out.stderr[-3000:])
                sys.exit(out.returncode)
            ms = [float(l.split()[1]) for l in out.stdout.splitlines() if l.startswith("RESULT")][0]
            res[v].append(ms)
    print(json.dumps({v: {"median_ms": sorted(x)[1], "all": x} for v, x in res.items()}))


if __name__ == "__main__":
    main()
