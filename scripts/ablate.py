#!/usr/bin/env python3
"""Ablation of the fused step kernel (diagnosis only): time ncf_train_step with
HIP events under the DIAG switches, interleaved rounds in one process.
Prints one JSON line with median ms per variant and per rows-per-launch."""
import json
import os
import sys

import numpy as np
import torch

os.environ.setdefault("NCF_HIP_LIB", "diag")  # the scatter switches exist in the diag build only

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import ncf_amd._lib as L
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    res = {}
    for rows in ([int(x) for x in sys.argv[2].split(',')] if len(sys.argv) > 2 else (65536, 16384)):
        eng, model, _ = bench.engine_for(cfg, dev, rows)
        eng.run(3, use_graph=False)
        torch.cuda.synchronize()
        variants = {"full": 0, "no_wgrad": 2, "no_user_scatter": 8, "no_item_scatter": 16,
                    "no_gmf_scatter": 32, "no_scatter": 8 | 16 | 32}
        times = {k: [] for k in variants}
        for _ in range(5):
            for name, d in variants.items():
                L.hip().ncf_debug_set_diag(d)
                times[name].append(eng.time_train_kernel(20))
        L.hip().ncf_debug_set_diag(0)
        res[str(rows)] = {k: float(np.median(v)) for k, v in times.items()}
        res[str(rows) + "_other"] = eng.time_kernels(10)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
