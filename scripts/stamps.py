#!/usr/bin/env python3
"""Phase attribution of the fused step kernel from s_memtime stamps
(diagnostics build: NCF_HIP_LIB=diag, `make -C ncf_amd/csrc diag`)."""
import json
import os
import sys

import numpy as np
import torch

os.environ["NCF_HIP_LIB"] = "diag"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = {0: "start", 1: "weights->LDS"}
for t in range(4):
    b = 2 + 14 * t
    NAMES.update({b: f"t{t}:idx+barrier", b + 1: f"t{t}:fwd", b + 2: f"t{t}:loss+gmf_bwd"})
    for j in range(3):
        NAMES.update({b + 3 + 3 * j: f"t{t}:L{2-j}:stage+bar", b + 4 + 3 * j: f"t{t}:L{2-j}:wgrad",
                      b + 5 + 3 * j: f"t{t}:L{2-j}:dgrad"})
    # layer 0 runs dgrad MFMA, then the scatter, then the wgrad
    NAMES.update({b + 10: f"t{t}:L0:dgrad_mfma", b + 11: f"t{t}:L0:scatter", b + 13: f"t{t}:L0:wgrad+end-barrier"})
    NAMES[b + 13] = f"t{t}:end-barrier"
NAMES.update({62: "epilogue:first barrier", 60: "epilogue:sums+stores", 61: "epilogue:drain",
              58: "ais:row indices requested", 59: "ais:tower image built", 63: "ais:kernel entry"})
for t in range(2):  # sub-phases of loss+gmf_bwd (slots of tiles 3-4, unused at bench size)
    NAMES.update({44 + 3 * t: f"t{t}:  bx-gather-issued", 45 + 3 * t: f"t{t}:  loss+dz"})


def main():
    import bench
    import ncf_amd._lib as L
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    eng, model, _ = bench.engine_for(cfg, dev, rows)
    eng.run(5, use_graph=False)
    wg = (int(eng.lay.flags) >> L.LAYOUT_WG_SHIFT) & L.LAYOUT_WG_MASK
    nwg = wg if wg else L.hip().ncf_slab_rows()
    buf = torch.zeros(nwg * 64, dtype=torch.int64, device=dev)
    since = {}
    spread = []
    for rep in range(3):
        buf.zero_()
        L.hip().ncf_debug_set_stamps(buf.data_ptr())
        eng.run(1, use_graph=False)
        torch.cuda.synchronize()
        L.hip().ncf_debug_set_stamps(None)
        st = buf.view(nwg, 64).cpu().numpy().astype(np.int64)
        rel = st - st[:, 0:1]
        dur = rel[:, 61][st[:, 61] > 0]
        if dur.size:  # per-workgroup duration: the kernel ends with the slowest one
            spread.append([float(np.percentile(dur, q)) for q in (0, 10, 50, 90, 100)])
        for idx, name in NAMES.items():
            ok = st[:, idx] > 0
            if ok.sum() > 0:
                since.setdefault(name, []).append(float(np.median(rel[ok, idx])))
    # phases in time order; delta = gap to the previous phase's median stamp
    order = sorted(since.items(), key=lambda kv: np.median(kv[1]))
    res, prev = {}, 0.0
    for name, v in order:
        t = float(np.median(v))
        res[name] = {"delta_cycles_median": t - prev, "since_start": t}
        prev = t
    sp = np.median(np.array(spread), axis=0).tolist() if spread else []
    print(json.dumps({"config": cfg, "rows": rows, "workgroups": int(nwg), "phases": res,
                      "wg_duration_cycles_p0_p10_p50_p90_max": sp}))


if __name__ == "__main__":
    main()
