#!/usr/bin/env python3
"""Diagnosis: time the pieces of ncf_prepare_epoch at bench size (HIP events,
many repetitions): plain gather (rows[perm]), full prepare (LDS-histogram and
global-histogram variants).  Prints one JSON line of ms per call."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    import numpy as np
    import ncf_amd._lib as L
    from ncf_amd import ops, synthetic
    dev = torch.device("cuda", 0)
    ds = synthetic.make_dataset("ml-1m", seed=0)
    U, I = ds["user_num"], ds["item_num"]
    rng = np.random.default_rng(0)
    pu, pi = ds["train_users"], ds["train_items"]
    users = np.concatenate([pu, np.repeat(pu, 4)])
    items = np.concatenate([pi, rng.integers(0, I, 4 * len(pi))])
    labels = np.concatenate([np.ones(len(pu)), np.zeros(4 * len(pu))])
    rows = torch.from_numpy(ops.pack_rows_host(users, items, labels)).to(dev)
    n = rows.numel()
    perm = torch.randperm(n, device=dev)
    out = torch.empty_like(rows)
    prep = ops.EpochPrep(dev)
    res = {"n": n}
    res["gather"] = timed(lambda: L.check(L.hip().ncf_gather_epoch(rows.data_ptr(), perm.data_ptr(), n,
                                                                   out.data_ptr(), L.stream_ptr(dev)), "g"))
    for bs in (65536, 256):
        res[f"prepare_lds_B{bs}"] = timed(lambda: prep(rows, perm, bs, I))
        L.hip().ncf_debug_set_diag(4)
        res[f"prepare_direct_B{bs}"] = timed(lambda: prep(rows, perm, bs, I))
        L.hip().ncf_debug_set_diag(0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
