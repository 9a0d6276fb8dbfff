#!/usr/bin/env python3
"""Host sampler timing: one ng_sample pass (datasets.py:53-69) and the epoch's
randperm words, sequential vs parallel, at the ml-1m / ml-20m shapes the bench
configs use (ncf_amd.synthetic; ml-20m via a fast same-shape generator unless
--real).  Checks the parallel outputs against the sequential ones as it goes.

    python scripts/sampler_bench.py [--shape ml-1m|ml-20m] [--threads 16] [--passes 6]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def fast_ml20m(seed=0):
    rng = np.random.default_rng(seed)
    U, I = 138_494, 26_745
    w = rng.lognormal(0.0, 1.0, U - 1)
    counts = np.minimum(20 + np.floor(w / w.sum() * (19_861_770 - 20 * (U - 1))).astype(np.int64), I // 2)
    p = np.arange(1, I, dtype=np.float64) ** -0.8
    p /= p.sum()
    pu = np.repeat(np.arange(1, U, dtype=np.int32), counts)
    pi = (rng.choice(I - 1, size=len(pu), p=p) + 1).astype(np.int32)
    return pu, pi, U, I


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="ml-1m")
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--passes", type=int, default=6)
    ap.add_argument("--real", action="store_true", help="ncf_amd.synthetic's generator for ml-20m (slow)")
    a = ap.parse_args()
    from ncf_amd.data import HostSampler, sampler_threads
    from ncf_amd.pipeline import WordsGen, torch_words
    if a.shape == "ml-20m" and not a.real:
        pu, pi, U, I = fast_ml20m()
    else:
        from ncf_amd import synthetic
        ds = synthetic.make_dataset(a.shape, seed=0)
        pu, pi, U, I = ds["train_users"], ds["train_items"], ds["user_num"], ds["item_num"]
    T = a.threads or sampler_threads()
    res = {"shape": a.shape, "positives": int(len(pu)), "threads": T}
    out_s = np.empty(4 * len(pu), np.int32)
    out_p = np.empty(4 * len(pu), np.int32)
    for name, thr, out in (("sequential", 1, out_s), ("parallel", T, out_p)):
        s = HostSampler(pu, pi, U, I, threads=thr)
        np.random.seed(0)
        ts = []
        for _ in range(a.passes):
            t0 = time.perf_counter()
            s.sample(I, 4, out=out)
            ts.append((time.perf_counter() - t0) * 1e3)
        res[name + "_ms"] = [round(x, 2) for x in ts]
        res[name + "_state"] = int(np.random.get_state()[2])
        if thr > 1:
            res["parallel_stats"] = s.stats()
    res["equal"] = bool(np.array_equal(out_s, out_p)) and res["sequential_state"] == res["parallel_state"]
    n = 5 * len(pu) - 1
    w1, w2 = np.empty(n, np.uint32), np.empty(n, np.uint32)
    gen = WordsGen(T)
    for name, g, w in (("words_sequential_ms", None, w1), ("words_parallel_ms", gen, w2)):
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            torch_words(12345, n, w, g)
            ts.append((time.perf_counter() - t0) * 1e3)
        res[name] = [round(x, 2) for x in ts]
    res["words_equal"] = bool(np.array_equal(w1, w2))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
