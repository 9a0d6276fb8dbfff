#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats + FETCH_SIZE / WRITE_SIZE passes)
into markdown (stdout) and <dir>/prof_summary.json.

HBM traffic per dispatch follows /opt/skills/guides/MI355X_MICROARCH.md (HBM):
FETCH_SIZE / WRITE_SIZE are KB; on gfx950 FETCH_SIZE counts half the bytes of
wide coalesced reads, so the corrected read bytes are 2 x FETCH_SIZE x 1024
(an upper estimate for narrower access widths); WRITE_SIZE is exact for
16-B/lane stores and f32 atomics.  Both raw and corrected values are reported."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    # kernels in an anonymous namespace print as "ncf::(anonymous namespace)::k<...>(args)":
    # drop that qualifier before cutting the argument list
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").strip()


def load_stats(d):
    f = glob.glob(os.path.join(d, "prof", "**", "*kernel_stats.csv"), recursive=True)
    if not f:
        return []
    rows = list(csv.DictReader(open(f[0])))
    return rows


def load_pmc(d, sub, counter):
    fs = glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(list)
    for f in fs:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    config = sys.argv[2] if len(sys.argv) > 2 else "c3"  # the bench config profiled (bench.py pmc_traffic keys on it)
    stats = load_stats(d)
    fetch = load_pmc(d, "pmc_fetch", "FETCH_SIZE")
    write = load_pmc(d, "pmc_write", "WRITE_SIZE")
    out = {"config": config, "kernels": []}
    print("| kernel | calls | avg us | % time | FETCH_SIZE KB | WRITE_SIZE KB | HBM bytes (2xF+W) | GB/s |")
    print("|---|---|---|---|---|---|---|---|")
    for r in stats:
        k = short(r["Name"])
        avg_us = float(r["AverageNs"]) / 1e3
        f = fetch.get(k)
        w = write.get(k)
        hbm = (2 * f + w) * 1024 if f is not None and w is not None else None
        gbs = hbm / (avg_us * 1e-6) / 1e9 if hbm else None
        out["kernels"].append({"kernel": k, "calls": int(r["Calls"]), "avg_us": avg_us,
                               "pct": float(r["Percentage"]), "fetch_kb": f, "write_kb": w,
                               "hbm_bytes_corrected": hbm, "hbm_GBps": gbs})
        print(f"| {k} | {r['Calls']} | {avg_us:.2f} | {float(r['Percentage']):.1f} | "
              f"{'' if f is None else f'{f:.0f}'} | {'' if w is None else f'{w:.0f}'} | "
              f"{'' if hbm is None else f'{hbm / 1e6:.2f} MB'} | {'' if gbs is None else f'{gbs:.0f}'} |")
    # SQ pass (MFMA utilisation): SQ_VALU_MFMA_BUSY_CYCLES summed over the 1,024
    # SIMDs (256 CUs x 4); GRBM_GUI_ACTIVE summed over the 8 XCDs (per XCD it is the
    # dispatch's busy cycles: /8 over the trace's duration gives ~2.5 GHz)
    sq = {c: load_pmc(d, "pmc_sq", c) for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES",
                                                 "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAVES")}
    if any(sq.values()):
        print()
        print("| kernel | MFMA busy cycles / SIMD | GRBM_GUI_ACTIVE / XCD | MFMA busy fraction | SQ_WAVE_CYCLES | SQ_WAIT_ANY | SQ_ACTIVE_INST_ANY |")
        print("|---|---|---|---|---|---|---|")
        for k in out["kernels"]:
            n = k["kernel"]
            mb = sq["SQ_VALU_MFMA_BUSY_CYCLES"].get(n)
            ga = sq["GRBM_GUI_ACTIVE"].get(n)
            if mb is None:
                continue
            per_simd = mb / 1024
            ga = ga / 8 if ga else ga
            k["sq"] = {c: sq[c].get(n) for c in sq}
            k["mfma_busy_per_simd"] = per_simd
            k["mfma_busy_frac"] = per_simd / ga if ga else None
            print(f"| {n} | {per_simd:.0f} | {'' if ga is None else f'{ga:.0f}'} | "
                  f"{'' if not ga else f'{per_simd / ga:.3f}'} | {sq['SQ_WAVE_CYCLES'].get(n, 0):.0f} | "
                  f"{sq['SQ_WAIT_ANY'].get(n, 0):.0f} | {sq['SQ_ACTIVE_INST_ANY'].get(n, 0):.0f} |")
    json.dump(out, open(os.path.join(d, "prof_summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
