#!/usr/bin/env bash
# SQ counters of the bench workload (diagnosis): where the step kernel's wave
# cycles go (parked in s_waitcnt/barrier, issue-stalled, active) and MFMA busy.
# Separate --pmc passes (at most 8 SQ counters each), kernel trace off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--config ${CONFIG:-c3} --steps 30 --warmup 5 --skip-cpu-baseline --skip-eval --kernel-steps 3 --e2e-epochs 0"
export FILTER="${FILTER:-ncf_step_kernel reduce_adam}"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d gpurun_out/sq$i -o run -- python3 bench.py $ARGS \
        > gpurun_out/sq$i.log 2>&1 || { echo "pass $i failed"; tail -20 gpurun_out/sq$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    import os
    if not any(f in k for f in os.environ["FILTER"].split()):
        continue
    print(k.replace("(anonymous namespace)::", "")[:70])
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
PY
