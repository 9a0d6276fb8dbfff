#!/usr/bin/env bash
# rocprofv3 evidence for the bench workload (run on the GPU box):
#   1. --kernel-trace --stats            per-kernel durations
#   2. --pmc FETCH_SIZE  (own pass)      HBM read bytes  (KB, x2 on gfx950 for wide reads)
#   3. --pmc WRITE_SIZE  (own pass)      HBM write bytes (KB)
# then scripts/prof_summary.py writes gpurun_out/prof_summary.{md,json}.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps ${STEPS:-60} --warmup 5 --skip-cpu-baseline --skip-eval --kernel-steps 5"
step() {
    local name=$1; shift
    echo "== $name"
    timeout -k 10 300 "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
step trace rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py $ARGS
step pmc_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py $ARGS
step pmc_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py $ARGS
python3 scripts/prof_summary.py gpurun_out > gpurun_out/prof_summary.md
cat gpurun_out/prof_summary.md
