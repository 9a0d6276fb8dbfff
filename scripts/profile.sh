#!/usr/bin/env bash
# rocprofv3 evidence for one bench config (run on the GPU box; CONFIG=c3 default):
#   1. --kernel-trace --stats            per-kernel durations
#   2. --pmc FETCH_SIZE  (own pass)      HBM read bytes  (KB, x2 on gfx950 for wide reads)
#   3. --pmc WRITE_SIZE  (own pass)      HBM write bytes (KB)
#   4. --pmc SQ counters (own pass)      MFMA busy / wave cycles of every kernel
# then scripts/prof_summary.py writes gpurun_out/prof_summary.{md,json} (tagged with the config).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CONFIG="${CONFIG:-c3}"
ARGS="--config $CONFIG --steps ${STEPS:-60} --warmup 5 --skip-cpu-baseline --skip-eval --kernel-steps 5 --e2e-epochs 0 --profile-run"
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
step pmc_sq rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq -o run -- python3 bench.py $ARGS
python3 scripts/prof_summary.py gpurun_out "$CONFIG" > gpurun_out/prof_summary.md
cat gpurun_out/prof_summary.md
