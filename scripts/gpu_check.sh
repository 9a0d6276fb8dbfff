#!/usr/bin/env bash
# One GPU-box session: smoke -> GPU parity tests -> bench -> rocprof kernel trace.
# Every GPU step has its own time limit; a crash/fault/timeout ends the script
# (test *failures*, exit 1, do not).  Output goes to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-200}"
WARMUP="${WARMUP:-20}"

run() {  # name, seconds, cmd...
    local name=$1 secs=$2
    shift 2
    echo "== $name: $*" | tee -a gpurun_out/steps.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
    tail -5 "gpurun_out/$name.log"
    # a GPU fault can surface as a Python exception (exit 1): stop on its signature too
    if grep -qE "illegal memory access|hipErrorIllegalAddress|HIP error|Memory access fault|GPU Hang" "gpurun_out/$name.log"; then
        echo "stopping after $name: GPU fault signature in log"
        exit 90
    fi
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
    return 0
}

rocm-smi --showproductname > gpurun_out/rocm_smi.log 2>&1 || true
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider
run bench 600 python bench.py --steps "$STEPS" --warmup "$WARMUP"
if [ "${ABLATE:-0}" = "1" ]; then
    run ablate 600 python scripts/ablate.py
fi
if [ "${PROFILE:-1}" = "1" ]; then
    run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
        python3 bench.py --steps 100 --warmup 10 --skip-cpu-baseline --skip-eval
fi
echo ALL-DONE
