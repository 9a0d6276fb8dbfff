#!/usr/bin/env bash
# One GPU-box session: smoke -> full GPU test suite -> bench (c3) -> rocprof passes.
# Each GPU step has its own time limit; a crash / fault / timeout ends the script
# (test failures, exit 1, do not).  Output in gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, seconds, cmd...
    local name=$1 secs=$2
    shift 2
    echo "== $name: $*" | tee -a gpurun_out/steps.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
    tail -3 "gpurun_out/$name.log"
    if grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault|GPU Hang" "gpurun_out/$name.log"; then
        echo "stopping after $name: GPU fault signature in log"; exit 90
    fi
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
[ "${SMOKE:-1}" = "1" ] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${TESTS:-1}" = "1" ] && run pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider
[ "${BENCH:-1}" = "1" ] && run bench 600 python bench.py --steps "${STEPS:-200}" --warmup "${WARMUP:-20}"
if [ "${PROFILE:-0}" = "1" ]; then
    run profile 900 bash scripts/profile.sh
fi
echo ALL-DONE
