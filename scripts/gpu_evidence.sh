#!/usr/bin/env bash
# One evidence session on the GPU box: smoke, the whole GPU test suite, the default
# bench line (C3 with the CPU baseline and the Trainer.fit e2e figure), a line per
# other config, then the C3 rocprofv3 kernel trace + FETCH/WRITE/SQ passes
# (scripts/profile.sh).  Each GPU step has its own time limit; a crash, fault or
# timeout ends the script.  Output in gpurun_out/.
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
    tail -2 "gpurun_out/$name.log"
    if grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault|GPU Hang" "gpurun_out/$name.log"; then
        echo "stopping after $name: GPU fault signature in log"; exit 90
    fi
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 900 python -u -m pytest tests -m gpu -v -s -x --timeout 300 --timeout-method thread -p no:cacheprovider
run bench 600 python bench.py
for cfg in ${CONFIGS:-c2 c4 cli stress c5}; do
    run "bench_$cfg" 300 python bench.py --config "$cfg" --steps 200 --warmup 20 --skip-cpu-baseline --e2e-epochs ${E2E:-2}
    tail -1 "gpurun_out/bench_$cfg.log" >> gpurun_out/configs.jsonl
done
if [ "${SAMPLER:-1}" = "1" ]; then
    for shape in ml-1m ml-20m; do
        run "sampler_$shape" 300 python scripts/sampler_bench.py --shape $shape --passes 6
        tail -1 "gpurun_out/sampler_$shape.log" >> gpurun_out/sampler.jsonl
    done
fi
if [ "${PROFILE:-1}" = "1" ]; then
    for cfg in ${PROFILE_CONFIGS:-c3}; do  # scripts/profile.sh writes fixed names: keep a copy per config
        export CONFIG=$cfg
        run "profile_$cfg" 900 bash scripts/profile.sh
        mkdir -p "gpurun_out/prof_$cfg"
        cp gpurun_out/prof_summary.md gpurun_out/prof_summary.json gpurun_out/prof/run_kernel_stats.csv "gpurun_out/prof_$cfg/"
    done
fi
echo ALL-DONE
