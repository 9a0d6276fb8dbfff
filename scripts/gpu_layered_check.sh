#!/usr/bin/env bash
# Layered-path check after a kernel change: the layered parity tests, two bench
# lines (CONFIG, default cli) and a kernel trace (gpurun_out/prof).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
    -k "${TESTS_K:-layered or cli or stress or dropout or odd or mlp-f or pre-f or 32 or user_order}" \
    -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    timeout -k 10 300 python bench.py --config "${CONFIG:-cli}" --steps 300 --warmup 20 --skip-cpu-baseline \
        --e2e-epochs 0 --skip-eval > gpurun_out/b$r.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/b$r.log').read().strip().splitlines()[-1]); print(round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --config "${CONFIG:-cli}" --steps 40 --warmup 3 --skip-cpu-baseline --skip-eval \
    --kernel-steps 3 --e2e-epochs 0 > gpurun_out/tr.log 2>&1
