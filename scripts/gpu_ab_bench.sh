#!/usr/bin/env bash
# GPU tests, then the bench under two settings of one environment variable
# (A/B, interleaved twice).  Usage: bash scripts/gpu_ab_bench.sh VAR VALUE_A VALUE_B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log
if grep -qE "illegal memory|Memory access fault|GPU Hang|HIP error" gpurun_out/pytest_gpu.log; then echo FAULT; exit 90; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VAR=$1; A=$2; B=$3
for r in 1 2; do
  for v in "$A" "$B"; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --steps 300 --warmup 20 --skip-cpu-baseline --skip-eval > gpurun_out/ab_$v.log 2>&1 || exit $?
    python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/ab_$v.log') if l.startswith('{')][-1]; print('$VAR=$v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1000,2), 'us/step')"
  done
done
