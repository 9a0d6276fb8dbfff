#!/usr/bin/env bash
# dp evidence + the full-shape multi-rank parity tests (owner / auto / weak scaling)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/owner
bash scripts/r5_dp.sh || exit 1
timeout -k 10 1000 python -u -m pytest tests/test_gpu_multirank_fullsize.py tests/test_gpu_multirank.py -v -s \
    --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/owner/fullsize2.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|max rel" gpurun_out/owner/fullsize2.log | cut -c1-300
exit $rc
