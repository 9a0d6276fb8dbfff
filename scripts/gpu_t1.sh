#!/usr/bin/env bash
# Focused GPU test run: the tests named by $K (pytest -k), output in gpurun_out/t1.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 "${SECS:-600}" python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "${K:-.}" > gpurun_out/t1.log 2>&1
rc=$?
echo "rc=$rc"
tail -40 gpurun_out/t1.log
exit $rc
