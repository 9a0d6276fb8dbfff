#!/usr/bin/env bash
# rocprofv3 kernel trace + FETCH/WRITE/SQ passes (scripts/profile.sh) for several bench
# configs in one GPU session; a copy of each summary under gpurun_out/prof_<config>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${PROFILE_CONFIGS:-c3 c2 c4}; do
    echo "== profile $cfg"
    CONFIG=$cfg timeout -k 10 600 bash scripts/profile.sh > "gpurun_out/profile_$cfg.log" 2>&1
    rc=$?
    echo "== profile $cfg rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "gpurun_out/profile_$cfg.log"; exit $rc; fi
    mkdir -p "gpurun_out/prof_$cfg"
    cp gpurun_out/prof_summary.md gpurun_out/prof_summary.json gpurun_out/prof/run_kernel_stats.csv "gpurun_out/prof_$cfg/"
done
echo ALL-DONE
