#!/usr/bin/env bash
# dp_mode "owner" evidence on the one-GPU box: per-rank local costs at emulated worlds
# (scripts/dp_modes.py: rank 0 of N over a one-rank RCCL group) and the full-shape
# multi-rank parity tests (gloo ranks on cuda:0).  STAGES: dp tests (default both).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/owner
export TMPDIR=/tmp PYTHONUNBUFFERED=1
STAGES="${STAGES:-dp tests}"
has() { case " $STAGES " in *" $1 "*) return 0 ;; esac; return 1; }
if has dp; then
    for spec in ${DP_SPECS:-c3:8:allreduce,owner c3:4:allreduce,owner c3:2:allreduce,owner c4:8:touched,owner c4:4:touched,owner c4:2:touched,owner}; do
        IFS=: read -r cfg n modes <<< "$spec"
        echo "== dp $cfg n$n $modes"
        timeout -k 10 300 python scripts/dp_modes.py "$cfg" "$n" "$modes" > "gpurun_out/owner/dp_${cfg}_n${n}.json" 2> "gpurun_out/owner/dp_${cfg}_n${n}.err"
        rc=$?
        tail -c 400 "gpurun_out/owner/dp_${cfg}_n${n}.json"; echo
        if [ $rc -ne 0 ]; then tail -20 "gpurun_out/owner/dp_${cfg}_n${n}.err"; exit $rc; fi
    done
fi
if has tests; then
    timeout -k 10 1000 python -u -m pytest tests/test_gpu_multirank_fullsize.py -k "${TESTS_K:-owner or c3-8}" -v -s \
        --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/owner/fullsize.log 2>&1
    rc=$?
    grep -E "PASSED|FAILED|ERROR|max rel" gpurun_out/owner/fullsize.log | cut -c1-400
    exit $rc
fi
