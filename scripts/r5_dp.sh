#!/usr/bin/env bash
# Round-5 data-parallel evidence: per-rank local costs of allreduce / touched / owner at
# emulated N = 2, 4, 8 (dp_modes.py, graph replay), then one rocprofv3 kernel trace per
# (config, mode) at N = 8 for the one-rank collectives' kernel time (subtracted by
# scaling_model.py --local graph).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/dp5
for spec in ${DP_SPECS:-c3:8:allreduce,owner c4:8:touched,owner c3:4:allreduce,owner c4:4:touched,owner c3:2:allreduce,owner c4:2:touched,owner}; do
    IFS=: read -r cfg n modes <<< "$spec"
    echo "== $cfg n$n $modes"
    timeout -k 10 300 python3 scripts/dp_modes.py "$cfg" "$n" "$modes" > "gpurun_out/dp5/dp_${cfg}_n${n}.json" \
        2> "gpurun_out/dp5/dp_${cfg}_n${n}.err" || { tail -20 "gpurun_out/dp5/dp_${cfg}_n${n}.err"; exit 1; }
    tail -c 300 "gpurun_out/dp5/dp_${cfg}_n${n}.json"; echo
done
for spec in ${TRACE_SPECS:-c3:allreduce c3:owner c4:touched c4:owner}; do
    IFS=: read -r cfg mode <<< "$spec"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/dp5/tr_${cfg}_${mode}" -o run \
        -- python3 scripts/dp_modes.py "$cfg" 8 "$mode" > "gpurun_out/dp5/tr_${cfg}_${mode}.log" 2>&1 \
        || { tail -20 "gpurun_out/dp5/tr_${cfg}_${mode}.log"; exit 1; }
done
echo DP-DONE
