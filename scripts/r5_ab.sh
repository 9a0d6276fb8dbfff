#!/usr/bin/env bash
# A/B of one environment variable over bench configs, interleaved (AB_VAR, AB_VALS, AB_CONFIGS),
# then one kernel trace per config with the first value.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/ab
for cfg in ${AB_CONFIGS:-c2 c5 c3}; do
    for r in 1 2; do
        for v in ${AB_VALS:-1 0}; do
            timeout -k 10 300 env "$AB_VAR=$v" python bench.py --config "$cfg" --steps "${AB_STEPS:-400}" --warmup 20 \
                --skip-cpu-baseline --skip-eval --e2e-epochs 0 > "gpurun_out/ab/${cfg}_${v}_$r.log" 2>&1 || {
                tail -20 "gpurun_out/ab/${cfg}_${v}_$r.log"; exit 1; }
            python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/ab/${cfg}_${v}_$r.log') if l.startswith('{')][-1]; print('$cfg $AB_VAR=$v', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1000,2), 'us/step', 'sustained', round((d.get('sustained') or {}).get('value', 0)/1e6,2), round((d.get('sustained') or {}).get('ms_per_step', 0)*1000,2))"
        done
    done
done
if [ "${AB_TRACE:-1}" = "1" ]; then
    v1=$(echo ${AB_VALS:-1 0} | cut -d' ' -f1)
    for cfg in ${AB_CONFIGS:-c2 c5 c3}; do
        timeout -k 10 300 env "$AB_VAR=$v1" rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/ab/tr_$cfg" \
            -o run -- python3 bench.py --config "$cfg" --steps 60 --warmup 5 --skip-cpu-baseline --skip-eval \
            --e2e-epochs 0 --kernel-steps 5 > "gpurun_out/ab/tr_$cfg.log" 2>&1 || { tail -20 "gpurun_out/ab/tr_$cfg.log"; exit 1; }
        find "gpurun_out/ab/tr_$cfg" -type f ! -name '*kernel_stats.csv' -delete  # the traces exceed the pull limit
    done
fi
echo AB-DONE
