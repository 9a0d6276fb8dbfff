#!/usr/bin/env bash
# A/B of an environment switch on the bench (GPU box):
#   AB_VAR=NCF_SPLIT_ADAM AB_VALUES="1 0" CONFIGS="c3 cli" REPS=2 bash scripts/gpu_ab_env.sh
# Every (rep, config, value) is one bench process, interleaved so drift hits all
# values alike; one summary line each.  Output in gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAR=${AB_VAR:?set AB_VAR}
for rep in $(seq 1 "${REPS:-2}"); do
  for cfg in ${CONFIGS:-c3}; do
    for val in ${AB_VALUES:-0 1}; do
      log=gpurun_out/ab_${cfg}_${VAR}_${val}_${rep}.log
      env "$VAR=$val" timeout -k 10 300 python bench.py --config "$cfg" --steps "${STEPS:-400}" --warmup 20 \
          --skip-cpu-baseline --e2e-epochs 0 --skip-eval > "$log" 2>&1 || exit $?
      python -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('$cfg $VAR=$val rep $rep', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step')"
    done
  done
done
