#!/usr/bin/env bash
# C2 / C5 step time: in-step Adam at 4 / 2 / 1-wave geometries against the two-launch form.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/geo
for cfg in ${CONFIGS:-c2 c5}; do
  for spec in 4:0 4:1 2:1 1:1 2:0; do
    IFS=: read -r wv ais <<< "$spec"
    timeout -k 10 300 env NCF_WG_WAVES=$wv NCF_ADAM_IN_STEP=$ais python bench.py --config $cfg --steps 400 --warmup 20 \
      --skip-cpu-baseline --skip-eval --e2e-epochs 0 > gpurun_out/geo/${cfg}_w${wv}_a${ais}.log 2>&1 || { tail -20 gpurun_out/geo/${cfg}_w${wv}_a${ais}.log; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/geo/${cfg}_w${wv}_a${ais}.log') if l.startswith('{')][-1]; print('$cfg waves=$wv ais=$ais', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1000,2), 'us/step')"
  done
done
