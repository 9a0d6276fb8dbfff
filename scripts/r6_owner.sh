#!/usr/bin/env bash
# Round 6: C3 emulated-N=8 owner chain A/B (dp_modes.py graph replay + a kernel trace per variant).
# VARIANTS: space-separated "name:ENV=val,ENV=val" (default: FACT vs per-row layer 0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6o; mkdir -p $O
CFG="${CFG:-c3}"; N="${N:-8}"; MODES="${MODES:-owner}"
TRACE="${TRACE:-1}"
for v in ${VARIANTS:-fact:NCF_PER_ROW=0 perrow:NCF_PER_ROW=1}; do
  name=${v%%:*}; envs=${v#*:}
  ENVA=(); IFS=, read -ra kv <<< "$envs"; for e in "${kv[@]}"; do [ -n "$e" ] && ENVA+=("$e"); done
  echo "== $name ${ENVA[*]}"
  env "${ENVA[@]}" timeout -k 10 300 python3 scripts/dp_modes.py "$CFG" "$N" "$MODES" > "$O/dp_${CFG}_n${N}_$name.json" \
      2> "$O/dp_${CFG}_n${N}_$name.err" || { tail -20 "$O/dp_${CFG}_n${N}_$name.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/dp_${CFG}_n${N}_$name.json'));print({m:(round(v['ms_per_step_graph']*1e3,1),v['launch_groups_ms']) for m,v in d['modes'].items()})"
  if [ "$TRACE" = 1 ]; then
    for e in "${ENVA[@]}"; do export "$e"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/tr_$name" -o run \
        -- python3 scripts/dp_modes.py "$CFG" "$N" "$MODES" > "$O/tr_$name.log" 2>&1 || { tail -20 "$O/tr_$name.log"; exit 1; }
    for e in "${ENVA[@]}"; do unset "${e%%=*}"; done
    f=$(find "$O/tr_$name" -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:8]: print('  %-60s %6s calls %8.2f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
  fi
done
echo R6O-DONE
