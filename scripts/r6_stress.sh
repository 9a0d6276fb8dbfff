#!/usr/bin/env bash
# Round 6: stress NCF(64,4) checks -- engine-level stress parity tests, then bench A/B over
# an env switch (AB_VAR, values AB_VALS), then (STAGES prof) a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6s; mkdir -p $O
STAGES="${STAGES:-tests bench}"
AB_VAR="${AB_VAR:-NCF_DX_WS}"; AB_VALS="${AB_VALS:-1 0 1}"
has() { case " $STAGES " in *" $1 "*) return 0 ;; esac; return 1; }
if has bitwise; then
  for v in $AB_VALS; do
    val=$v; [ "$v" = default ] && val=
    env $AB_VAR=$val timeout -k 10 200 python scripts/r6_bitwise.py ${CFG:-stress} ${BW_STEPS:-30} 2>&1 | grep "sha=" || exit 1
  done
fi
if has tests; then
  timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "${TESTS_K:-64 or LAYERED or layered or stress}" \
    > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  grep -E "passed|failed" $O/tests.log | tail -2
fi
if has bench; then
  for v in $AB_VALS; do
    val=$v; [ "$v" = default ] && val=
    env $AB_VAR=$val timeout -k 10 200 python bench.py --config ${CFG:-stress} --steps 50 --warmup 10 --skip-cpu-baseline \
      --no-script-epoch --e2e-epochs 0 > $O/bench_${AB_VAR}_$v.log 2>&1 || { tail -20 $O/bench_${AB_VAR}_$v.log; exit 1; }
    python3 -c "import json;l=[x for x in open('$O/bench_${AB_VAR}_$v.log') if x.startswith('{')][-1];d=json.loads(l);print('$AB_VAR=$v',round(d['value']/1e6,2),'M/s',round(d['ms_per_step']*1e3,1),'us/step', 'sustained', round(d['sustained']['value']/1e6,2) if d.get('sustained') else None)"
  done
fi
if has prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof${PTAG:-} -o run -- python3 bench.py --config ${CFG:-stress} --steps 20 --warmup 4 \
     --skip-cpu-baseline --no-script-epoch --e2e-epochs 0 --skip-eval > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  f=$(find $O/prof${PTAG:-} -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:12]: print('  %-70s %6s calls %9.2f us' % (r['Name'].replace('(anonymous namespace)::','')[:70], r['Calls'], float(r['AverageNs'])/1e3))"
fi
echo R6S-DONE
