#!/usr/bin/env bash
# Round 6: wide-chain (dm 512) parity tests, stress bench A/B (NCF_WIDE_CHAIN=0/1), kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6w; mkdir -p $O
STAGES="${STAGES:-tests bench prof}"
has() { case " $STAGES " in *" $1 "*) return 0 ;; esac; return 1; }
if has tests; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py -k "64 or LAYERED or layered or stress" tests/test_gpu_fullsize.py -k "stress or 64" \
    > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  grep -E "passed|failed" $O/tests.log | tail -2
fi
if has bench; then
  for v in 1 0 1; do
    NCF_WIDE_CHAIN=$v timeout -k 10 200 python bench.py --config stress --steps 50 --warmup 10 --skip-cpu-baseline \
      --no-script-epoch --e2e-epochs 0 > $O/bench_stress_w$v.log 2>&1 || { tail -20 $O/bench_stress_w$v.log; exit 1; }
    python3 -c "import json,sys;l=[x for x in open('$O/bench_stress_w$v.log') if x.startswith('{')][-1];d=json.loads(l);print('wide=$v',d['value']/1e6,'M/s',d['ms_per_step']*1e3,'us/step')"
  done
fi
if has prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o stress -- python3 bench.py --config stress --steps 20 --warmup 4 \
     --skip-cpu-baseline --no-script-epoch --e2e-epochs 0 --skip-eval > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  f=$(find $O/prof -name "*kernel_stats.csv" | head -1); head -16 "$f" | cut -c1-160
fi
