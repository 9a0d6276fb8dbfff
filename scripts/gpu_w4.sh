# min-waves launch bound on the bf16-split GEMM kernels (stress) + the metrics loader test
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/w4
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "metrics_unequal or hr_ndcg" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > ${O}_tests.log 2>&1 || { echo tests-failed; tail -30 ${O}_tests.log; exit 1; }
tail -1 ${O}_tests.log
for v in default w4; do
  if [ $v = default ]; then unset NCF_HIP_LIB; else export NCF_HIP_LIB=$v; fi
  for r in 1 2; do
    timeout -k 10 240 python bench.py --config stress --steps 100 --skip-cpu-baseline --e2e-epochs 0 --skip-eval > ${O}_bench_$v$r.json 2> ${O}_bench_$v$r.err || { echo bench-$v-failed; tail ${O}_bench_$v$r.err; exit 1; }
    python -c "import json; d=json.loads(open('${O}_bench_$v$r.json').read().strip().splitlines()[-1]); print('stress $v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step')"
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_trace_$v -o run -- python3 bench.py --config stress --steps 20 --warmup 5 --skip-cpu-baseline --skip-eval --kernel-steps 5 --e2e-epochs 0 --profile-run > ${O}_trace_$v.log 2>&1 || { echo trace-$v-failed; exit 1; }
done
echo all-done
