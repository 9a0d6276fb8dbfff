# bf16 split GEMM core (layered path): parity subset, then stress / cli kernel traces and
# bench lines for the split core (default library) and the f32-MFMA core (NCF_HIP_LIB=f32)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/x6
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "layered or stress or cli or odd or mlp-f or pre-f or dropout or multitile" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > ${O}_tests.log 2>&1 || { echo tests-failed; tail -40 ${O}_tests.log; exit 1; }
tail -2 ${O}_tests.log
for v in x6s f32 x6p; do
  if [ $v = x6s ]; then unset NCF_HIP_LIB; else export NCF_HIP_LIB=$v; fi
  for cfg in stress cli; do
    timeout -k 10 240 python bench.py --config $cfg --steps 100 --skip-cpu-baseline --e2e-epochs 0 --skip-eval > ${O}_bench_${cfg}_$v.json 2> ${O}_bench_${cfg}_$v.err || { echo bench-$cfg-$v-failed; tail ${O}_bench_${cfg}_$v.err; exit 1; }
    python -c "import json; d=json.loads(open('${O}_bench_${cfg}_$v.json').read().strip().splitlines()[-1]); print('$cfg $v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step')"
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_trace_$v -o run -- python3 bench.py --config stress --steps 20 --warmup 5 --skip-cpu-baseline --skip-eval --kernel-steps 5 --e2e-epochs 0 --profile-run > ${O}_trace_$v.log 2>&1 || { echo trace-$v-failed; exit 1; }
done
echo all-done
