# round-to-nearest bf16 split: the layered parity tests and whole epochs (cli, stress),
# stress / cli lines against the f32-core variant
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/rne
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -k "layered or stress or cli or odd or mlp-f or pre-f or dropout or multitile" "tests/test_gpu_fullsize.py::test_full_epoch_vs_oracle[stress-64-4-65536-3-0.0001]" "tests/test_gpu_fullsize.py::test_full_epoch_vs_oracle[cli-32-3-65536-4-1e-05]" -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > ${O}_tests.log 2>&1; echo tests-rc=$?
grep -E "passed|failed" ${O}_tests.log | tail -2
for v in default f32; do
  if [ $v = default ]; then unset NCF_HIP_LIB; else export NCF_HIP_LIB=$v; fi
  for cfg in stress cli; do
    timeout -k 10 240 python bench.py --config $cfg --steps 100 --skip-cpu-baseline --e2e-epochs 0 --skip-eval > ${O}_bench_${cfg}_$v.json 2> ${O}_bench_${cfg}_$v.err || { echo bench-$cfg-$v-failed; tail ${O}_bench_${cfg}_$v.err; exit 1; }
    python -c "import json; d=json.loads(open('${O}_bench_${cfg}_$v.json').read().strip().splitlines()[-1]); print('$cfg $v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step')"
  done
done
echo all-done
