# deferred Adam v2 (disjoint A/B/C lists, no claims): parity tests, then lazy vs dense
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r03g
timeout -k 10 500 python -u -m pytest tests/test_gpu_lazy_adam.py tests/test_gpu_integration.py tests/test_gpu_multirank.py -x -v --timeout 170 --timeout-method thread > ${O}_tests.log 2>&1 || { echo tests-failed; tail -30 ${O}_tests.log; exit 1; }
for cfg in c2 c5 c4; do
  NCF_LAZY_ADAM=1 timeout -k 10 240 python bench.py --config $cfg --skip-cpu-baseline --e2e-epochs 0 --skip-eval > ${O}_bench_${cfg}_lazy.json 2> ${O}_bench_${cfg}_lazy.err || { echo bench-$cfg-failed; tail ${O}_bench_${cfg}_lazy.err; exit 1; }
  NCF_LAZY_ADAM=0 timeout -k 10 240 python bench.py --config $cfg --skip-cpu-baseline --e2e-epochs 0 --skip-eval > ${O}_bench_${cfg}_dense.json 2> ${O}_bench_${cfg}_dense.err || { echo bench-$cfg-failed; exit 1; }
done
echo all-done
