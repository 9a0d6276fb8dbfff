# deferred Adam A/B after the rolling catch-up / overlapped-claim rework
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r03f
timeout -k 10 400 python -u -m pytest tests/test_gpu_lazy_adam.py tests/test_gpu_integration.py "tests/test_gpu_multirank.py::test_two_ranks_match_single_rank" -x -v --timeout 170 --timeout-method thread > ${O}_tests.log 2>&1 || { echo tests-failed; exit 1; }
for cfg in c2 c5 c4; do
  timeout -k 10 240 python bench.py --config $cfg --skip-cpu-baseline --e2e-epochs 0 --skip-eval > ${O}_bench_${cfg}.json 2> ${O}_bench_${cfg}.err || { echo bench-$cfg-failed; exit 1; }
done
for span in 8 64; do
  NCF_LAZY_SPAN=$span timeout -k 10 240 python bench.py --config c2 --skip-cpu-baseline --e2e-epochs 0 --skip-eval > ${O}_bench_c2_span${span}.json 2> ${O}_bench_c2_span${span}.err
done
echo all-done
