# step-scalar cache: the whole GPU suite (C4 whole epoch included), then C3 / C2 / C5 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r03i
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > ${O}_gpu_tests.log 2>&1 || { echo tests-failed; tail -30 ${O}_gpu_tests.log; exit 1; }
for cfg in c3 c2 c5; do
  timeout -k 10 240 python bench.py --config $cfg --skip-cpu-baseline --e2e-epochs 0 --skip-eval > ${O}_bench_${cfg}.json 2> ${O}_bench_${cfg}.err || { echo bench-$cfg-failed; tail ${O}_bench_${cfg}.err; exit 1; }
done
echo all-done
