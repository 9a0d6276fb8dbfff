# layered GEMM core with K-contiguous LDS tiles and 16-byte LDS reads: parity, stress / cli lines, stress trace + SQ
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r03m
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -k "layered or dropout or multitile or fact" "tests/test_gpu_fullsize.py::test_full_epoch_vs_oracle[stress-64-4-65536-3-0.0001]" "tests/test_gpu_fullsize.py::test_full_epoch_vs_oracle[cli-32-3-65536-4-1e-05]" -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > ${O}_tests.log 2>&1 || { echo tests-failed; tail -30 ${O}_tests.log; exit 1; }
for cfg in stress cli; do
  timeout -k 10 240 python bench.py --config $cfg --skip-cpu-baseline --e2e-epochs 0 --skip-eval > ${O}_bench_${cfg}.json 2> ${O}_bench_${cfg}.err || { echo bench-failed; tail ${O}_bench_${cfg}.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03m_trace -o run -- python3 bench.py --config stress --steps 20 --warmup 5 --skip-cpu-baseline --skip-eval --kernel-steps 5 --e2e-epochs 0 --profile-run > ${O}_trace.log 2>&1 || { echo trace-failed; exit 1; }
echo all-done
