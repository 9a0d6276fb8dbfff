# round 3: multirank first (last run hung in it), then the rest of the GPU tests, sampler sweeps, benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r03c
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_lazy_adam.py -x -v -s --timeout 170 --timeout-method thread > ${O}_gpu_multirank.log 2>&1 || { echo multirank-failed; exit 1; }
for b in 16384 32768 65536; do
  NCF_SAMPLER_BLOCK=$b timeout -k 10 300 python scripts/sampler_bench.py --shape ml-1m --threads 12 --passes 8 >> ${O}_sampler_ml1m.jsonl 2>&1
  NCF_SAMPLER_BLOCK=$b timeout -k 10 300 python scripts/sampler_bench.py --shape ml-20m --threads 12 --passes 4 >> ${O}_sampler_ml20m.jsonl 2>&1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 250 --timeout-method thread --deselect tests/test_gpu_fullsize.py::test_full_epoch_vs_oracle[c4-16-3-65536-3-1e-05] > ${O}_gpu_tests.log 2>&1 || { echo tests-failed; exit 1; }
timeout -k 10 400 python bench.py > ${O}_bench_c3.json 2> ${O}_bench_c3.err
timeout -k 10 200 python bench.py --config c2 --skip-cpu-baseline --e2e-epochs 4 > ${O}_bench_c2.json 2> ${O}_bench_c2.err
NCF_LAZY_ADAM=0 timeout -k 10 200 python bench.py --config c2 --skip-cpu-baseline --e2e-epochs 0 > ${O}_bench_c2_dense.json 2> ${O}_bench_c2_dense.err
timeout -k 10 300 python bench.py --config c4 --skip-cpu-baseline --e2e-epochs 2 > ${O}_bench_c4.json 2> ${O}_bench_c4.err
NCF_LAZY_ADAM=0 timeout -k 10 300 python bench.py --config c4 --skip-cpu-baseline --e2e-epochs 0 > ${O}_bench_c4_dense.json 2> ${O}_bench_c4_dense.err
echo all-done
