# round 3: sampler timing (host), GPU tests, C3 headline bench, C2 / C4 with and without deferred Adam
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r03b
nproc > ${O}_nproc.txt
timeout -k 10 300 python scripts/sampler_bench.py --shape ml-1m --threads 12 --passes 8 > ${O}_sampler_ml1m.json 2>&1 &&
timeout -k 10 300 python scripts/sampler_bench.py --shape ml-20m --threads 12 --passes 4 > ${O}_sampler_ml20m.json 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > ${O}_gpu_tests.log 2>&1 &&
timeout -k 10 400 python bench.py > ${O}_bench_c3.json 2> ${O}_bench_c3.err &&
timeout -k 10 200 python bench.py --config c2 --skip-cpu-baseline --e2e-epochs 4 > ${O}_bench_c2.json 2> ${O}_bench_c2.err &&
NCF_LAZY_ADAM=0 timeout -k 10 200 python bench.py --config c2 --skip-cpu-baseline --e2e-epochs 0 > ${O}_bench_c2_dense.json 2> ${O}_bench_c2_dense.err &&
timeout -k 10 300 python bench.py --config c4 --skip-cpu-baseline --e2e-epochs 2 > ${O}_bench_c4.json 2> ${O}_bench_c4.err &&
NCF_LAZY_ADAM=0 timeout -k 10 300 python bench.py --config c4 --skip-cpu-baseline --e2e-epochs 0 > ${O}_bench_c4_dense.json 2> ${O}_bench_c4_dense.err
