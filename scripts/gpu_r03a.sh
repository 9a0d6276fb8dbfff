set -o pipefail
cd $GRAFT_REPO_ROOT
nproc > gpurun_out/r03a_nproc.txt
timeout -k 10 300 python scripts/sampler_bench.py --shape ml-1m --threads 12 --passes 8 > gpurun_out/r03a_sampler_ml1m.json 2>&1 &&
timeout -k 10 300 python scripts/sampler_bench.py --shape ml-20m --threads 12 --passes 4 > gpurun_out/r03a_sampler_ml20m.json 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03a_gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/r03a_bench_c3.json 2> gpurun_out/r03a_bench_c3.err
