export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fact_adam.py tests/test_gpu_owner.py tests/test_gpu_multirank.py tests/test_gpu_distill.py -k "fact or owner or different or c5_id" -q --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5c_tests.log 2>&1 || { tail -40 gpurun_out/r5c_tests.log; exit 1; }
tail -2 gpurun_out/r5c_tests.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --skip-cpu-baseline --skip-eval --e2e-epochs 0 > gpurun_out/r5c_bench_c3.log 2>&1 || { tail -20 gpurun_out/r5c_bench_c3.log; exit 1; }
python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r5c_bench_c3.log') if l.startswith('{')][-1]; print('C3', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1000,2), 'us/step', {k: (round(v*1e3,2) if isinstance(v,float) else v) for k,v in d['kernel_ms'].items() if not isinstance(v, dict)})"
for c in c3 c4; do timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_owner2_$c -o run -- python3 scripts/dp_modes.py $c 8 owner > gpurun_out/prof_owner2_$c.log 2>&1 || exit 1; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3fa -o run -- python3 bench.py --steps 60 --warmup 5 --skip-cpu-baseline --skip-eval --kernel-steps 5 --e2e-epochs 0 --profile-run > gpurun_out/prof_c3fa.log 2>&1 || exit 1
echo ALL-OK
