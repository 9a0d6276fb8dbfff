export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fact_adam.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5q_tests.log 2>&1 || { tail -30 gpurun_out/r5q_tests.log; exit 1; }
tail -1 gpurun_out/r5q_tests.log
for v in 1 0 1; do
  NCF_FACT_IN_ADAM=$v timeout -k 10 300 python bench.py --steps 200 --warmup 20 --skip-cpu-baseline --skip-eval --e2e-epochs 0 > gpurun_out/r5q_bench_$v.log 2>&1 || { tail -20 gpurun_out/r5q_bench_$v.log; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r5q_bench_$v.log') if l.startswith('{')][-1]; print('FACT_IN_ADAM=$v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1000,2), 'us/step', {k: (round(v*1e3,2) if isinstance(v,float) else v) for k,v in d['kernel_ms'].items() if not isinstance(v, dict)})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3fa2 -o run -- python3 bench.py --steps 60 --warmup 5 --skip-cpu-baseline --skip-eval --kernel-steps 5 --e2e-epochs 0 --profile-run > gpurun_out/prof_c3fa2.log 2>&1 || exit 1
python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/prof_c3fa2/run_kernel_stats.csv')))[:4]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2))"
