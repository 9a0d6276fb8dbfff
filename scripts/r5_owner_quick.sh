export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_owner.py tests/test_gpu_multirank.py -k "owner" -q --maxfail=3 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5o_tests.log 2>&1 || { tail -30 gpurun_out/r5o_tests.log; exit 1; }
tail -1 gpurun_out/r5o_tests.log
mkdir -p gpurun_out/dp6
for c in c3 c4; do
  timeout -k 10 300 python3 scripts/dp_modes.py $c 8 owner > gpurun_out/dp6/dp_${c}_n8.json 2> gpurun_out/dp6/dp_${c}_n8.err || { tail -5 gpurun_out/dp6/dp_${c}_n8.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dp6/tr_$c -o run -- python3 scripts/dp_modes.py $c 8 owner > gpurun_out/dp6/tr_$c.log 2>&1 || exit 1
  python3 -c "
import csv, json
d=json.loads(open('gpurun_out/dp6/dp_${c}_n8.json').read().strip().splitlines()[-1])
print('$c graph us', round(d['modes']['owner']['ms_per_step_graph']*1e3,1))
for r in list(csv.DictReader(open('gpurun_out/dp6/tr_$c/run_kernel_stats.csv')))[:6]: print('  ', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,2))"
done
