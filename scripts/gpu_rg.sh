# Row-streaming GEMMs on pre-split weights (stress shape): parity, then stress traces and
# bench lines for the default library and the A/B variants given in VARIANTS
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/rg
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "layered or stress or cli or odd or mlp-f or pre-f or dropout or multitile" "tests/test_gpu_fullsize.py::test_full_epoch_vs_oracle[stress-64-4-65536-3-0.0001]" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > ${O}_tests.log 2>&1 || { echo tests-failed; tail -40 ${O}_tests.log; exit 1; }
tail -2 ${O}_tests.log
for v in ${VARIANTS:-default}; do
  if [ $v = default ]; then unset NCF_HIP_LIB; else export NCF_HIP_LIB=$v; fi
  timeout -k 10 240 python bench.py --config stress --steps 100 --skip-cpu-baseline --e2e-epochs 0 --skip-eval > ${O}_bench_stress_$v.json 2> ${O}_bench_stress_$v.err || { echo bench-$v-failed; tail ${O}_bench_stress_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('${O}_bench_stress_$v.json').read().strip().splitlines()[-1]); print('stress $v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,1), 'us/step')"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_trace_$v -o run -- python3 bench.py --config stress --steps 20 --warmup 5 --skip-cpu-baseline --skip-eval --kernel-steps 5 --e2e-epochs 0 --profile-run > ${O}_trace_$v.log 2>&1 || { echo trace-$v-failed; exit 1; }
done

if [ -n "${PMC:-}" ]; then
  unset NCF_HIP_LIB
  for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
    n=$(echo $c | cut -d' ' -f1)
    timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d ${O}_pmc_$n -o run -- python3 bench.py --config stress --steps 10 --warmup 3 --skip-cpu-baseline --skip-eval --kernel-steps 2 --e2e-epochs 0 --profile-run > ${O}_pmc_$n.log 2>&1 || { echo pmc-$n-failed; exit 1; }
  done
  echo pmc-done
fi
echo all-done
