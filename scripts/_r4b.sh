set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fault() { grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault|GPU Hang|core dumped" "$1"; }
timeout -k 10 800 python -u -m pytest -v -s --timeout 500 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "prepare_epoch or geometry_vs_oracle" \
  tests/test_gpu_multirank_fullsize.py tests/test_gpu_multirank.py::test_two_ranks_match_single_rank \
  tests/test_gpu_trainer.py::test_trainer_matches_reference_script tests/test_gpu_lazy_adam.py > gpurun_out/r4b_tests2.log 2>&1
rc=$?; echo "tests2 rc=$rc"; fault gpurun_out/r4b_tests2.log && exit 90
[ $rc -gt 1 ] && exit $rc
for w in 8 4; do
  NCF_WG_WAVES=$w timeout -k 10 200 python scripts/dp_modes.py c3 8 allreduce,zero1 > gpurun_out/r4b_dp_c3_w$w.json 2>&1 || exit 1
done
for w in 8 4 2 1; do
  NCF_WG_WAVES=$w timeout -k 10 200 python bench.py --config c2 --steps 2000 --warmup 200 --skip-cpu-baseline --e2e-epochs 0 > gpurun_out/r4b_c2_w$w.json 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --skip-cpu-baseline --e2e-epochs 0 > gpurun_out/r4b_c3.json 2>&1 || exit 1
for a in "c2 1024" "c3 8192"; do NCF_WG_WAVES=8 timeout -k 10 120 python scripts/stamps.py $a >> gpurun_out/r4b_stamps.jsonl 2>>gpurun_out/r4b_stamps.err || exit 1; done
echo DONE
