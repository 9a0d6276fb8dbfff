set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fault() { grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault|GPU Hang|core dumped" "$1"; }
timeout -k 10 900 python -u -m pytest -v -s --timeout 500 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_multirank_fullsize.py tests/test_gpu_multirank.py > gpurun_out/r4c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; fault gpurun_out/r4c_tests.log && exit 90
[ $rc -gt 1 ] && exit $rc
for w in 8 4 2 1; do
  NCF_WG_WAVES=$w timeout -k 10 200 python bench.py --config c5 --steps 3000 --warmup 300 --skip-cpu-baseline --e2e-epochs 0 > gpurun_out/r4c_c5_w$w.json 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --skip-cpu-baseline --e2e-epochs 0 > gpurun_out/r4c_c3.json 2>&1 || exit 1
echo DONE
