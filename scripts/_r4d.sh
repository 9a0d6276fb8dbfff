set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fault() { grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault|GPU Hang|core dumped" "$1"; }
runt() {  # name, seconds, pytest args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m pytest -v -s --timeout 500 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/r4d_$n.log 2>&1
  local rc=$?; echo "$n rc=$rc $(tail -1 gpurun_out/r4d_$n.log)"; fault gpurun_out/r4d_$n.log && exit 90
  [ $rc -gt 1 ] && exit $rc
  return 0
}
runt parity 600 tests/test_gpu_parity.py
runt fullsize 600 tests/test_gpu_fullsize.py -k "c2 or c3"
runt multirank 900 tests/test_gpu_multirank_fullsize.py tests/test_gpu_multirank.py
for w in 8 4 2 1; do
  NCF_WG_WAVES=$w timeout -k 10 200 python bench.py --config c2 --steps 2000 --warmup 200 --skip-cpu-baseline --e2e-epochs 0 > gpurun_out/r4d_c2_w$w.json 2>&1 || exit 1
  NCF_WG_WAVES=$w timeout -k 10 200 python bench.py --config c5 --steps 3000 --warmup 300 --skip-cpu-baseline --e2e-epochs 0 > gpurun_out/r4d_c5_w$w.json 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --skip-cpu-baseline --e2e-epochs 0 > gpurun_out/r4d_c3.json 2>&1 || exit 1
echo DONE
