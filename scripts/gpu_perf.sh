set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log
if grep -qE "illegal memory|Memory access fault|GPU Hang|HIP error" gpurun_out/pytest_gpu.log; then echo FAULT; exit 90; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --skip-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 python scripts/stamps.py > gpurun_out/stamps.log 2>&1 || exit $?
echo DONE
