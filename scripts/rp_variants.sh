#!/usr/bin/env bash
# Per-kernel GPU durations of the bench workload for library variants (diagnosis):
#   make -C ncf_amd/csrc variant NAME=x VFLAGS=-DFOO   (-> ncf_amd/libncf_hip_x.so)
#   VARIANTS="default x" bash scripts/rp_variants.sh     (on the GPU box)
# One rocprofv3 --kernel-trace --stats pass per variant into gpurun_out/rp_<variant>/.
# (Back-to-back HIP-event timing of a short kernel from Python is bound by the host's
# launch rate; the kernel trace is not.)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then unset NCF_HIP_LIB; else export NCF_HIP_LIB=$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_$v -o run -- \
    python3 bench.py --config "${CONFIG:-c3}" --steps 40 --warmup 5 --skip-cpu-baseline --skip-eval --kernel-steps 5 \
    --e2e-epochs 0 > gpurun_out/rp_${CONFIG:-c3}_$v.log 2>&1
  mv gpurun_out/rp_$v "gpurun_out/rp_${CONFIG:-c3}_$v"
  find "gpurun_out/rp_${CONFIG:-c3}_$v" -type f ! -name '*kernel_stats.csv' -delete  # traces exceed the pull limit
done
