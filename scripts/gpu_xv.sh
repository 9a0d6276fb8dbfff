set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in base xtower xemb; do
  if [ $v = base ]; then unset NCF_HIP_LIB; else export NCF_HIP_LIB=$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xv_$v -o run -- python3 bench.py --config c3 --steps 60 --warmup 5 --skip-cpu-baseline --skip-eval --kernel-steps 5 --e2e-epochs 0 --profile-run > gpurun_out/xv_$v.log 2>&1 || exit 1
done
