# rocprofv3 evidence for C2 and C4 (trace + FETCH/WRITE/SQ passes), plus a C2 trace with deferred Adam
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in c2 c4; do
  CONFIG=$cfg timeout -k 10 900 bash scripts/profile.sh > gpurun_out/profile_$cfg.log 2>&1 || { echo profile-$cfg-failed; tail -20 gpurun_out/profile_$cfg.log; exit 1; }
  mkdir -p gpurun_out/prof_$cfg
  cp gpurun_out/prof_summary.md gpurun_out/prof_summary.json gpurun_out/prof/run_kernel_stats.csv gpurun_out/prof_$cfg/
  echo profile-$cfg-done
done
NCF_LAZY_ADAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2_lazy -o run -- python3 bench.py --config c2 --steps 60 --warmup 5 --skip-cpu-baseline --skip-eval --kernel-steps 5 --e2e-epochs 0 --profile-run > gpurun_out/prof_c2_lazy.log 2>&1 || { echo lazy-trace-failed; exit 1; }
echo all-done
