# Round-3 (second session) evidence: the evidence session (smoke, all GPU tests, bench
# lines, stress rocprofv3 passes), then the driver's own bench command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SAMPLER=0 PROFILE=1 PROFILE_CONFIGS=stress bash scripts/gpu_evidence.sh || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_cmd.json 2> gpurun_out/bench_driver_cmd.err || exit $?
tail -c 300 gpurun_out/bench_driver_cmd.json
