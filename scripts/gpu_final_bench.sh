# final bench lines: the driver's command on the fresh box first, the default line, and
# the N = 2 rehearsal (gloo, one device) of the multi-rank flow
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/fb_driver.json 2> gpurun_out/fb_driver.err || { tail gpurun_out/fb_driver.err; exit 1; }
tail -c 200 gpurun_out/fb_driver.json; echo
timeout -k 10 400 python3 bench.py > gpurun_out/fb_default.json 2> gpurun_out/fb_default.err || { tail gpurun_out/fb_default.err; exit 1; }
tail -c 200 gpurun_out/fb_default.json; echo
NCF_BENCH_SAME_DEVICE=1 NCF_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/fb_rehearsal2.json 2> gpurun_out/fb_rehearsal2.err || { tail -20 gpurun_out/fb_rehearsal2.err; exit 1; }
tail -c 200 gpurun_out/fb_rehearsal2.json; echo
echo all-done
