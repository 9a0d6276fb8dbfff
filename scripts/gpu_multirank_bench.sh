# Rehearsal of bench.py's N > 1 flow on the one-GPU box: 2 and 3 ranks on cuda:0 over
# gloo, self-spawned and under torch.distributed.run (the driver's launcher), C3 and C4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp NCF_BENCH_SAME_DEVICE=1 NCF_BENCH_BACKEND=gloo
O=gpurun_out/mr
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > ${O}_spawn2_c3.json 2> ${O}_spawn2_c3.err || { echo spawn2-failed; tail -30 ${O}_spawn2_c3.err; exit 1; }
tail -c 600 ${O}_spawn2_c3.json; echo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > ${O}_run2_c3.json 2> ${O}_run2_c3.err || { echo run2-failed; tail -30 ${O}_run2_c3.err; exit 1; }
tail -c 300 ${O}_run2_c3.json; echo
timeout -k 10 400 python bench.py --gpus 3 --config c4 --no-weak --skip-eval --steps 20 --warmup 5 > ${O}_spawn3_c4.json 2> ${O}_spawn3_c4.err || { echo spawn3-c4-failed; tail -30 ${O}_spawn3_c4.err; exit 1; }
tail -c 300 ${O}_spawn3_c4.json; echo
echo all-done
