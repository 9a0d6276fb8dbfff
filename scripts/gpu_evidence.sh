#!/usr/bin/env bash
# Evidence sessions on the GPU box (gpurun -- 'bash scripts/gpu_evidence.sh').  The
# stages to run are named in STAGES (default: the round-end set, in this order):
#   smoke      __graft_entry__.smoke()
#   tests      pytest -m gpu (TESTS: the selection, default the whole suite)
#   bench      the default bench line (C3, CPU baseline, Trainer.fit e2e figure)
#   configs    one line per other config (CONFIGS, default c2 c4 cli stress c5)
#   sampler    host sampler passes at ml-1m / ml-20m (scripts/sampler_bench.py)
#   profile    rocprofv3 kernel trace + FETCH / WRITE / SQ passes per config
#              (PROFILE_CONFIGS, default c3; scripts/profile.sh)
#   multirank  bench.py's N > 1 flow rehearsed on the one GPU: 2 ranks on cuda:0 over
#              gloo, self-spawned and under torch.distributed.run (C3), 3 ranks at C4
#   stamps     phase stamps of the step kernel (diagnostics library, scripts/stamps.py)
#   ab         the bench under two values of one variable, interleaved twice
#              (AB="VAR VALUE_A VALUE_B")
# Each GPU step has its own time limit; a crash, fault or timeout ends the script.
# Output in gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
STAGES="${STAGES:-smoke tests bench configs sampler profile}"
run() {  # name, seconds, cmd...
    local name=$1 secs=$2
    shift 2
    echo "== $name: $*" | tee -a gpurun_out/steps.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
    tail -2 "gpurun_out/$name.log"
    if grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault|GPU Hang" "gpurun_out/$name.log"; then
        echo "stopping after $name: GPU fault signature in log"; exit 90
    fi
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    if [ $rc -ne 0 ] && [ "${STOP_ON_FAIL:-0}" = "1" ]; then echo "stopping after $name (failed)"; exit 1; fi
    return 0
}
has() { case " $STAGES " in *" $1 "*) return 0 ;; esac; return 1; }

has smoke && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
if has tests; then
    # shellcheck disable=SC2086
    run pytest_gpu 1100 python -u -m pytest ${TESTS:-tests -m gpu} -v -s -x --timeout 500 --timeout-method thread \
        -p no:cacheprovider
fi
has bench && run bench 600 python bench.py
if has configs; then
    for cfg in ${CONFIGS:-c2 c4 cli stress c5}; do
        run "bench_$cfg" 300 python bench.py --config "$cfg" --steps 200 --warmup 20 --skip-cpu-baseline \
            --e2e-epochs "${E2E:-2}"
        tail -1 "gpurun_out/bench_$cfg.log" >> gpurun_out/configs.jsonl
    done
fi
if has sampler; then
    for shape in ml-1m ml-20m; do
        run "sampler_$shape" 300 python scripts/sampler_bench.py --shape $shape --passes 6
        tail -1 "gpurun_out/sampler_$shape.log" >> gpurun_out/sampler.jsonl
    done
fi
if has profile; then
    for cfg in ${PROFILE_CONFIGS:-c3}; do  # scripts/profile.sh writes fixed names: keep a copy per config
        export CONFIG=$cfg
        run "profile_$cfg" 900 bash scripts/profile.sh
        mkdir -p "gpurun_out/prof_$cfg"
        cp gpurun_out/prof_summary.md gpurun_out/prof_summary.json gpurun_out/prof/run_kernel_stats.csv \
            "gpurun_out/prof_$cfg/"
        # the box's copy of the tree: later stages of this call (bench, configs) read the
        # newest committed summary of their config for the roofline's traffic field
        cp gpurun_out/prof_summary.json "profiles/${PROF_TAG:-r05}_${cfg}_prof_summary.json"
    done
fi
if has multirank; then
    export NCF_BENCH_SAME_DEVICE=1 NCF_BENCH_BACKEND=gloo
    run mr_spawn2_c3 300 python bench.py --gpus 2 --steps 20 --warmup 5
    run mr_run2_c3 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5
    run mr_spawn3_c4 400 env NCF_BENCH_SUSTAINED_EPOCHS=0 python bench.py --gpus 3 --config c4 --no-weak \
        --skip-eval --steps 20 --warmup 5
    unset NCF_BENCH_SAME_DEVICE NCF_BENCH_BACKEND
fi
if has stamps; then
    run stamps 300 python scripts/stamps.py ${STAMPS_ARGS:-}
fi
if has ab; then
    # shellcheck disable=SC2086
    set -- $AB
    VAR=$1 A=$2 B=$3
    for r in 1 2; do
        for v in "$A" "$B"; do
            run "ab_${v}_$r" 300 env "$VAR=$v" python bench.py --steps 300 --warmup 20 --skip-cpu-baseline --skip-eval
            python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/ab_${v}_$r.log') if l.startswith('{')][-1]; print('$VAR=$v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1000,2), 'us/step')"
        done
    done
fi
echo ALL-DONE
