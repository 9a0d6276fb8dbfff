"""Host cost of the data-parallel step on one GPU: a one-rank RCCL group with an
explicit exchange mode runs the real reduce-scatter / all-gather launches, so the
per-step time of C3 with the collectives issued eagerly between two graphs
(NCF_CAPTURE_ALLREDUCE=0, the world > 1 default) against captured in the step graph
(=1) and against the single-process step shows what the N > 1 bench pays on the host.

  python scripts/dp_overhead.py [steps]
"""
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(eng, steps):
    from bench import run_steps
    run_steps(eng, 20, True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(eng, steps, True)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e6


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from bench import make_train_data, CONFIGS
    from ncf_amd.engine import TrainEngine
    from ncf_amd.models import NCF
    from ncf_amd.pipeline import EpochPipeline
    ds, train = make_train_data("c3")
    _, f, nl, B = CONFIGS["c3"]
    U, I = ds["user_num"], ds["item_num"]
    out = {}
    for name, mode, cap in [("single", "single", "0"), ("zero1-eager", "zero1", "0"), ("zero1-captured", "zero1", "1"),
                            ("allreduce-eager", "allreduce", "0"), ("allreduce-captured", "allreduce", "1")]:
        os.environ["NCF_CAPTURE_ALLREDUCE"] = cap
        np.random.seed(0)
        torch.manual_seed(0)
        model = NCF(U, I, f, nl, 0.0, "NeuMF-end").to(dev)
        pipe = EpochPipeline(train, dev, B, I, user_num=U, prefetch=True)
        eng = TrainEngine(model, lr=1e-3, world_size=1, rank=0, process_group=dist.group.WORLD, dp_mode=mode)
        eng.stream_buffers = pipe.buffers
        eng.set_epoch_stream(pipe.next_epoch(peek_eval_draw=False), B, checked=True)

        def next_epoch(eng=eng, pipe=pipe):
            eng.set_epoch_stream(pipe.next_epoch(peek_eval_draw=False), B, checked=True)
        eng.next_epoch = next_epoch
        eng.batches_done = 0
        us = timed(eng, steps)
        out[name] = us
        print(f"{name}: {us:.1f} us/step ({B / us:.1f}M interactions/s)", flush=True)
        pipe.close()
        del eng, model, pipe
        torch.cuda.empty_cache()
    dist.destroy_process_group()
    print(out)


if __name__ == "__main__":
    main()
