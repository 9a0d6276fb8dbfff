#!/usr/bin/env python3
"""Per-rank device cost of each data-parallel exchange mode at N ranks, measured on one
GPU: the engine runs as rank 0 of `world` (its shard of every global batch, the lists
of the whole global batch) over a one-rank RCCL group, so every launch of the step is
the real one and the collective moves nothing.  Prints, per mode, the graph-replayed
ms per step and the per-launch-group event times -- the local part of the N-rank step
(the wire time of the all-reduce comes on top and is the same bytes for 'allreduce' and
'touched' wherever a global batch touches nearly every row, as at C3)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch.distributed as dist
    import bench
    from ncf_amd.engine import TrainEngine
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["allreduce", "touched"]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    shape, f, nl, gb = bench.CONFIGS[cfg]
    ds, train = bench.make_train_data(cfg)
    from ncf_amd.pipeline import EpochPipeline
    pipe = EpochPipeline(train, dev, gb, ds["item_num"], user_num=ds["user_num"], prefetch=False)
    rows = pipe.next_epoch(peek_eval_draw=False)
    res = {}
    for mode in modes:
        # zero1 at an emulated world over a one-rank group: the collectives in
        # their exact all-reduce forms (ncf_amd.distributed, NCF_DP_EMULATE)
        os.environ["NCF_DP_EMULATE"] = "1" if mode == "zero1" else "0"
        torch.manual_seed(0)
        model, _ = bench.build_model(cfg, ds["user_num"], ds["item_num"], dev)
        eng = TrainEngine(model, lr=1e-3, world_size=world, rank=0, process_group=dist.group.WORLD, dp_mode=mode)
        eng.set_epoch_stream(rows, gb, checked=True)
        eng.run(2 * eng.num_batches)
        torch.cuda.synchronize()
        k = 4 * eng.num_batches
        t0 = time.perf_counter()
        eng.run(k)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / k * 1e3
        kt = eng.time_kernels(20)
        res[mode] = {"ms_per_step_graph": ms, "launch_groups_ms": kt}
        if mode == "owner":  # the two all-to-alls' chunk per peer (bytes), the list slots
            P = eng._ow_plan
            res[mode]["owner"] = {"grad_chunk_bytes": 4 * int(P.send_floats), "param_chunk_bytes": 4 * int(P.param_floats),
                                  "max_u": int(P.max_u), "max_i": int(P.max_i),
                                  "lists_MB": int(P.lists_bytes) / 1e6}
        del eng, model
        torch.cuda.empty_cache()
    pipe.close()
    dist.destroy_process_group()
    print(json.dumps({"config": cfg, "world_emulated": world, "per_rank_batch": -(-gb // world), "modes": res}))


if __name__ == "__main__":
    main()
