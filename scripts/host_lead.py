#!/usr/bin/env python3
"""Where the host stands against the device around epoch boundaries (C3 by default):
per epoch, the host wall time of next_epoch() (pipeline join + switch) and of
eng.run(steps of the epoch) (graph replays: enqueue only), beside the device time of
the same spans (events on the launch stream).  Host enqueue slower than the device
means the GPU idles at every boundary by the host's boundary work."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    shape, f, nl, gb = bench.CONFIGS[cfg]
    ds, train = bench.make_train_data(cfg)
    eng, model, pipe = bench.setup_engine(cfg, ds, train, 1, 0, dev, None, gb)
    eng.batches_done = 0
    bench.run_steps(eng, 2 * eng.num_batches, True)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream(dev)
    out = []
    for _ in range(epochs):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        h0 = time.perf_counter()
        ev[0].record(st)
        eng.next_epoch()
        h1 = time.perf_counter()
        ev[1].record(st)
        eng.run(eng.num_batches)
        eng.batches_done += eng.num_batches
        h2 = time.perf_counter()
        ev[2].record(st)
        # how far the device is behind when the host is done enqueueing
        lag_ms = None
        t_q = time.perf_counter()
        ev[2].synchronize()
        lag_ms = (time.perf_counter() - t_q) * 1e3
        out.append({"host_next_epoch_ms": (h1 - h0) * 1e3, "host_run_ms": (h2 - h1) * 1e3,
                    "dev_boundary_ms": ev[0].elapsed_time(ev[1]), "dev_run_ms": ev[1].elapsed_time(ev[2]),
                    "device_behind_host_ms": lag_ms,
                    "boundary_ms": pipe.stats["boundary_ms"][-1]})
    # free-running: no synchronize between epochs (the bench's timed loop); host and
    # device clocks share the base point of a drained stream
    torch.cuda.synchronize()
    base = torch.cuda.Event(enable_timing=True)
    base.record(st)
    base.synchronize()
    hb = time.perf_counter()
    marks = []
    for _ in range(epochs):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        h0 = time.perf_counter()
        e0.record(st)
        eng.next_epoch()
        h1 = time.perf_counter()
        e1.record(st)
        eng.run(eng.num_batches)
        eng.batches_done += eng.num_batches
        marks.append((h0, h1, e0, e1, list(pipe.stats["boundary_ms"][-1])))
    torch.cuda.synchronize()
    free = [{"host_enter_ms": (h0 - hb) * 1e3, "host_exit_ms": (h1 - hb) * 1e3,
             "dev_reach_ms": base.elapsed_time(e0), "dev_exit_ms": base.elapsed_time(e1), "boundary_ms": bm}
            for h0, h1, e0, e1, bm in marks]
    pipe.close()
    print(json.dumps({"config": cfg, "steps_per_epoch": eng.num_batches, "epochs": out, "free_running": free}))


if __name__ == "__main__":
    main()
