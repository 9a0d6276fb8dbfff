#!/usr/bin/env python3
"""Hash of the trained state after K graph-replayed steps of a bench config -- run it
under two library builds (NCF_HIP_LIB=<variant>) to check that a kernel change that
claims to keep the arithmetic gives bitwise the same parameters, moments and losses.
usage: r6_bitwise.py CONFIG STEPS"""
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from ncf_amd.engine import TrainEngine
    from ncf_amd.pipeline import EpochPipeline
    cfg = sys.argv[1] if len(sys.argv) > 1 else "stress"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    _, _, _, gb = bench.CONFIGS[cfg]
    ds, train = bench.make_train_data(cfg)
    pipe = EpochPipeline(train, dev, gb, ds["item_num"], user_num=ds["user_num"], prefetch=False)
    rows = pipe.next_epoch(peek_eval_draw=False)
    torch.manual_seed(0)
    model, _ = bench.build_model(cfg, ds["user_num"], ds["item_num"], dev)
    eng = TrainEngine(model, lr=1e-3)
    eng.set_epoch_stream(rows, gb, checked=True)
    eng.run(steps)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in (eng.flat, eng.exp_avg, eng.exp_avg_sq, eng.loss_hist):
        h.update(t.detach().cpu().numpy().tobytes())
    losses = eng.loss_hist[:steps].cpu().tolist()
    print(f"{cfg} steps={steps} lib={os.environ.get('NCF_HIP_LIB', '') or 'default'} sha={h.hexdigest()[:16]} "
          f"loss[0]={losses[0]:.8f} loss[-1]={losses[-1]:.8f}")
    pipe.close()


if __name__ == "__main__":
    main()
