#!/usr/bin/env python3
"""G11: the reference's NeuMF-pre chain, end to end, by running the REFERENCE itself
(build container only; /root/reference does not exist on the GPU box):

  scripts/pretrain.py --model GMF --epochs 2 --factor_num 8               -> GMF_8f_best.pth
  scripts/pretrain.py --model MLP --epochs 2 --factor_num 8 --num_layers 3 -> MLP_3l_8f_best.pth
  scripts/train_neumf.py --model NeuMF-pre --pretraining --epochs 2 --factor_num 8 --num_layers 3
      (loads both checkpoints through NCF.load_pretrain_weights, models.py:48-95, and
       trains with optim.SGD(lr * 10), train_neumf.py:62-90)

each run seeded with np.random.seed(0) / torch.manual_seed(0) first, on the
ml-100k-shaped synthetic files of ncf_amd.synthetic (seed 0) -- the G7 setup.
Stored: the stdout lines of each run that carry results (epoch lines, parameter
counts, result blocks), the checkpoint file names written, and a sha256 of each
checkpoint's tensors.  Only the reference's outputs are stored, no source text.
"""
import contextlib
import hashlib
import io
import os
import runpy
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
KEEP = ("Epoch ", "HR@", "NDCG@", "Parameters:", "Model parameters:", "Best Result", "Loading pretrained",
        "Pretrained weights loaded", "Pretraining:")

RUNS = [
    ("gmf", "scripts/pretrain.py", ["--model", "GMF", "--epochs", "2", "--factor_num", "8"]),
    ("mlp", "scripts/pretrain.py", ["--model", "MLP", "--epochs", "2", "--factor_num", "8", "--num_layers", "3"]),
    ("neumf_pre", "scripts/train_neumf.py", ["--model", "NeuMF-pre", "--pretraining", "--epochs", "2",
                                             "--factor_num", "8", "--num_layers", "3"]),
]


def sha(state):
    h = hashlib.sha256()
    for k, v in state.items():
        h.update(k.encode())
        h.update(np.ascontiguousarray(v.numpy()).tobytes())
    return h.hexdigest()


def main():
    work = tempfile.mkdtemp(prefix="ncf_ref_")
    dst = os.path.join(work, "ref")
    shutil.copytree(REF, dst, ignore=shutil.ignore_patterns(".git", "results"))
    for root, dirs, files in os.walk(dst):
        os.chmod(root, 0o755)
    here_cwd = os.getcwd()
    os.chdir(dst)
    sys.path.insert(0, dst)
    sys.path.insert(1, os.path.dirname(os.path.dirname(HERE)))
    import torch
    from ncf_amd import synthetic
    synthetic.write_reference_files(synthetic.make_dataset("ml-100k", seed=0), "data/processed")
    out = {}
    for tag, script, args in RUNS:
        before = set(os.listdir("results/models")) if os.path.isdir("results/models") else set()
        np.random.seed(0)
        torch.manual_seed(0)
        argv = sys.argv
        sys.argv = [os.path.basename(script)] + args
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            runpy.run_path(script, run_name="__main__")
        sys.argv = argv
        lines = [ln for ln in buf.getvalue().splitlines() if ln.startswith(KEEP)]
        out[f"{tag}_stdout"] = np.array(lines)
        new = sorted(set(os.listdir("results/models")) - before)
        out[f"{tag}_checkpoints"] = np.array(new)
        for f in new:
            out[f"{tag}::{f}::sha256"] = np.array(sha(torch.load(os.path.join("results/models", f),
                                                                 weights_only=True)))
        print(tag, lines, new)
    os.chdir(here_cwd)
    np.savez_compressed(os.path.join(HERE, "G11_pretrain_chain.npz"), **out)


if __name__ == "__main__":
    main()
