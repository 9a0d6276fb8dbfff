#!/usr/bin/env python3
"""G8: golden vectors of the distillation path (config C5), produced by running
the REFERENCE's src/distillation classes in this build container
(``python tests/golden/make_golden_kd.py``; /root/reference is not on the GPU
box).  Imports the reference the same way as make_golden.py (a scratch copy,
since its config singleton needs a writable cwd).  Stored: inputs, the seeded
initial teacher/student/adapter weights, and the reference's outputs -- loss and
student gradients of one step, then per-step losses and the student's parameters
after T Adam steps (scripts/train_student.py:131,148-158).  No reference source.

Cases (teacher -> student):
  c5   NCF(16,3,NeuMF-end) -> NCF(8,2,MLP)        SURVEY C5
  cli  NCF(32,2,NeuMF-end) -> NCF(16,1,NeuMF-end) train_student.py defaults
  same NCF(8,2,GMF)        -> NCF(8,2,GMF)        equal widths: identity keys and
                                                  matched tower features (oracle only)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _import_reference  # noqa: E402

U, I, B, T = 50, 80, 256, 5
CASES = {"c5": ((16, 3, "NeuMF-end"), (8, 2, "MLP")),
         "cli": ((32, 2, "NeuMF-end"), (16, 1, "NeuMF-end")),
         "same": ((8, 2, "GMF"), (8, 2, "GMF"))}
STRATS = ["response", "feature", "attention"]


def main():
    NCF, _, _ = _import_reference()
    import torch
    import src.distillation as D
    cls = {"response": D.ResponseDistillation, "feature": D.FeatureDistillation,
           "attention": D.AttentionDistillation}
    rng = np.random.default_rng(8)
    users = rng.integers(0, U, (T, B))
    items = rng.integers(0, I, (T, B))
    labels = (rng.random((T, B)) < 0.2).astype(np.float32)
    out = {"users": users, "items": items, "labels": labels}
    for case, (tc, sc) in CASES.items():
        for st in STRATS:
            tag = f"{case}_{st}"
            torch.manual_seed(7)
            teacher = NCF(U, I, tc[0], tc[1], 0.0, tc[2])
            student = NCF(U, I, sc[0], sc[1], 0.0, sc[2])
            kw = {"temperature": 2.0, "alpha": 0.5}
            if st == "feature":
                kw["beta"] = 0.3
            if st == "attention":
                kw["gamma"] = 0.2
            dist = cls[st](teacher, student, **kw)
            for k, v in teacher.state_dict().items():
                out[f"{tag}::teacher::{k}"] = v.numpy().copy()
            for k, v in student.state_dict().items():
                out[f"{tag}::student0::{k}"] = v.numpy().copy()
            if st == "feature":
                for k, v in dist.adaptation_layers.state_dict().items():
                    out[f"{tag}::adapter::{k}"] = v.numpy().copy()
            opt = torch.optim.Adam(student.parameters(), lr=1e-3)
            losses = []
            for s in range(T):
                u = torch.from_numpy(users[s])
                i = torch.from_numpy(items[s])
                y = torch.from_numpy(labels[s])
                opt.zero_grad()
                loss = dist(u, i, y)
                loss.backward()
                if s == 0:
                    out[f"{tag}::loss0"] = np.float64(loss.item())
                    for k, p in student.named_parameters():
                        if p.grad is not None:
                            out[f"{tag}::grad0::{k}"] = p.grad.numpy().copy()
                opt.step()
                losses.append(loss.item())
            out[f"{tag}::losses"] = np.array(losses)
            for k, v in student.state_dict().items():
                out[f"{tag}::student_t{T}::{k}"] = v.numpy().copy()
    np.savez_compressed(os.path.join(HERE, "G8_distill.npz"), **out)
    print("wrote G8_distill.npz", len(out), "arrays")


if __name__ == "__main__":
    main()
