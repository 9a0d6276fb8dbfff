#!/usr/bin/env python3
"""G8: golden vectors of the distillation path (config C5), produced by running
the REFERENCE's src/distillation classes in this build container
(``python tests/golden/make_golden_kd.py``; /root/reference is not on the GPU
box).  Imports the reference the same way as make_golden.py (a scratch copy,
since its config singleton needs a writable cwd).  Stored: inputs, the seeded
initial teacher/student/adapter weights, and the reference's outputs -- loss and
student gradients of one step, then per-step losses and the student's parameters
after T Adam steps (scripts/train_student.py:131,148-158).  No reference source.

G9_student_loop.npz: the loop of scripts/train_student.py:75-168 (seeded, 1 epoch,
ml-100k-shaped synthetic files from ncf_amd.synthetic, teacher NCF(16,3,NeuMF-end)
initialised with torch seed 123 and loaded like :84-89, student NCF(8,2,MLP)) with
the reference's NCFData, DataLoader (num_workers=4 as :80), load_all, metrics and
distillation classes.  The script itself cannot be run here: it imports
tensorboardX (not installed) and UnifiedDistillation (empty unified.py), so the
loop is restated line by line around the reference's own objects; the per-epoch
stdout line (:168 format) is stored.

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
    g9_student_loop(NCF, D)


def g9_student_loop(NCF, D):
    import contextlib
    import io
    import time
    import torch
    import torch.utils.data as data
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from ncf_amd import synthetic
    from src.data.datasets import NCFData, load_all
    from src.training.metrics import metrics
    synthetic.write_reference_files(synthetic.make_dataset("ml-100k", seed=0), "data/processed")
    out = {}
    for strat in ("response", "feature"):
        np.random.seed(0)
        torch.manual_seed(0)
        train_data, test_data, user_num, item_num, train_mat = load_all()                  # :75
        train_dataset = NCFData(train_data, item_num, train_mat, 4, True)                  # :77
        test_dataset = NCFData(test_data, item_num, train_mat, 0, False)
        train_loader = data.DataLoader(train_dataset, batch_size=256, shuffle=True, num_workers=4)  # :80
        test_loader = data.DataLoader(test_dataset, batch_size=100, shuffle=False, num_workers=0)
        gen_state = torch.get_rng_state()
        torch.manual_seed(123)                       # the teacher checkpoint's weights
        teacher_sd = NCF(user_num, item_num, 16, 3, 0.0, "NeuMF-end").state_dict()
        torch.set_rng_state(gen_state)
        teacher = NCF(user_num, item_num, 16, 3, 0.0, "NeuMF-end")                       # :86
        teacher.load_state_dict(teacher_sd)                                                 # :87
        teacher.eval()
        student = NCF(user_num, item_num, 8, 2, 0.0, "MLP")                                 # :92
        with contextlib.redirect_stdout(io.StringIO()):
            if strat == "response":
                dist = D.ResponseDistillation(teacher, student, temperature=2.0, alpha=0.5)  # :96-102
            else:
                dist = D.FeatureDistillation(teacher, student, temperature=2.0, alpha=0.5, beta=0.3)
        optimizer = torch.optim.Adam(student.parameters(), lr=1e-3)                        # :131
        lines = []
        for epoch in range(1):                                                              # :141-168
            dist.train()
            start_time = time.time()
            train_loader.dataset.ng_sample()
            total_loss, num_batches = 0, 0
            with contextlib.redirect_stdout(io.StringIO()):
                for user, item, label in train_loader:
                    label = label.float()
                    optimizer.zero_grad()
                    loss = dist(user, item, label)
                    loss.backward()
                    optimizer.step()
                    total_loss += loss.item()
                    num_batches += 1
            avg_loss = total_loss / num_batches
            student.eval()
            with torch.no_grad():
                HR, NDCG = metrics(student, test_loader, 10)
            hr, ndcg = np.mean(HR), np.mean(NDCG)
            el = time.time() - start_time
            lines.append(f"{epoch:03d} - Loss: {avg_loss:.6f}, HR: {hr:.3f}, NDCG: {ndcg:.3f}, "
                         f"Time: {time.strftime('%H:%M:%S', time.gmtime(el))}")
        out[f"{strat}_stdout"] = np.array(lines)
        out[f"{strat}_avg_loss"] = np.float64(avg_loss)
        print(strat, lines)
    np.savez_compressed(os.path.join(HERE, "G9_student_loop.npz"), **out)


if __name__ == "__main__":
    main()
