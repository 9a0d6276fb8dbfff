#!/usr/bin/env python3
"""Distil a student from a trained teacher on MI355X -- same CLI, defaults,
stdout lines and checkpoint names as the reference scripts/train_student.py
(:22-62, :168, :179-183).  Every step is the fused device plan of the chosen
distillation module (ncf_amd.distill): teacher logits once per epoch stream,
ncf_train_step_kd + ncf_kd_feature_step, reduce + Adam, hipGraph replay.
'unified' uses this build's UnifiedDistillation (the reference file is empty)."""
import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.utils.data as data

sys.path.append(os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from src.ncf.models import NCF  # noqa: E402
from src.utils.config import config  # noqa: E402
from src.data.datasets import load_all, NCFData  # noqa: E402
from src.training import Trainer  # noqa: E402
from src.distillation import (  # noqa: E402
    ResponseDistillation,
    FeatureDistillation,
    AttentionDistillation,
    UnifiedDistillation,
)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lr", type=float, default=config.lr, help="learning rate")
    p.add_argument("--dropout", type=float, default=config.dropout, help="dropout rate")
    p.add_argument("--batch_size", type=int, default=config.batch_size, help="batch size for training")
    p.add_argument("--epochs", type=int, default=config.epochs, help="training epochs")
    p.add_argument("--top_k", type=int, default=config.top_k, help="compute metrics@top_k")
    p.add_argument("--factor_num", type=int, default=config.factor_num // 2,
                   help="predictive factors numbers in the student model")
    p.add_argument("--num_layers", type=int, default=config.num_layers - 1, help="number of layers in MLP for student")
    p.add_argument("--num_ng", type=int, default=config.num_ng, help="sample negative items for training")
    p.add_argument("--test_num_ng", type=int, default=config.test_num_ng, help="sample part of negative items for testing")
    p.add_argument("--out", action="store_true", default=True, help="save model or not")
    p.add_argument("--gpu", type=str, default="0", help="gpu card ID")
    p.add_argument("--teacher_model", type=str, default=config.model_type,
                   choices=["GMF", "MLP", "NeuMF-end", "NeuMF-pre"], help="Teacher model type")
    p.add_argument("--student_model", type=str, default="NeuMF-end", choices=["GMF", "MLP", "NeuMF-end"],
                   help="Student model type")
    p.add_argument("--temperature", type=float, default=config.temperature, help="Temperature for distillation")
    p.add_argument("--alpha", type=float, default=config.alpha, help="Weight for BCE vs KD loss")
    p.add_argument("--beta", type=float, default=0.3, help="Weight for feature distillation loss")
    p.add_argument("--gamma", type=float, default=0.2, help="Weight for attention distillation loss")
    p.add_argument("--distillation", type=str, default="response",
                   choices=["response", "feature", "attention", "unified"], help="Distillation strategy to use")
    p.add_argument("--seed", type=int, default=None, help="seed numpy + torch (the reference never seeds)")
    args = p.parse_args()
    if args.seed is not None:
        np.random.seed(args.seed)
        torch.manual_seed(args.seed)
    if not torch.cuda.is_available():
        raise SystemExit("This build trains on a HIP device (MI355X); no GPU visible")
    device = torch.device("cuda", int(args.gpu.split(",")[0]))
    print(" Using GPU:", torch.cuda.get_device_name(device))

    train_data, test_data, user_num, item_num, train_mat = load_all()
    train_dataset = NCFData(train_data, item_num, train_mat, args.num_ng, True)
    test_dataset = NCFData(test_data, item_num, train_mat, 0, False)
    test_loader = data.DataLoader(test_dataset, batch_size=args.test_num_ng + 1, shuffle=False, num_workers=0)

    teacher_path = config.model_dir / f"teacher_{args.teacher_model}_best.pth"
    assert os.path.exists(teacher_path), f"Lack of teacher model: {teacher_path}"
    teacher_model = NCF(user_num, item_num, args.factor_num * 2, args.num_layers + 1, args.dropout, args.teacher_model)
    teacher_model.load_state_dict(torch.load(teacher_path, map_location="cpu", weights_only=True))
    teacher_model.to(device)
    teacher_model.eval()
    student_model = NCF(user_num, item_num, args.factor_num, args.num_layers, args.dropout, args.student_model)
    student_model.to(device)

    kw = {"temperature": args.temperature, "alpha": args.alpha}
    if args.distillation == "response":
        distillation = ResponseDistillation(teacher_model, student_model, **kw)
    elif args.distillation == "feature":
        distillation = FeatureDistillation(teacher_model, student_model, beta=args.beta, **kw)
    elif args.distillation == "attention":
        distillation = AttentionDistillation(teacher_model, student_model, gamma=args.gamma, **kw)
    else:
        distillation = UnifiedDistillation(teacher_model, student_model, beta=args.beta, gamma=args.gamma, **kw)
    distillation.to(device)

    trainer = Trainer(student_model, train_dataset, test_loader, batch_size=args.batch_size, lr=args.lr,
                      top_k=args.top_k, device=device, distill=distillation)
    best_hr, best_ndcg, best_epoch = 0, 0, 0
    for epoch in range(args.epochs):
        distillation.train()
        start_time = time.time()
        avg_loss = trainer.train_epoch()
        student_model.eval()
        HR, NDCG = trainer.evaluate(args.top_k)
        hr, ndcg = np.mean(HR), np.mean(NDCG)
        elapsed_time = time.time() - start_time
        print(f"{epoch:03d} - Loss: {avg_loss:.6f}, HR: {hr:.3f}, NDCG: {ndcg:.3f}, "
              f"Time: {time.strftime('%H:%M:%S', time.gmtime(elapsed_time))}")
        if hr > best_hr:
            best_hr, best_ndcg, best_epoch = hr, ndcg, epoch
            if args.out:
                path = config.model_dir / f"student_{args.student_model}_best.pth"
                torch.save(student_model.state_dict(), path)
                print(f"Saved best model to {path}")
    print(f"End. Best epoch {best_epoch:03d}: HR = {best_hr:.3f}, NDCG = {best_ndcg:.3f}")


if __name__ == "__main__":
    main()
