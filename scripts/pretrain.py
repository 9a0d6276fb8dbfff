#!/usr/bin/env python3
"""Pretrain GMF or MLP on MI355X -- CLI, prints and checkpoint names of the
reference scripts/pretrain.py (:112-171, :97-102), loop run by ncf_amd.Trainer.
Usage: python scripts/pretrain.py --model GMF --epochs 20
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.utils.data as data

sys.path.append(os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from src.ncf.models import NCF  # noqa: E402
from src.data.datasets import NCFData, load_all  # noqa: E402
from src.utils.config import config  # noqa: E402
from src.training import Trainer  # noqa: E402


def train_model(model_type, args, device):
    print(f"\nTraining {model_type} model...")
    train_data, test_data, user_num, item_num, train_mat = load_all()
    train_dataset = NCFData(train_data, item_num, train_mat, args.num_ng, True)
    test_dataset = NCFData(test_data, item_num, train_mat, 0, False)
    test_loader = data.DataLoader(test_dataset, batch_size=args.test_num_ng + 1, shuffle=False, num_workers=0)
    model = NCF(user_num, item_num, args.factor_num, args.num_layers, args.dropout, model_type).to(device)
    param_count = sum(p.numel() for p in model.parameters() if p.requires_grad)
    print(f"Model: {model_type}")
    print(f"Parameters: {param_count:,}")
    print(f"Factor num: {args.factor_num}")
    print(f"Layers: {args.num_layers}")
    trainer = Trainer(model, train_dataset, test_loader, batch_size=args.batch_size, lr=args.lr, top_k=args.top_k,
                      device=device)
    print(f"Training for {args.epochs} epochs...")
    fname = (f"{model_type}_{args.num_layers}l_{args.factor_num}f_best.pth" if model_type == "MLP"
             else f"{model_type}_{args.factor_num}f_best.pth")

    def save(m):
        if args.save:
            path = config.model_dir / fname
            torch.save(m.state_dict(), path)
            print(f"Saved best model to {path}")
    res = trainer.fit(args.epochs, model_type=model_type, save_fn=save)
    print("\nTraining completed!")
    print(f"Best HR@{args.top_k}: {res['best_hr']:.4f} at epoch {res['best_epoch']}")
    return res["best_hr"], res["best_ndcg"], param_count


def main():
    p = argparse.ArgumentParser(description="Train GMF or MLP model")
    p.add_argument("--model", type=str, required=True, choices=["GMF", "MLP"])
    p.add_argument("--epochs", type=int, default=config.epochs)
    p.add_argument("--lr", type=float, default=config.lr)
    p.add_argument("--dropout", type=float, default=config.dropout)
    p.add_argument("--batch_size", type=int, default=config.batch_size)
    p.add_argument("--factor_num", type=int, default=config.factor_num)
    p.add_argument("--num_layers", type=int, default=config.num_layers)
    p.add_argument("--num_ng", type=int, default=config.num_ng)
    p.add_argument("--test_num_ng", type=int, default=config.test_num_ng)
    p.add_argument("--top_k", type=int, default=config.top_k)
    p.add_argument("--save", action="store_true", default=True)
    p.add_argument("--gpu", type=str, default="0")
    p.add_argument("--seed", type=int, default=None)
    args = p.parse_args()
    if args.seed is not None:
        np.random.seed(args.seed)
        torch.manual_seed(args.seed)
    device = torch.device("cuda", int(args.gpu.split(",")[0]))
    hr, ndcg, n = train_model(args.model, args, device)
    print("\n--- RESULTS ---")
    print(f"Model: {args.model}")
    print(f"HR@{args.top_k}: {hr}")
    print(f"NDCG@{args.top_k}: {ndcg}")
    print(f"Parameters: {n}")
    print("--- END RESULTS ---")


if __name__ == "__main__":
    main()
