#!/usr/bin/env python3
"""Train NeuMF on MI355X -- same CLI, defaults, stdout protocol and checkpoint
names as the reference scripts/train_neumf.py (:169-219, :131, :146-157), with
the loop run by ncf_amd.Trainer (fused HIP step, hipGraph replay).
Usage: python scripts/train_neumf.py --model NeuMF-end --num_layers 3
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


def count_parameters(model):
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def find_pretrained_model(model_type, num_layers, factor_num):
    if model_type == "GMF":
        filename = f"GMF_{factor_num}f_best.pth"
    elif model_type == "MLP":
        filename = f"MLP_{num_layers}l_{factor_num}f_best.pth"
    else:
        return None
    model_path = config.model_dir / filename
    return model_path if model_path.exists() else None


def train_neumf(args, device):
    print(f"\nTraining {args.model} with {args.num_layers} layers...")
    print(f"Pretraining: {'Yes' if args.pretraining else 'No'}")
    train_data, test_data, user_num, item_num, train_mat = load_all()
    print(f"Dataset: {user_num} users, {item_num} items")
    train_dataset = NCFData(train_data, item_num, train_mat, args.num_ng, True)
    test_dataset = NCFData(test_data, item_num, train_mat, 0, False)
    test_loader = data.DataLoader(test_dataset, batch_size=args.test_num_ng + 1, shuffle=False, num_workers=0)
    model = NCF(user_num, item_num, args.factor_num, args.num_layers, args.dropout, args.model)
    if args.pretraining:
        gmf_path = find_pretrained_model("GMF", None, args.factor_num)
        mlp_path = find_pretrained_model("MLP", args.num_layers, args.factor_num)
        if gmf_path and mlp_path and gmf_path.exists() and mlp_path.exists():
            print("Loading pretrained weights...")
            gmf_state = torch.load(gmf_path, map_location="cpu", weights_only=True)
            mlp_state = torch.load(mlp_path, map_location="cpu", weights_only=True)
            model.load_pretrain_weights(gmf_state, mlp_state)
            print("Pretrained weights loaded successfully")
        else:
            print("Warning: Pretrained weights not found!")
            print(f"GMF path: {gmf_path} (exists: {gmf_path and gmf_path.exists()})")
            print(f"MLP path: {mlp_path} (exists: {mlp_path and mlp_path.exists()})")
            print("Training without pretraining...")
            args.pretraining = False
    model.to(device)
    param_count = count_parameters(model)
    print(f"Model parameters: {param_count:,}")
    opt, lr = ("sgd", args.lr * 10) if args.pretraining else ("adam", args.lr)
    trainer = Trainer(model, train_dataset, test_loader, batch_size=args.batch_size, lr=lr, optimizer=opt,
                      top_k=args.top_k, device=device)
    print(f"Training for {args.epochs} epochs...")
    suffix = "pre" if args.pretraining else "end"
    fname = f"NeuMF_{suffix}_{args.num_layers}l_{args.factor_num}f_best.pth"

    def save(m):
        if args.save:
            torch.save(m.state_dict(), config.model_dir / fname)
            print(f"Saved best model: {fname}")
    res = trainer.fit(args.epochs, model_type=args.model, pretraining=args.pretraining, save_fn=save)
    best_hr, best_ndcg, best_epoch = res["best_hr"], res["best_ndcg"], res["best_epoch"]
    print("\nTraining completed!")
    print(f"Best Result: Epoch {best_epoch:03d}: HR={best_hr:.3f}, NDCG={best_ndcg:.3f}")
    print("\n--- RESULTS ---")
    print(f"Model: {args.model}")
    print(f"Layers: {args.num_layers}")
    print(f"Pretraining: {args.pretraining}")
    print(f"HR@{args.top_k}: {best_hr}")
    print(f"NDCG@{args.top_k}: {best_ndcg}")
    print(f"Parameters: {param_count}")
    print("--- END RESULTS ---")
    return res


def main():
    p = argparse.ArgumentParser(description="Train NeuMF model")
    p.add_argument("--model", type=str, default="NeuMF-end", choices=["NeuMF-end", "NeuMF-pre"])
    p.add_argument("--epochs", type=int, default=config.epochs)
    p.add_argument("--factor_num", type=int, default=config.factor_num)
    p.add_argument("--num_layers", type=int, default=config.num_layers)
    p.add_argument("--pretraining", action="store_true")
    p.add_argument("--lr", type=float, default=config.lr)
    p.add_argument("--batch_size", type=int, default=config.batch_size)
    p.add_argument("--dropout", type=float, default=config.dropout)
    p.add_argument("--num_ng", type=int, default=config.num_ng)
    p.add_argument("--test_num_ng", type=int, default=config.test_num_ng)
    p.add_argument("--top_k", type=int, default=config.top_k)
    p.add_argument("--save", action="store_true", default=True)
    p.add_argument("--gpu", type=str, default="0")
    p.add_argument("--seed", type=int, default=None, help="seed numpy + torch (the reference never seeds)")
    args = p.parse_args()
    if args.seed is not None:
        np.random.seed(args.seed)
        torch.manual_seed(args.seed)
    if not torch.cuda.is_available():
        raise SystemExit("This build trains on a HIP device (MI355X); no GPU visible")
    device = torch.device("cuda", int(args.gpu.split(",")[0]))
    print(f"Using GPU: {torch.cuda.get_device_name(device)}")
    result = train_neumf(args, device)
    print("\nFinal Results:")
    print(f"Model: {result['model_type']}")
    print(f"Layers: {result['num_layers']}")
    print(f"Pretraining: {result['pretraining']}")
    print(f"HR@{args.top_k}: {result['best_hr']:.4f}")
    print(f"NDCG@{args.top_k}: {result['best_ndcg']:.4f}")
    print(f"Parameters: {result['parameters']:,}")


if __name__ == "__main__":
    main()
