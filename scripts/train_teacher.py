#!/usr/bin/env python3
"""Train the distillation teacher on MI355X -- same CLI, defaults, stdout lines
and checkpoint name as the reference scripts/train_teacher.py (:112-145, :89,
:98-100): NCF(config.user_num, config.item_num, factor_num, num_layers) trained
with BCE + Adam, best-HR checkpoint results/models/teacher_{model}_best.pth.
The loop runs on ncf_amd.Trainer (fused HIP step, hipGraph replay).  TensorBoard
scalars are written when tensorboardX is importable (it is optional here)."""
import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.utils.data as data

sys.path.append(os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from src.ncf.models import NCF  # noqa: E402
from src.data.datasets import NCFData, load_all  # noqa: E402
from src.utils.config import config  # noqa: E402
from src.training import Trainer  # noqa: E402
from src.utils.visualization import plot_training_metrics  # noqa: E402


def _writer(log_dir):
    try:
        from tensorboardX import SummaryWriter
    except ImportError:
        return None
    return SummaryWriter(log_dir=log_dir)


def train_teacher(model_type, user_num, item_num, train_mat, device, args):
    train_data, test_data, _, _, _ = load_all()
    train_dataset = NCFData(train_data, item_num, train_mat, args.num_ng, True)
    test_dataset = NCFData(test_data, item_num, train_mat, 0, False)
    test_loader = data.DataLoader(test_dataset, batch_size=args.test_num_ng + 1, shuffle=False, num_workers=0)
    model = NCF(user_num, item_num, args.factor_num, args.num_layers, args.dropout, model_type)
    if model_type == "NeuMF-pre":
        gmf_path = config.model_dir / f"GMF_{args.factor_num}f_best.pth"
        mlp_path = config.model_dir / f"MLP_{args.num_layers}l_{args.factor_num}f_best.pth"
        if gmf_path.exists() and mlp_path.exists():
            model.load_pretrain_weights(torch.load(gmf_path, map_location="cpu", weights_only=True),
                                        torch.load(mlp_path, map_location="cpu", weights_only=True))
            print("Loaded pretrained GMF and MLP weights for NeuMF-pre")
        else:
            raise FileNotFoundError("Pretrained GMF or MLP weights not found")
    model.to(device)
    trainer = Trainer(model, train_dataset, test_loader, batch_size=args.batch_size, lr=args.lr,
                      top_k=args.top_k, device=device)
    writer = _writer(config.log_dir / f"teacher_{model_type}_{time.strftime('%Y%m%d_%H%M%S')}")
    best_hr = best_loss = best_ndcg = best_epoch = 0
    history = []
    for epoch in range(args.epochs):
        model.train()
        start_time = time.time()
        avg_loss = trainer.train_epoch()
        model.eval()
        HR, NDCG = trainer.evaluate(args.top_k)
        hr, ndcg = np.mean(HR), np.mean(NDCG)
        elapsed_time = time.time() - start_time
        if writer is not None:
            writer.add_scalar("Loss/Train", avg_loss, epoch)
            writer.add_scalar(f"HR@{args.top_k}", hr, epoch)
            writer.add_scalar(f"NDCG@{args.top_k}", ndcg, epoch)
        print(f"Epoch {epoch + 1:03d}: Loss={avg_loss:.4f}, HR={hr:.3f}, NDCG={ndcg:.3f}, "
              f"Time={time.strftime('%H:%M:%S', time.gmtime(elapsed_time))}")
        history.append({"epoch": epoch + 1, "loss": avg_loss, "hr": hr, "ndcg": ndcg})
        if hr > best_hr:
            best_hr, best_ndcg, best_loss, best_epoch = hr, ndcg, avg_loss, epoch
            if args.out:
                path = config.model_dir / f"teacher_{model_type}_best.pth"
                torch.save(model.state_dict(), path)
                print(f"Saved best model to {path}")
    plot_training_metrics(run_histories=[history], model_name=f"Teacher_{model_type}",
                          output_path=config.figure_dir / f"teacher_{model_type}_metrics.png")
    if writer is not None:
        writer.close()
    return best_loss, best_hr, best_ndcg, best_epoch


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lr", type=float, default=config.lr, help="learning rate")
    p.add_argument("--dropout", type=float, default=config.dropout, help="dropout rate")
    p.add_argument("--batch_size", type=int, default=config.batch_size, help="batch size")
    p.add_argument("--epochs", type=int, default=config.epochs, help="training epochs")
    p.add_argument("--top_k", type=int, default=config.top_k, help="compute metrics@top_k")
    p.add_argument("--factor_num", type=int, default=config.factor_num, help="predictive factors")
    p.add_argument("--num_layers", type=int, default=config.num_layers, help="number of layers in MLP")
    p.add_argument("--num_ng", type=int, default=config.num_ng, help="sample negative items for training")
    p.add_argument("--test_num_ng", type=int, default=config.test_num_ng, help="sample negative items for testing")
    p.add_argument("--out", action="store_true", default=True, help="save model")
    p.add_argument("--gpu", type=str, default="0", help="gpu card ID")
    p.add_argument("--model", type=str, default="NeuMF-end", choices=["NeuMF-end", "NeuMF-pre"], help="model type")
    p.add_argument("--seed", type=int, default=None, help="seed numpy + torch (the reference never seeds)")
    args = p.parse_args()
    if args.seed is not None:
        np.random.seed(args.seed)
        torch.manual_seed(args.seed)
    if not torch.cuda.is_available():
        raise SystemExit("This build trains on a HIP device (MI355X); no GPU visible")
    device = torch.device("cuda", int(args.gpu.split(",")[0]))
    print(f"Using GPU: {torch.cuda.get_device_name(device)}")
    best_loss, best_hr, best_ndcg, best_epoch = train_teacher(
        model_type=args.model, user_num=config.user_num, item_num=config.item_num,
        train_mat=load_all()[4], device=device, args=args)
    print(f"Best Epoch {best_epoch:03d}: Loss={best_loss:.4f}, HR={best_hr:.3f}, NDCG={best_ndcg:.3f}")


if __name__ == "__main__":
    main()
