"""src.utils.visualization (reference src/utils/visualization.py): the one helper
scripts/train_teacher.py calls, plot_training_metrics(run_histories, model_name,
output_path) -- mean +- std over runs per epoch, one panel per metric (matplotlib,
Agg backend).  Off the hot path."""
from pathlib import Path

import numpy as np


def plot_training_metrics(run_histories, model_name, output_path="results/figures/training_metrics.png",
                          metrics=("loss", "hr", "ndcg"), metric_labels=None):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    labels = metric_labels or {"loss": "Loss", "hr": "HR@10", "ndcg": "NDCG@10"}
    output_path = Path(output_path)
    output_path.parent.mkdir(parents=True, exist_ok=True)
    n = min(len(h) for h in run_histories)
    epochs = np.arange(1, n + 1)
    fig, axes = plt.subplots(len(metrics), 1, figsize=(10, 4 * len(metrics)), squeeze=False)
    for ax, m in zip(axes[:, 0], metrics):
        vals = np.array([[float(h[e][m]) for e in range(n)] for h in run_histories])
        mu, sd = vals.mean(0), vals.std(0)
        ax.plot(epochs, mu, label=model_name)
        ax.fill_between(epochs, mu - sd, mu + sd, alpha=0.2)
        ax.set_title(labels.get(m, m))
        ax.set_xlabel("Epoch")
        ax.set_ylabel(labels.get(m, m))
        ax.grid(True)
        ax.legend()
    fig.tight_layout()
    fig.savefig(output_path)
    plt.close(fig)
