"""YAML-backed configuration singleton (reference src/utils/config.py:4-65).

Same keys, defaults and attribute names.  Like the reference it reads
``configs/experiments/neumf.yaml`` relative to the working directory and
creates ``results/{logs,models,figures}``; when that file is absent it falls
back to the copy shipped with this repository (the reference raises
FileNotFoundError there).  ``NCF_CONFIG`` overrides the path.
"""
from __future__ import annotations

import os
from pathlib import Path

import yaml

_PKG_DEFAULT = Path(__file__).resolve().parent.parent / "configs" / "experiments" / "neumf.yaml"


class Config:
    def __init__(self, config_path="configs/experiments/neumf.yaml"):
        self.config_path = Path(os.environ.get("NCF_CONFIG", config_path))
        if not self.config_path.exists() and _PKG_DEFAULT.exists():
            self.config_path = _PKG_DEFAULT
        self._load_config()
        self._set_defaults()
        self._create_directories()

    def _load_config(self):
        if not self.config_path.exists():
            raise FileNotFoundError(f"Config file not found: {self.config_path}")
        with open(self.config_path, "r") as f:
            self._config = yaml.safe_load(f) or {}

    def _set_defaults(self):
        c = self._config
        d, m, t, di, o = (c.get(k, {}) or {} for k in ("data", "model", "training", "distillation", "output"))
        self.raw_data = Path(d.get("raw_data", "data/raw/u.data"))
        self.train_rating = Path(d.get("train_rating", "data/processed/u.train.rating"))
        self.test_rating = Path(d.get("test_rating", "data/processed/u.test.rating"))
        self.test_negative = Path(d.get("test_negative", "data/processed/u.test.negative"))
        self.user_num = m.get("user_num", 943)
        self.item_num = m.get("item_num", 1682)
        self.factor_num = m.get("factor_num", 32)
        self.num_layers = m.get("num_layers", 3)
        self.dropout = m.get("dropout", 0.0)
        self.model_type = m.get("type", "NeuMF-end")
        self.batch_size = t.get("batch_size", 256)
        self.epochs = t.get("epochs", 20)
        self.lr = t.get("lr", 0.001)
        self.num_ng = t.get("num_ng", 4)
        self.test_num_ng = t.get("test_num_ng", 99)
        self.top_k = t.get("top_k", 10)
        self.temperature = di.get("temperature", 2.0)
        self.alpha = di.get("alpha", 0.5)
        self.output_dir = Path(o.get("dir", "results"))
        self.log_dir = self.output_dir / "logs"
        self.model_dir = self.output_dir / "models"
        self.figure_dir = self.output_dir / "figures"

    def _create_directories(self):
        for p in (self.output_dir, self.log_dir, self.model_dir, self.figure_dir):
            p.mkdir(parents=True, exist_ok=True)

    def get(self, key, default=None):
        return getattr(self, key, default)


config = Config()
