"""Temporal leave-one-out preprocessing (reference src/data/preprocessing.py:10-265,
scripts/preprocess.py): raw ``u.data`` (tab-separated user, item, rating,
timestamp) -> ``u.train.rating``, ``u.test.rating``, ``u.test.negative``.

Off the training hot path (a one-off, CPU).  Same class, file names, formats,
random-number consumption and split rules as the reference, without its per-row
``iterrows`` loops:
  * rows sorted with the same pandas calls (``sort_values(['user_id',
    'timestamp'])`` then, per user, ``sort_values('timestamp')``), so ties are
    broken exactly as the reference breaks them;
  * per user, all but the last interaction to train and the last to test; users
    with a single interaction go to train only (:59-83);
  * num_items = max train item + 1 (:183-201); test negatives drawn with the
    NumPy global legacy generator one ``randint(num_items)`` at a time, rejected
    against the user's train items and test item, at most 10x attempts, written
    sorted (:92-135).
"""
from __future__ import annotations

import json
import logging
import pickle
from datetime import datetime
from pathlib import Path

import numpy as np
import pandas as pd


def _logger(name):
    lg = logging.getLogger(name)
    lg.setLevel(logging.INFO)
    lg.handlers = []
    h = logging.StreamHandler()
    h.setFormatter(logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s"))
    lg.addHandler(h)
    Path("results/logs").mkdir(parents=True, exist_ok=True)
    f = logging.FileHandler(f"results/logs/{name}_{datetime.now().strftime('%Y%m%d_%H%M%S')}.log")
    f.setFormatter(logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s"))
    lg.addHandler(f)
    lg.propagate = False
    return lg


class LeaveOneOutPreprocessor:
    def __init__(self, raw_path="data/raw/u.data", processed_dir="data/processed", num_negatives=99):
        self.raw_path = Path(raw_path)
        self.processed_dir = Path(processed_dir)
        self.num_negatives = num_negatives
        self.logger = _logger("preprocessing")
        self.results = {}
        self.train_file = self.processed_dir / "u.train.rating"
        self.test_rating_file = self.processed_dir / "u.test.rating"
        self.test_negative_file = self.processed_dir / "u.test.negative"
        self.processed_dir.mkdir(parents=True, exist_ok=True)

    def load_and_prepare_data(self):
        df = pd.read_csv(self.raw_path, sep="\t", names=["user_id", "item_id", "rating", "timestamp"],
                         dtype={"user_id": int, "item_id": int, "rating": int, "timestamp": int})
        self.logger.info(f"Loaded {len(df):,} interactions")
        df_sorted = df.sort_values(["user_id", "timestamp"]).reset_index(drop=True)
        return df_sorted[["user_id", "item_id", "timestamp"]].copy()

    def temporal_split(self, df):
        train_parts, test_rows = [], []
        for _, g in df.groupby("user_id"):
            ui = g.sort_values("timestamp")[["user_id", "item_id"]].to_numpy(dtype=np.int64)
            if len(ui) < 2:
                train_parts.append(ui)
                continue
            train_parts.append(ui[:-1])
            test_rows.append(ui[-1])
        train = np.concatenate(train_parts) if train_parts else np.zeros((0, 2), np.int64)
        test = np.stack(test_rows) if test_rows else np.zeros((0, 2), np.int64)
        self.logger.info(f"Training interactions: {len(train):,}")
        self.logger.info(f"Test interactions: {len(test):,}")
        return train, test

    def generate_test_negatives(self, train_data, test_data, num_items):
        seen = {}
        for u, i in train_data:
            seen.setdefault(int(u), set()).add(int(i))
        for u, i in test_data:
            seen.setdefault(int(u), set()).add(int(i))
        lines = []
        max_attempts = self.num_negatives * 10
        for u, pos in test_data:
            u, pos = int(u), int(pos)
            items = seen.get(u, set())
            neg = set()
            attempts = 0
            while len(neg) < self.num_negatives and attempts < max_attempts:
                j = np.random.randint(num_items)
                if j not in items:
                    neg.add(j)
                attempts += 1
            if len(neg) < self.num_negatives:
                self.logger.warning(f"Could only generate {len(neg)} negatives for user {u}")
            lines.append(f"({u},{pos})\t" + "\t".join(map(str, sorted(neg))))
        return lines

    def save_splits(self, train_data, test_data, test_negatives):
        pd.DataFrame(train_data, columns=["user_id", "item_id"]).to_csv(self.train_file, sep="\t", index=False,
                                                                         header=False)
        pd.DataFrame(test_data, columns=["user_id", "item_id"]).to_csv(self.test_rating_file, sep="\t", index=False,
                                                                        header=False)
        with open(self.test_negative_file, "w") as f:
            f.write("\n".join(test_negatives))

    def verify_split(self, train_data, test_data):
        tr = {(int(u), int(i)) for u, i in train_data}
        leak = tr.intersection((int(u), int(i)) for u, i in test_data)
        if leak:
            self.logger.error(f" DATA LEAKAGE DETECTED: {len(leak)} interactions appear in both train and test!")
            raise RuntimeError("Data leakage detected in train/test split!")

    def build_interaction_matrix(self, train_data):
        num_users = int(train_data[:, 0].max()) + 1
        num_items = int(train_data[:, 1].max()) + 1
        return None, num_users, num_items

    def save_results(self):
        out = Path("results") / "reports"
        out.mkdir(parents=True, exist_ok=True)
        name = f"preprocessing_{datetime.now().strftime('%Y%m%d_%H%M%S')}"
        with open(out / f"{name}_results.json", "w") as f:
            json.dump(self.results, f, indent=2)
        with open(out / f"{name}_results.pkl", "wb") as f:
            pickle.dump(self.results, f)

    def run(self):
        df = self.load_and_prepare_data()
        train, test = self.temporal_split(df)
        _, num_users, num_items = self.build_interaction_matrix(train)
        negs = self.generate_test_negatives(train, test, num_items)
        self.verify_split(train, test)
        self.save_splits(train, test, negs)
        self.results["preprocessing"] = {
            "num_users": int(num_users), "num_items": int(num_items),
            "total_original_interactions": int(len(df)), "train_interactions": int(len(train)),
            "test_interactions": int(len(test)), "users_with_test": int(len(test)),
            "test_coverage": float(len(test) / num_users * 100),
            "sparsity": float(1 - (len(train) / (num_users * num_items))),
            "split_method": "temporal_leave_one_out"}
        self.save_results()
        self.logger.info(f"   Users: {num_users:,}  Items: {num_items:,}  Train: {len(train):,}  Test: {len(test):,}")
