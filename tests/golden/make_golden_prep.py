#!/usr/bin/env python3
"""G10: the reference's LeaveOneOutPreprocessor (src/data/preprocessing.py) run in
this build container on a small seeded raw ratings file with timestamp ties
(python tests/golden/make_golden_prep.py).  Stored: the raw rows and the three
output files' text.  No reference source."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _import_reference  # noqa: E402


def raw_rows(seed=3, users=120, items=90):
    rng = np.random.default_rng(seed)
    rows = []
    for u in range(1, users + 1):
        k = int(rng.integers(1, 30))
        its = rng.choice(np.arange(1, items + 1), size=k, replace=False)
        ts = rng.integers(0, 12, size=k) * 1000  # coarse: many timestamp ties per user
        for i, t in zip(its, ts):
            rows.append((u, int(i), int(rng.integers(1, 6)), int(t)))
    return np.array(rows, dtype=np.int64)


def main():
    _import_reference()
    from src.data.preprocessing import LeaveOneOutPreprocessor
    raw = raw_rows()
    os.makedirs("data/raw", exist_ok=True)
    with open("data/raw/u.data", "w") as f:
        f.write("\n".join("\t".join(map(str, r)) for r in raw) + "\n")
    np.random.seed(0)
    LeaveOneOutPreprocessor(num_negatives=20).run()
    out = {"raw": raw}
    for n in ("u.train.rating", "u.test.rating", "u.test.negative"):
        out[n] = np.array(open(os.path.join("data/processed", n)).read())
    np.savez_compressed(os.path.join(HERE, "G10_preprocess.npz"), **out)
    print({k: (v.shape if hasattr(v, "shape") else None) for k, v in out.items()})


if __name__ == "__main__":
    main()
