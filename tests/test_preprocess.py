"""Preprocessing parity: ncf_amd.preprocessing /
src.data.preprocessing.LeaveOneOutPreprocessor against the reference's own run on
the same raw file and seed (tests/golden/G10_preprocess.npz, make_golden_prep.py):
the three output files must be byte-identical (split, tie order, test negatives)."""
import os

import numpy as np


def test_preprocessor_matches_reference_files(golden, tmp_path, monkeypatch):
    g = golden("G10_preprocess")
    monkeypatch.chdir(tmp_path)
    os.makedirs("data/raw")
    with open("data/raw/u.data", "w") as f:
        f.write("\n".join("\t".join(map(str, r)) for r in g["raw"]) + "\n")
    from src.data.preprocessing import LeaveOneOutPreprocessor
    np.random.seed(0)
    LeaveOneOutPreprocessor(num_negatives=20).run()
    for n in ("u.train.rating", "u.test.rating", "u.test.negative"):
        assert open(os.path.join("data/processed", n)).read() == str(g[n]), n


def test_preprocessed_files_load(golden, tmp_path, monkeypatch):
    """The output feeds load_all() (datasets.py:9-36) unchanged."""
    g = golden("G10_preprocess")
    monkeypatch.chdir(tmp_path)
    os.makedirs("data/processed")
    for n in ("u.train.rating", "u.test.rating", "u.test.negative"):
        with open(os.path.join("data/processed", n), "w") as f:
            f.write(str(g[n]))
    from ncf_amd.data import load_all
    train, test, U, I, mat = load_all(test_num=21)
    assert len(test) == 21 * len(str(g["u.test.rating"]).strip().splitlines())
    assert mat.nnz == len(train)
