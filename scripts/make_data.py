#!/usr/bin/env python3
"""Write a synthetic MovieLens-shaped dataset in the reference's file formats
(data/processed/u.train.rating, u.test.rating, u.test.negative), so the
training scripts (ours or the reference's, unchanged) have data to read.
Usage: python scripts/make_data.py --shape ml-100k --out data/processed
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from ncf_amd import synthetic  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--shape", default="ml-100k", choices=sorted(synthetic.SHAPES))
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--out", default="data/processed")
    a = p.parse_args()
    ds = synthetic.make_dataset(a.shape, seed=a.seed)
    tr, neg = synthetic.write_reference_files(ds, a.out)
    print(f"wrote {tr} ({len(ds['train_users'])} rows) and {neg} ({len(ds['test_users'])} users); "
          f"user_num={ds['user_num']} item_num={ds['item_num']}")


if __name__ == "__main__":
    main()
