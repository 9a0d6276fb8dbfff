#!/usr/bin/env python3
"""Temporal leave-one-out preprocessing (reference scripts/preprocess.py): data/raw/u.data ->
data/processed/u.{train.rating,test.rating,test.negative}."""
import os
import sys

sys.path.append(os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from src.data.preprocessing import LeaveOneOutPreprocessor  # noqa: E402

if __name__ == "__main__":
    LeaveOneOutPreprocessor().run()
