#!/usr/bin/env python
"""Compare training runs (CLI of reference scripts/compare_training.py:171-196).

    python scripts/compare_training.py [--csv results/training_metrics.csv]
                                       [--plot results/plots/training_comparison.png]

Reads the metrics CSV the training CLIs append to, prints speedup / efficiency per experiment
and writes the 2x2 comparison figure.  With no arguments it behaves like the reference.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from lumen.utils.compare import compare  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser(description="Compare training scaling results")
    p.add_argument("--csv", default="results/training_metrics.csv")
    p.add_argument("--plot", default="results/plots/training_comparison.png")
    a = p.parse_args(argv)
    if not os.path.isfile(a.csv):
        print(f"No metrics file at {a.csv}: run the training scripts first")
        return None
    return compare(a.csv, a.plot)


if __name__ == "__main__":
    main()
