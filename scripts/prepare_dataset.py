#!/usr/bin/env python
"""Prepare the instruction-tuning dataset (CLI of reference scripts/prepare_dataset.py:124-155).

    python scripts/prepare_dataset.py [--num_samples N] [--output_dir ./data]
                                      [--source synthetic|hub|<local json/jsonl/parquet/csv/arrow>]

Writes ``{output_dir}/glaive_code_full`` or ``glaive_code_{N//1000}k`` (Arrow, one ``text``
column) consumed by the training CLIs' ``--dataset_path``.  The default source is the offline
synthetic corpus because the MI355X boxes have no network; ``--source hub`` reproduces the
reference's download when the Hub is reachable.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from lumen.data.prepare import dir_size_mb, prepare_dataset  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser(description="Prepare the Llama-2 chat formatted code dataset")
    p.add_argument("--num_samples", type=int, default=None,
                   help="number of rows (default: all rows of the source)")
    p.add_argument("--output_dir", type=str, default="./data")
    p.add_argument("--source", type=str, default="synthetic",
                   help="'synthetic' (offline), 'hub' (glaiveai/glaive-code-assistant), or a path")
    p.add_argument("--seed", type=int, default=42)
    a = p.parse_args(argv)
    t0 = time.time()
    out = prepare_dataset(a.output_dir, a.num_samples, a.source, a.seed)
    from datasets import load_from_disk

    n = len(load_from_disk(out))
    print(f"Saved {n:,} examples to {out} ({dir_size_mb(out):.1f} MB) in {time.time() - t0:.1f}s")
    return out


if __name__ == "__main__":
    main()
