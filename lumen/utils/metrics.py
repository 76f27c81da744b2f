"""Experiment naming + metrics CSV (reference training/utils.py:11-88).

Same CSV (``results/training_metrics.csv``), same leading columns
``experiment,num_gpus,zero_stage,strategy,training_time_hours,samples_per_second,
peak_memory_gb,final_loss`` (reference training/train_baseline.py:246-255), plus lumen's
``tokens_per_second`` and ``tflops_per_gpu`` appended after them.  Rows written by an older run
with fewer columns stay readable: the header is extended, never reordered.
"""
from __future__ import annotations

import csv
import json
import os
from pathlib import Path
from typing import Dict

BASE_COLUMNS = ["experiment", "num_gpus", "zero_stage", "strategy", "training_time_hours",
                "samples_per_second", "peak_memory_gb", "final_loss"]
EXTRA_COLUMNS = ["tokens_per_second", "tflops_per_gpu"]


def create_experiment_name(num_gpus: int, zero_stage: int) -> str:
    """'baseline' for stage 0, else 'zero{stage}_{N}gpu' (reference training/utils.py:11-33)."""
    return "baseline" if zero_stage == 0 else f"zero{zero_stage}_{num_gpus}gpu"


def get_zero_stage_from_config(config_path: str) -> int:
    with open(config_path) as f:
        return int(json.load(f)["zero_optimization"]["stage"])


def save_training_metrics(metrics: Dict, csv_path: str = "results/training_metrics.csv") -> str:
    Path(os.path.dirname(csv_path) or ".").mkdir(parents=True, exist_ok=True)
    cols = BASE_COLUMNS + [c for c in EXTRA_COLUMNS if c in metrics]
    cols += [k for k in metrics if k not in cols]
    rows = []
    if os.path.isfile(csv_path):
        with open(csv_path, newline="") as f:
            r = csv.DictReader(f)
            old_cols = list(r.fieldnames or [])
            rows = list(r)
        cols = old_cols + [c for c in cols if c not in old_cols]
    rows.append({k: metrics.get(k, "") for k in cols})
    with open(csv_path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        for row in rows:
            w.writerow({k: row.get(k, "") for k in cols})
    print(f"\nMetrics saved to {csv_path}")
    return csv_path


def print_metrics_summary(metrics: Dict) -> None:
    print("\n" + "=" * 70)
    print("TRAINING METRICS")
    print("=" * 70)
    print(f"\nExperiment: {metrics['experiment']}")
    print(f"GPUs: {metrics['num_gpus']}")
    print(f"Strategy: {metrics['strategy']}")
    print()
    print(f"Training time: {metrics['training_time_hours']:.4f} hours")
    print(f"Throughput: {metrics['samples_per_second']:.1f} samples/sec")
    if "tokens_per_second" in metrics:
        print(f"Throughput: {metrics['tokens_per_second']:.0f} tokens/sec")
    print(f"Memory/GPU: {metrics['peak_memory_gb']:.2f} GB")
    print(f"Final loss: {metrics['final_loss']:.4f}")
    print("=" * 70)
