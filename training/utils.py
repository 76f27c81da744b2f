"""Shared helpers (reference training/utils.py API): experiment naming, ZeRO stage lookup,
metrics CSV.  Importable both as ``training.utils`` and as ``utils`` from inside training/."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lumen.utils.metrics import (create_experiment_name, get_zero_stage_from_config,  # noqa: E402,F401
                                 print_metrics_summary, save_training_metrics)
