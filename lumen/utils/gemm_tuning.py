"""hipBLASLt algorithm selection for the frozen-weight GEMMs (PyTorch TunableOp).

The base-model GEMMs (q|k|v, o, gate|up, down, lm_head: fwd and dX) are plain library GEMMs and
are ~60% of a training step.  hipBLASLt's default heuristic picks one solution per shape; the
TunableOp front end benchmarks every hipBLASLt (and rocBLAS) solution for a shape once and
records the fastest.  lumen ships the tuned table for its benchmark shapes
(``configs/tunableop/``) and loads it read-only at startup, so timed runs never tune.  Rows whose
library versions do not match the running image are rejected by TunableOp's own validators and
the default heuristic is used instead.

    python bench.py --tune_gemms configs/tunableop/mi355x_llama2-7b.csv   # (re)generate
"""
from __future__ import annotations

import os
from typing import Optional

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_TABLE = os.path.join(ROOT, "configs", "tunableop", "mi355x_gemms.csv")


def load_tuned_gemms(path: Optional[str] = None) -> bool:
    """Use the tuned solutions in ``path`` (tuning stays off).  Returns True when loaded."""
    path = path or os.environ.get("LUMEN_GEMM_TABLE", DEFAULT_TABLE)
    if not path or path == "off" or not os.path.isfile(path) or not torch.cuda.is_available():
        return False
    import torch.cuda.tunable as tn

    tn.enable(True)
    tn.tuning_enable(False)
    try:
        tn.record_untuned_enable(False)
    except Exception:  # noqa: BLE001 - older builds
        pass
    ok = bool(tn.read_file(path))
    if not ok:
        tn.enable(False)
    return ok


def start_gemm_tuning(out_path: str, max_ms: int = 60, rotating_mb: Optional[int] = None) -> None:
    """Tune every GEMM shape met from now on; results are written to ``out_path`` at exit.

    Candidates are timed over a rotating set of operand buffers larger than the 256 MB
    Infinity Cache (``rotating_mb``, env ``LUMEN_TUNE_ROTATING_MB``, default 1024), i.e. with
    weights streaming from HBM as they do inside a training step, not from a warm cache."""
    import torch.cuda.tunable as tn

    if rotating_mb is None:
        rotating_mb = int(os.environ.get("LUMEN_TUNE_ROTATING_MB", "1024"))
    # 0 disables the rotating buffers: they copy ldc * n elements from C's own pointer, which
    # overruns a column-view output (lumen.ops.gemm.mm_nt tails) at the end of its allocation
    tn.set_rotating_buffer_size(max(rotating_mb, 0))

    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    tn.enable(True)
    tn.tuning_enable(True)
    tn.set_filename(out_path, False)
    tn.set_max_tuning_duration(max_ms)
    tn.set_max_tuning_iterations(100)
    if os.path.isfile(out_path):
        tn.read_file(out_path)


def tuned_entries() -> int:
    import torch.cuda.tunable as tn

    try:
        return len(tn.get_results())
    except Exception:  # noqa: BLE001
        return 0
