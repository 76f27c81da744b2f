"""Loader for the in-tree native extension ``lumen/_C*.so`` (built by ``lumen.csrc.build``).

Policy: on a GPU tensor the HIP kernel is THE implementation.  If the extension is missing on a
GPU box every op raises (no silent eager fallback) unless ``LUMEN_ALLOW_TORCH_FALLBACK=1`` is set
explicitly (used only for A/B debugging).  CPU tensors always take the torch reference path,
which is also the numerics oracle of the GPU tests.
"""
from __future__ import annotations

import importlib
import os

import torch

_C = None
_err = None


def _load():
    global _C, _err
    if _C is not None or _err is not None:
        return _C
    try:
        _C = importlib.import_module("lumen._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _err = e
    return _C


def native():
    """The extension module or None."""
    return _load()


def native_error():
    _load()
    return _err


def allow_fallback() -> bool:
    return os.environ.get("LUMEN_ALLOW_TORCH_FALLBACK", "0") == "1"


def use_native(t: torch.Tensor) -> bool:
    """True when `t` lives on the GPU and the HIP path must run."""
    if not t.is_cuda:
        return False
    if _load() is not None and os.environ.get("LUMEN_DISABLE_NATIVE", "0") != "1":
        return True
    if allow_fallback():
        return False
    raise RuntimeError(
        "lumen native extension not available for a GPU tensor "
        f"({native_error()!r}); build it with `python -m lumen.csrc.build` "
        "(or set LUMEN_ALLOW_TORCH_FALLBACK=1 to run the slow torch reference)")


DTYPE_CODE = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}
