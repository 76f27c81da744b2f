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
        stale = provenance_error()
        if stale and os.environ.get("LUMEN_ALLOW_STALE_NATIVE", "0") != "1":
            raise RuntimeError(stale)
        _C = importlib.import_module("lumen._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _err = e
    return _C


def provenance() -> dict:
    """The build manifest of the loaded extension (source digest, arch, build host / time) and
    whether the sources in the tree still match it."""
    from ..csrc.build import read_manifest, source_digest

    man = read_manifest() or {}
    cur = source_digest()["sha256"]
    return {"sources_sha256": man.get("sha256"), "tree_sha256": cur,
            "matches_tree": man.get("sha256") == cur, "arch": man.get("arch"),
            "built_at": man.get("built_at"), "build_host": man.get("host")}


def provenance_error():
    """A message when the in-tree extension was built from other sources than the tree holds
    (a stale .so would silently run old kernels), else None."""
    from ..csrc.build import ext_path, read_manifest, source_digest

    if not os.path.exists(ext_path()):
        return None  # the import error says it is missing
    man = read_manifest()
    if man is None:
        return ("lumen native extension has no build manifest (lumen/_C.sources.json): rebuild "
                "with `python -m lumen.csrc.build`")
    if man.get("sha256") != source_digest()["sha256"]:
        return ("lumen native extension is stale: built from sources "
                f"{str(man.get('sha256'))[:12]}, the tree holds {source_digest()['sha256'][:12]}; "
                "rebuild with `python -m lumen.csrc.build`")
    return None


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
