"""Fast 2-D transpose (HIP kernel ``kernels/transpose.hip``; torch on CPU)."""
from __future__ import annotations

from typing import Optional

import torch

from ._native import native, use_native


def native_ok(x: torch.Tensor) -> bool:
    return (use_native(x) and x.dim() == 2 and x.dtype in (torch.bfloat16, torch.float16)
            and x.stride(1) == 1 and x.stride(0) % 8 == 0 and x.shape[0] % 8 == 0)


def transpose_2d(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Contiguous x^T for a 2-D 16-bit tensor with unit column stride (into ``out`` if given:
    a contiguous [cols, rows] tensor)."""
    if out is None:
        out = torch.empty(x.shape[1], x.shape[0], device=x.device, dtype=x.dtype)
    if native_ok(x):
        native().transpose2d(x, out)
    else:
        out.copy_(x.t())
    return out
