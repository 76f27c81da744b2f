"""Fast 2-D transpose (HIP kernel ``kernels/transpose.hip``; torch on CPU)."""
from __future__ import annotations

import torch

from ._native import native, use_native


def transpose_2d(x: torch.Tensor) -> torch.Tensor:
    """Contiguous x^T for a 2-D 16-bit tensor with unit column stride."""
    if (use_native(x) and x.dim() == 2 and x.dtype in (torch.bfloat16, torch.float16)
            and x.stride(1) == 1 and x.stride(0) % 8 == 0 and x.shape[0] % 8 == 0):
        out = torch.empty(x.shape[1], x.shape[0], device=x.device, dtype=x.dtype)
        native().transpose2d(x, out)
        return out
    return x.t().contiguous()
