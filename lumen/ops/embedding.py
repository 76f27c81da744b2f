"""Token-embedding lookup: HIP row gather (``kernels/embedding.hip``) for frozen
16-bit tables on the GPU; ``F.embedding`` otherwise (CPU, f32 tables, trainable tables)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._native import native, use_native


def embedding(ids: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """[..] int ids -> [.., H] rows of ``weight`` (no gradient w.r.t. a frozen table)."""
    if (use_native(weight) and not (weight.requires_grad and torch.is_grad_enabled())
            and weight.dtype in (torch.bfloat16, torch.float16) and weight.is_contiguous()
            and weight.shape[1] % 8 == 0 and ids.is_cuda):
        flat = ids.reshape(-1)
        if flat.dtype != torch.int64 or not flat.is_contiguous():
            flat = flat.to(torch.int64).contiguous()
        out = torch.empty(flat.numel(), weight.shape[1], device=weight.device, dtype=weight.dtype)
        native().embedding(weight, flat, out)
        return out.view(*ids.shape, weight.shape[1])
    return F.embedding(ids, weight)
