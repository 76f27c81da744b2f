"""SwiGLU over a fused [gate | up] GEMM output (HIP kernel ``kernels/swiglu.hip``)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._native import native, use_native


def swiglu_ref(gu: torch.Tensor) -> torch.Tensor:
    g, u = gu.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(gu.dtype)


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        gu = gu.contiguous()
        out = torch.empty(*gu.shape[:-1], gu.shape[-1] // 2, device=gu.device, dtype=gu.dtype)
        native().swiglu(False, gu, None, out)
        ctx.save_for_backward(gu)
        return out

    @staticmethod
    def backward(ctx, dact):
        (gu,) = ctx.saved_tensors
        dgu = torch.empty_like(gu)
        native().swiglu(True, gu, dact.contiguous(), dgu)
        return dgu


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    if use_native(gu):
        return _SwiGLU.apply(gu)
    return swiglu_ref(gu)
