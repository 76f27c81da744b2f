"""Projection GEMMs for decode: y = x @ W^T.

At decode batch 1 the projection is a pure stream of the weight matrix; for the shapes where it
measured faster the HIP weight-streaming kernel (``kernels/skinny_gemm.hip``) runs it instead
of a library GEMM.
Larger batches (and CPU tensors) go to ``torch.matmul`` (hipBLASLt with the tuned table)."""
from __future__ import annotations

import os

import torch

from ._native import native, use_native

# Measured per shape against hipBLASLt with the tuned table (lumen/bench/skinny_bench.py
# --m1-forms, profiles/r02_serve/m1_forms.jsonl): at M = 1 the rows-per-lane weight-streaming
# kernel reaches 4.3-6.5 TB/s and beats hipBLASLt at every Llama-2-7B projection (qkv 17.1 vs
# 26.0 us, o 7.9 vs 18.1, gate_up 27.7 vs 49.1, down 16.3 vs 37.4); at M > 1 hipBLASLt wins, so
# those stay library GEMMs.
SKINNY_MAX_M = int(os.environ.get("LUMEN_SKINNY_MAX_M", "1"))
SKINNY_MAX_N = int(os.environ.get("LUMEN_SKINNY_MAX_N", str(1 << 30)))
# SwiGLU formed inside the batch-1 down projection: measured 21.4 us vs 18.5 us for the swiglu
# kernel + GEMV (every workgroup re-activates the whole gate|up vector), so off by default.
SWIGLU_GEMV = os.environ.get("LUMEN_SWIGLU_GEMV", "0") == "1"


def skinny_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (0 < x.shape[0] <= min(SKINNY_MAX_M, 16) and w.shape[0] <= SKINNY_MAX_N
            and use_native(x) and x.dim() == 2
            and w.dim() == 2 and x.dtype == w.dtype and x.dtype in (torch.bfloat16, torch.float16)
            and x.stride(1) == 1 and w.is_contiguous() and x.shape[1] == w.shape[1]
            and (w.shape[0] % 4 == 0 and w.shape[1] % 8 == 0 and x.stride(0) % 8 == 0
                 if x.shape[0] <= 4 else w.shape[0] % 16 == 0 and w.shape[1] % 128 == 0))


def linear_nt(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """x [M, K] @ w[N, K]^T -> [M, N]."""
    if skinny_ok(x, w):
        y = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=x.dtype)
        native().skinny_gemm(x, w, y)
        return y
    return torch.matmul(x, w.t())


def swiglu_linear_nt(gu: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """(silu(gu[:, :F]) * gu[:, F:]) @ w[N, F]^T, the MLP down projection.  At batch 1, where the
    weight-streaming kernel runs it, the activation is formed inside that kernel (no separate
    SwiGLU launch); otherwise SwiGLU kernel + ``linear_nt``."""
    from .activation import swiglu

    F = gu.shape[1] // 2
    if (SWIGLU_GEMV and gu.shape[0] == 1 and gu.shape[1] == 2 * F and skinny_ok(gu[:, :F], w)
            and gu.stride(0) % 8 == 0):
        y = torch.empty(1, w.shape[0], device=gu.device, dtype=gu.dtype)
        native().gemv_swiglu(gu, w, y)
        return y
    return linear_nt(swiglu(gu), w)
