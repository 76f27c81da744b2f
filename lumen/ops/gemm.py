"""Projection GEMMs for decode: y = x @ W^T.

At decode batch 1 the projection is a pure stream of the weight matrix; for the shapes where it
measured faster the HIP weight-streaming kernel (``kernels/skinny_gemm.hip``) runs it instead
of a library GEMM.
Larger batches (and CPU tensors) go to ``torch.matmul`` (hipBLASLt with the tuned table)."""
from __future__ import annotations

import os

import torch

from ._native import native, use_native

# Measured per shape against hipBLASLt with the tuned table (lumen/bench/skinny_bench.py,
# profiles/r02_serve/skinny_bench.jsonl): the VALU weight-streaming kernel wins at M = 1 for
# N <= 4096 (o_proj 10.4 vs 22.6 us, down_proj 25.0 vs 27.7 us); hipBLASLt wins at the wide
# projections and at every M > 1, so those stay library GEMMs.
SKINNY_MAX_M = int(os.environ.get("LUMEN_SKINNY_MAX_M", "1"))
SKINNY_MAX_N = int(os.environ.get("LUMEN_SKINNY_MAX_N", "4096"))


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
