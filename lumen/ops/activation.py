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


class _RecomputeMLP(torch.autograd.Function):
    """down(swiglu(gate_up(y))) for frozen gate|up / down weights, keeping only ``y`` for the
    backward: the [T, 2F] gate|up output -- 5.4 H-wide rows per token, the largest activation a
    Llama layer saves -- is recomputed by one GEMM in the backward instead of being stored
    (selective activation checkpointing).  The down projection's forward is NOT re-run (full
    layer recompute does that too).  Weights are fetched through their ``weight_fn`` /
    ``weight_t_fn`` at backward time (ZeRO-3 rebinds gathered weights)."""

    @staticmethod
    def forward(ctx, y, gu_w, gu_wt, dn_w, dn_wt):
        from .gemm import mm_nt

        gu = mm_nt(y, gu_w())
        if use_native(gu):
            act = torch.empty(*gu.shape[:-1], gu.shape[-1] // 2, device=gu.device,
                              dtype=gu.dtype)
            native().swiglu(False, gu, None, act)
        else:
            act = swiglu_ref(gu)
        del gu
        out = mm_nt(act, dn_w())
        ctx.save_for_backward(y)
        ctx.fns = (gu_w, gu_wt, dn_w, dn_wt)
        return out

    @staticmethod
    def backward(ctx, dout):
        from .gemm import mm_nt

        (y,) = ctx.saved_tensors
        gu_w, gu_wt, dn_w, dn_wt = ctx.fns
        dact = _dx(dout.contiguous(), dn_w, dn_wt)
        gu = mm_nt(y, gu_w())                     # the recompute
        if use_native(gu):
            dgu = torch.empty_like(gu)
            native().swiglu(True, gu, dact, dgu)
        else:  # the reference op's own autograd: same rounding as the unrecomputed layer
            with torch.enable_grad():
                g_ = gu.detach().requires_grad_(True)
                swiglu_ref(g_).backward(dact)
            dgu = g_.grad
        del gu, dact
        return _dx(dgu, gu_w, gu_wt), None, None, None, None


def _dx(dy, w_fn, wt_fn):
    """dX = dY @ W, as the TN GEMM against a cached W^T when the layer keeps one."""
    from .gemm import mm_nt

    wt = wt_fn() if wt_fn is not None else None
    return mm_nt(dy, wt) if wt is not None else torch.matmul(dy, w_fn())


def recompute_mlp(y: torch.Tensor, gate_up, down) -> torch.Tensor:
    """Selective-recompute MLP over two frozen, adapter-free ``Linear`` modules (see
    ``_RecomputeMLP``)."""
    return _RecomputeMLP.apply(y.contiguous(), gate_up.weight_fn, gate_up._wt_fn(),
                               down.weight_fn, down._wt_fn())
