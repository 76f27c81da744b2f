"""LM head + causal-LM cross-entropy (HIP kernel ``kernels/cross_entropy.hip``).

Reference behaviour (transformers Llama, reference training/train_baseline.py:122): logits =
lm_head(h) upcast to f32, CrossEntropyLoss(ignore_index=-100) averaged over non-ignored shifted
labels.  Here the logits stay 16-bit, the CE kernel turns them into d(loss)/d(logits) in place
during the forward (scaled by 1/num_valid), and the backward is a single GEMM dH = dlogits @ W
times the upstream scalar.  ``weight_fn`` returns the (possibly ZeRO-3-gathered) weight when
called, so the backward re-reads it through the parameter coordinator instead of pinning it.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.nn.functional as F

from ._native import native, use_native

IGNORE_INDEX = -100

# fp16 dynamic loss scaling: the engine points this at the device scalar it will multiply the
# loss by (loss scale / grad accum) before each forward, so the CE kernel writes dlogits already
# scaled -- (p - y) * S / n, like the reference's upcast-logits graph -- instead of the
# unscaled p / n that underflows fp16.  None in bf16 / fp32.
GRAD_SCALE_HINT = [None]


class _LMHeadCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, labels, weight_fn, n_valid, dummy_w, wt_fn=None):
        W = weight_fn()
        logits = torch.matmul(h, W.t())
        loss_sum = torch.zeros(1, dtype=torch.float32, device=h.device)
        hint = GRAD_SCALE_HINT[0]
        ctx.hint = hint
        native().cross_entropy(logits, labels, loss_sum, None, IGNORE_INDEX,
                               1.0 / max(n_valid, 1), True, hint)
        ctx.weight_fn = weight_fn
        ctx.wt_fn = wt_fn
        ctx.w_grad = dummy_w is not None and dummy_w.requires_grad
        ctx.save_for_backward(logits, h if ctx.w_grad else torch.empty(0))
        return (loss_sum / max(n_valid, 1)).squeeze(0)

    @staticmethod
    def backward(ctx, g):
        dlogits, h = ctx.saved_tensors
        # TN against the frozen head's cached W^T when it keeps one (K-contiguous operands:
        # 778 vs 874 us at Llama-2-7B's 8 x 512 tokens, gpurun r5_55), else NN against W
        wt = ctx.wt_fn() if ctx.wt_fn is not None else None
        dh = torch.matmul(dlogits, wt.t()) if wt is not None else torch.matmul(dlogits, ctx.weight_fn())
        # upstream grad (a 0-dim f32 tensor): multiplied in f32 math, never cast to 16 bits
        # first (2^16, the initial fp16 loss scale, is not representable in fp16); dlogits that
        # already carry the hinted scale are divided by it (ratio 1 on the engine's path)
        if (g.dtype == torch.float32 and g.is_cuda and dh.is_contiguous() and dh.numel() % 8 == 0
                and (ctx.hint is None or (ctx.hint.dtype == torch.float32 and ctx.hint.is_cuda))):
            native().scale_dev(dh, g.reshape(1), ctx.hint)  # one vectorized pass
        else:
            dh.mul_(g / ctx.hint if ctx.hint is not None else g)
        dw = None
        if ctx.w_grad:
            dw = torch.matmul(dlogits.t(), h)
            dw.mul_(g / ctx.hint if ctx.hint is not None else g)
        return dh, None, None, None, dw, None


def lm_head_cross_entropy(h: torch.Tensor, labels: torch.Tensor,
                          weight_fn: Callable[[], torch.Tensor], n_valid: int,
                          weight_param: torch.Tensor = None, wt_fn=None) -> torch.Tensor:
    """Mean CE over labels != -100.  h [T, H], labels [T] (already shifted).  ``wt_fn``: the
    frozen head's cached W^T [H, V] (``Linear.weight_t_fn``) for a TN input-gradient GEMM."""
    if use_native(h):
        return _LMHeadCE.apply(h.contiguous(), labels.contiguous(), weight_fn, int(n_valid),
                               weight_param, wt_fn)
    W = weight_fn()
    if not W.requires_grad:
        W = W.detach()  # see ops.lora._frozen
    logits = torch.matmul(h, W.t()).float()
    loss = F.cross_entropy(logits, labels, ignore_index=IGNORE_INDEX, reduction="sum")
    return loss / max(int(n_valid), 1)


def cross_entropy_rows(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Per-row CE (no grad) -- used by evaluation / serving logprob checks."""
    if use_native(logits):
        out = torch.empty(logits.shape[0], dtype=torch.float32, device=logits.device)
        native().cross_entropy(logits.contiguous(), labels.contiguous(), None, out, IGNORE_INDEX,
                               1.0, False, None)
        return out
    return F.cross_entropy(logits.float(), labels, ignore_index=IGNORE_INDEX, reduction="none")
