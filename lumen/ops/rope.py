"""Rotary embeddings (HIP kernel ``kernels/rope.hip``; torch reference on CPU).

Training: ``qkv_rope_split`` turns the fused QKV GEMM output [B*S, (nh+2nkv)*D] into rotated
q [B,nh,S,D], k [B,nkv,S,D] and v [B,nkv,S,D] in one pass (rotate_half convention of
transformers' Llama, theta from the config).  Serving: ``rope_inplace`` rotates q/k heads inside
the token-major QKV buffer at arbitrary positions.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from ._native import native, use_native

_TABLES: Dict[tuple, Tuple[torch.Tensor, torch.Tensor]] = {}


def rope_tables(D: int, max_pos: int, theta: float, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """f32 cos/sin tables [max_pos, D/2] (built once per device on the host, f64 math)."""
    key = (D, max_pos, float(theta), str(device))
    t = _TABLES.get(key)
    if t is None:
        inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
        ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
        t = (ang.cos().float().to(device).contiguous(), ang.sin().float().to(device).contiguous())
        _TABLES[key] = t
    return t


def _rotate_ref(x, cos, sin, inverse=False):
    # x [..., S, D]; cos/sin [S, D/2]
    half = x.shape[-1] // 2
    a, b = x[..., :half].float(), x[..., half:].float()
    sgn = -1.0 if inverse else 1.0
    oa = a * cos - sgn * b * sin
    ob = b * cos + sgn * a * sin
    return torch.cat([oa, ob], -1).to(x.dtype)


def qkv_rope_split_ref(qkv, B, S, nh, nkv, D, cos_t, sin_t, pos=None):
    x = qkv.view(B, S, nh + 2 * nkv, D)
    q = x[:, :, :nh].transpose(1, 2)
    k = x[:, :, nh:nh + nkv].transpose(1, 2)
    v = x[:, :, nh + nkv:].transpose(1, 2).contiguous()
    if pos is None:
        cos, sin = cos_t[:S], sin_t[:S]
        cos, sin = cos[None, None], sin[None, None]
    else:
        p = pos.view(B, S).long()
        cos, sin = cos_t[p][:, None], sin_t[p][:, None]
    return _rotate_ref(q, cos, sin).contiguous(), _rotate_ref(k, cos, sin).contiguous(), v


class _QKVRope(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, B, S, nh, nkv, D, cos_t, sin_t, pos):
        C = native()
        qkv = qkv.contiguous()
        dev, dt = qkv.device, qkv.dtype
        q = torch.empty(B, nh, S, D, device=dev, dtype=dt)
        k = torch.empty(B, nkv, S, D, device=dev, dtype=dt)
        v = torch.empty(B, nkv, S, D, device=dev, dtype=dt)
        C.qkv_rope(False, qkv, q, k, v, pos, cos_t, sin_t, S, nh, nkv, D)
        ctx.dims = (B, S, nh, nkv, D)
        ctx.save_for_backward(cos_t, sin_t, pos if pos is not None else torch.empty(0))
        ctx.has_pos = pos is not None
        ctx.qkv_shape = qkv.shape
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        C = native()
        B, S, nh, nkv, D = ctx.dims
        cos_t, sin_t, pos = ctx.saved_tensors
        ref = dq if dq is not None else (dk if dk is not None else dv)
        dqkv = torch.empty(ctx.qkv_shape, device=ref.device, dtype=ref.dtype)
        z = lambda h: torch.zeros(B, h, S, D, device=ref.device, dtype=ref.dtype)  # noqa: E731
        dq = dq.contiguous() if dq is not None else z(nh)
        dk = dk.contiguous() if dk is not None else z(nkv)
        dv = dv.contiguous() if dv is not None else z(nkv)
        C.qkv_rope(True, dqkv, dq, dk, dv, pos if ctx.has_pos else None, cos_t, sin_t, S, nh, nkv, D)
        return dqkv, None, None, None, None, None, None, None, None


def qkv_rope_split(qkv: torch.Tensor, B: int, S: int, nh: int, nkv: int, D: int,
                   cos_t: torch.Tensor, sin_t: torch.Tensor, pos: Optional[torch.Tensor] = None):
    if use_native(qkv):
        if pos is not None:
            pos = pos.to(torch.int32).contiguous()
        return _QKVRope.apply(qkv, B, S, nh, nkv, D, cos_t, sin_t, pos)
    return qkv_rope_split_ref(qkv, B, S, nh, nkv, D, cos_t, sin_t, pos)


def rope_inplace(x2d: torch.Tensor, pos: torch.Tensor, nheads: int, D: int,
                 cos_t: torch.Tensor, sin_t: torch.Tensor, col_offset: int = 0) -> None:
    """Rotate `nheads` heads starting at column `col_offset` of token-major x2d [T, W] in place."""
    T = x2d.shape[0]
    if T == 0:
        return
    if use_native(x2d):
        sub = x2d[:, col_offset:]
        native().rope_inplace(sub, pos.to(torch.int32).contiguous(), cos_t, sin_t, T,
                              x2d.stride(0), nheads, D)
        return
    view = x2d[:, col_offset:col_offset + nheads * D].view(T, nheads, D)
    p = pos.long()
    cos, sin = cos_t[p][:, None], sin_t[p][:, None]
    view.copy_(_rotate_ref(view, cos, sin))


_NEG_SIN = {}


def _neg(sin_t):
    k = (sin_t.data_ptr(), sin_t.shape, str(sin_t.device))
    t = _NEG_SIN.get(k)
    if t is None:
        t = (-sin_t).contiguous()
        _NEG_SIN[k] = t
    return t


class _RopeQKV(torch.autograd.Function):
    """In-place RoPE on the q and k heads of the fused QKV buffer (training path of the HIP
    flash attention); backward = the inverse rotation (sin -> -sin) applied in place."""

    @staticmethod
    def forward(ctx, qkv, pos, nqk, D, cos_t, sin_t):
        native().rope_inplace(qkv, pos, cos_t, sin_t, qkv.shape[0], qkv.stride(0), nqk, D)
        ctx.mark_dirty(qkv)
        ctx.save_for_backward(pos)
        ctx.meta = (nqk, D, cos_t, sin_t)
        return qkv

    @staticmethod
    def backward(ctx, g):
        (pos,) = ctx.saved_tensors
        nqk, D, cos_t, sin_t = ctx.meta
        # g is the flash-attention backward's fresh dQKV buffer (sole consumer): rotate it in
        # place instead of copying 3*T*H*2 bytes
        if getattr(g, "_lumen_rope_undone", False):  # the flash-attention backward did it
            return g, None, None, None, None, None
        g = g if g.is_contiguous() else g.contiguous()
        native().rope_inplace(g, pos, cos_t, _neg(sin_t), g.shape[0], g.stride(0), nqk, D)
        return g, None, None, None, None, None


def rope_qkv_(qkv: torch.Tensor, pos: torch.Tensor, nh: int, nkv: int, D: int, cos_t, sin_t):
    """Rotate q and k heads of qkv [T, (nh+2nkv)*D] in place (autograd-aware)."""
    if use_native(qkv):
        return _RopeQKV.apply(qkv, pos.to(torch.int32).contiguous(), nh + nkv, D, cos_t, sin_t)
    T = qkv.shape[0]
    out = qkv.clone()
    view = out[:, :(nh + nkv) * D].view(T, nh + nkv, D)
    p = pos.long()
    rot = _rotate_ref(view, cos_t[p][:, None], sin_t[p][:, None])
    return torch.cat([rot.reshape(T, -1), out[:, (nh + nkv) * D:]], 1)
