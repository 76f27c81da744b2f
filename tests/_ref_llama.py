"""Independent fp32 PyTorch Llama forward: the oracle of the production-shape numerics tests.

Written from the model definition (HF LlamaForCausalLM semantics: RMSNorm eps, rotate-half
RoPE theta 1e4, causal softmax attention, SwiGLU, untied head; PEFT LoRA y += s B(A(drop x)))
with plain torch ops in fp32 -- no lumen kernel, fused op or fold is involved.  The only lumen
function used is ``dropout_mask_ref``: it DEFINES which elements the kernels drop (a counter
hash of the per-call seed), so the oracle applies the identical mask.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from lumen.ops.lora import dropout_mask_ref


def ref_params(model, device) -> Dict:
    """fp32 copies of a lumen Llama's weights; adapters as fp32 leaves with requires_grad."""
    f = lambda t: t.detach().to(device=device, dtype=torch.float32).clone()  # noqa: E731
    P = {"embed": f(model.embed_tokens.weight), "norm": f(model.norm.weight),
         "head": f(model.lm_head.weight), "layers": []}
    for l in model.layers:
        d = {"ln1": f(l.input_layernorm.weight), "qkv": f(l.self_attn.qkv_proj.weight),
             "o": f(l.self_attn.o_proj.weight), "ln2": f(l.post_attention_layernorm.weight),
             "gu": f(l.mlp.gate_up_proj.weight), "down": f(l.mlp.down_proj.weight)}
        for key, lin in (("qkv", l.self_attn.qkv_proj), ("o", l.self_attn.o_proj),
                         ("gu", l.mlp.gate_up_proj), ("down", l.mlp.down_proj)):
            lo = lin.lora
            if lo is not None and lin.lora_enabled:
                d[key + "_lora"] = (f(lo.lora_A).requires_grad_(True),
                                    f(lo.lora_B).requires_grad_(True), list(lo.segs), lo.r,
                                    lo.scale)
        P["layers"].append(d)
    return P


def rms(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


def rope(x, pos, theta):
    """x [T, heads, D] rotated at integer positions pos [T] (HF rotate_half convention)."""
    D = x.shape[-1]
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, device=x.device, dtype=torch.float64) / D))
    ang = pos.to(torch.float64)[:, None] * inv[None]
    cos = torch.cat([ang.cos(), ang.cos()], -1).float()[:, None]
    sin = torch.cat([ang.sin(), ang.sin()], -1).float()[:, None]
    rot = torch.cat([-x[..., D // 2:], x[..., :D // 2]], -1)
    return x * cos + rot * sin


def lin(x, W, lora=None, p: float = 0.0, seed: int = 0):
    y = x @ W.t()
    if lora is None:
        return y
    A, B, segs, r, scale = lora
    xd = x
    if p > 0:
        keep = dropout_mask_ref(seed, x.shape[0], x.shape[1], p, x.device)
        xd = torch.where(keep, x / (1.0 - p), torch.zeros((), device=x.device))
    Z = xd @ A.t()
    parts, cur = [], 0
    for (n_off, n_len, r_off, b_off) in sorted(segs):
        if n_off > cur:
            parts.append(y[:, cur:n_off])
        parts.append(y[:, n_off:n_off + n_len]
                     + scale * (Z[:, r_off:r_off + r] @ B[b_off:b_off + n_len].t()))
        cur = n_off + n_len
    if cur < y.shape[1]:
        parts.append(y[:, cur:])
    return torch.cat(parts, 1)


def attention(q, k, v, lens: List[int], kv_last=None):
    """Causal attention of packed sequences: q [T, nh, D], k/v [T, nkv, D].  ``kv_last``: a
    function applied to the K / V the LAST query row of each sequence reads (a decode row
    attending to a quantized cache), the other rows reading them as given."""
    nh, nkv, D = q.shape[1], k.shape[1], q.shape[2]
    outs, s0 = [], 0
    for L in lens:
        qs = q[s0:s0 + L].transpose(0, 1)                       # [nh, L, D]
        ks = k[s0:s0 + L].transpose(0, 1).repeat_interleave(nh // nkv, 0)
        vs = v[s0:s0 + L].transpose(0, 1).repeat_interleave(nh // nkv, 0)
        sc = (qs @ ks.transpose(1, 2)) / math.sqrt(D)
        mask = torch.ones(L, L, dtype=torch.bool, device=q.device).triu(1)
        sc = sc.masked_fill(mask, float("-inf"))
        o = sc.softmax(-1) @ vs
        if kv_last is not None:
            kq, vq = kv_last(ks), kv_last(vs)
            sl = (qs[:, -1:] @ kq.transpose(1, 2)) / math.sqrt(D)
            o = torch.cat([o[:, :-1], sl.softmax(-1) @ vq], 1)
        outs.append(o.transpose(0, 1).reshape(L, nh * D))
        s0 += L
    return torch.cat(outs, 0)


def _identity(t):
    return t


def bf16_round(t):
    """Round to bf16 and back (the storage precision of every activation of a bf16 model)."""
    return t.to(torch.bfloat16).float()


def fp8_round(t):
    """Round to OCP e4m3fn and back (the fp8 KV cache's element type)."""
    return t.to(torch.float8_e4m3fn).float()


def ref_hidden(P: Dict, cfg, ids: torch.Tensor, lens: List[int], p: float = 0.0,
               seeds: Optional[List[int]] = None, store=_identity,
               kv_last=None) -> torch.Tensor:
    """Final-norm hidden states [T, H] of packed sequences ``ids`` [T] with lengths ``lens``.
    ``seeds``: the dropout seed of every adapted linear call, in call order (q|k|v then o per
    layer -- the order lumen draws them from torch's CPU generator).  ``store``: rounding
    applied to every activation between ops (``bf16_round``: the bf16 noise floor of the same
    math, each op itself in fp32); ``kv_last``: see ``attention``."""
    nh, nkv, D, Fd = (cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim,
                      cfg.intermediate_size)
    eps, theta = cfg.rms_norm_eps, cfg.rope_theta
    pos = torch.cat([torch.arange(L, device=ids.device) for L in lens])
    h = store(P["embed"][ids])
    it = iter(seeds or [])

    def call(x, L, key):
        lo = L.get(key + "_lora")
        seed = next(it) if (lo is not None and p > 0) else 0
        return store(lin(x, L[key], lo, p, seed))

    for L in P["layers"]:
        x = store(rms(h, L["ln1"], eps))
        qkv = call(x, L, "qkv")
        q, k, v = qkv.split([nh * D, nkv * D, nkv * D], 1)
        T = q.shape[0]
        q = store(rope(q.reshape(T, nh, D), pos, theta))
        k = store(rope(k.reshape(T, nkv, D), pos, theta))
        o = store(attention(q, k, v.reshape(T, nkv, D), lens, kv_last))
        h = store(h + call(o, L, "o"))
        x = store(rms(h, L["ln2"], eps))
        gu = call(x, L, "gu")
        h = store(h + call(store(F.silu(gu[:, :Fd]) * gu[:, Fd:]), L, "down"))
    return rms(h, P["norm"], eps)


def ref_loss(P: Dict, cfg, ids: torch.Tensor, labels: torch.Tensor, lens: List[int],
             p: float = 0.0, seeds: Optional[List[int]] = None, store=_identity) -> torch.Tensor:
    """Mean next-token cross-entropy over labels != -100 (labels already shifted)."""
    h = ref_hidden(P, cfg, ids, lens, p, seeds, store)
    logits = h @ P["head"].t()
    return F.cross_entropy(logits, labels, ignore_index=-100)
