"""Llama / Llama-2 decoder (the model the reference fine-tunes).

Reference: ``AutoModelForCausalLM.from_pretrained("meta-llama/Llama-2-7b-hf", fp16)``
(training/train_baseline.py:122-126) -> transformers LlamaForCausalLM: 32 layers, hidden 4096,
32 heads x 128, SwiGLU FFN 11008, RMSNorm eps 1e-5, RoPE theta 1e4, vocab 32000, untied head.

MI355X-first layout: q|k|v and gate|up are fused into one GEMM each (one weight, one launch, one
LoRA "A" product for the shared input), RoPE is fused with the head-major split, residual adds
are fused into the RMSNorms, the loss is fused with the LM head.  The decoder-layer loop calls
an optional ZeRO-3 parameter coordinator (``self.coordinator``) around each unit (embedding,
each layer, final norm + head) so partitioned weights are gathered / prefetched / released.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.utils.checkpoint as cp

from ..ops._native import use_native
from ..ops.embedding import embedding
from ..ops.lora import arena_reset
from ..ops.activation import (fused_mlp, fused_mlp_ok, overlap_mlp, overlap_mlp_plan,
                              recompute_mlp, swiglu)
from ..ops.attention import causal_attention, flash_attention_qkv, prepare_varlen
from ..ops.loss import lm_head_cross_entropy
from ..ops.rope import qkv_rope_split, rope_qkv_, rope_tables
from .config import ModelConfig
from .layers import Linear, RMSNorm


class LlamaAttention(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype=None, device=None):
        super().__init__()
        self.cfg = cfg
        D, nh, nkv, H = cfg.head_dim, cfg.num_attention_heads, cfg.num_key_value_heads, cfg.hidden_size
        self.qkv_proj = Linear(H, (nh + 2 * nkv) * D, dtype=dtype, device=device,
                               seg_sizes=[nh * D, nkv * D, nkv * D],
                               seg_names=["q_proj", "k_proj", "v_proj"])
        self.o_proj = Linear(nh * D, H, dtype=dtype, device=device, seg_names=["o_proj"])

    def forward(self, x2d: torch.Tensor, B: int, S: int, pos: Optional[torch.Tensor] = None,
                cu: Optional[tuple] = None):
        """``cu`` (packed batches): sequence offsets into the B*S token rows; attention stays
        within each sequence and ``pos`` holds the per-sequence positions."""
        c = self.cfg
        nh, nkv, D = c.num_attention_heads, c.num_key_value_heads, c.head_dim
        cos, sin = rope_tables(D, c.max_position_embeddings, c.rope_theta, x2d.device)
        # the HIP flash / fused-RoPE path takes 16-bit activations; an fp32 model on the GPU
        # (--dtype fp32) or the explicit torch fallback runs the portable path below
        if (x2d.is_cuda and D == 128 and USE_FLASH and x2d.dtype != torch.float32
                and use_native(x2d)):
            # HIP path: RoPE in place on the fused buffer (inside the adapter write-back when
            # q|k are adapted), flash attention reads q/k/v from it and writes O token-major
            # (no split / transpose copies)
            if pos is None:
                pos = _positions(B, S, x2d.device)
            pos = pos.to(torch.int32).contiguous()
            if self.qkv_proj.has_active_lora and FUSED_ROPE:
                qkv = self.qkv_proj(x2d, rope=(pos, cos, sin, (nh + nkv) * D))
            else:
                qkv = rope_qkv_(self.qkv_proj(x2d), pos, nh, nkv, D, cos, sin)
            # the FA backward undoes the rotation in its dQ / dK epilogues (FUSED_ROPE_BWD)
            o = flash_attention_qkv(qkv, cu if cu is not None else tuple(range(0, B * S + 1, S)),
                                    nh, nkv, D, True,
                                    rope=(pos, cos, sin) if FUSED_ROPE_BWD else None,
                                    out_ext=self.o_proj.fold_ext())
            return self.o_proj(o)
        qkv = self.qkv_proj(x2d)
        if cu is not None:  # packed rows, portable path: one causal block per sequence
            outs = []
            for s0, s1 in zip(cu[:-1], cu[1:]):
                q, k, v = qkv_rope_split(qkv[s0:s1], 1, s1 - s0, nh, nkv, D, cos, sin,
                                         pos[s0:s1] if pos is not None else None)
                outs.append(causal_attention(q, k, v))
            return self.o_proj(torch.cat(outs, 0))
        q, k, v = qkv_rope_split(qkv, B, S, nh, nkv, D, cos, sin, pos)
        o = causal_attention(q, k, v)
        return self.o_proj(o)


USE_FLASH = True
FUSED_ROPE = True  # RoPE inside the q|k|v adapter write-back (lora_v2 UP kernel)
FUSED_ROPE_BWD = True  # inverse RoPE inside the flash-attention dQ / dK epilogues
_POS = {}


def _positions(B: int, S: int, device) -> torch.Tensor:
    key = (B, S, str(device))
    t = _POS.get(key)
    if t is None:
        t = torch.arange(S, dtype=torch.int32, device=device).repeat(B)
        _POS[key] = t
    return t


def parse_ckpt_policy(v, policies=("none", "selective", "full")):
    """``"policy"`` or ``"policy:N"`` (the first N layers recompute) -> (policy, N or None)."""
    n = None
    if isinstance(v, str) and ":" in v:
        v, ns = v.split(":", 1)
        try:
            n = int(ns)
        except ValueError:
            n = -1
        if n < 0:
            raise ValueError(f"gradient checkpointing layer count must be an integer >= 0: {ns!r}")
    if v not in policies:
        raise ValueError(f"gradient checkpointing policy must be one of {policies} "
                         "(optionally ':N' for the first N layers)")
    if n == 0:
        v, n = "none", None
    return v, (None if v == "none" else n)


class LlamaMLP(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype=None, device=None):
        super().__init__()
        H, Fd = cfg.hidden_size, cfg.intermediate_size
        self.gate_up_proj = Linear(H, 2 * Fd, dtype=dtype, device=device, seg_sizes=[Fd, Fd],
                                   seg_names=["gate_proj", "up_proj"])
        self.down_proj = Linear(Fd, H, dtype=dtype, device=device, seg_names=["down_proj"])
        self.recompute = False  # selective checkpointing: gate|up output recomputed in backward

    @property
    def recompute_eligible(self) -> bool:
        """Selective recompute needs frozen gate|up / down weights without active adapters
        (``recompute_mlp`` re-runs only the frozen gate|up GEMM in the backward)."""
        gu, dn = self.gate_up_proj, self.down_proj
        return not (gu.has_active_lora or dn.has_active_lora or gu.weight.requires_grad
                    or dn.weight.requires_grad)

    def forward(self, x2d):
        gu, dn = self.gate_up_proj, self.down_proj
        if self.recompute and self.training and torch.is_grad_enabled() and self.recompute_eligible:
            return recompute_mlp(x2d, gu, dn)
        if self.recompute_eligible:
            if fused_mlp_ok(x2d, gu, dn):
                return fused_mlp(x2d, gu, dn)
            n1 = overlap_mlp_plan(x2d, gu, dn)
            if n1:
                return overlap_mlp(x2d, gu, dn, n1)
        return dn(swiglu(gu(x2d)))


class LlamaDecoderLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype=None, device=None):
        super().__init__()
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps, dtype, device)
        self.self_attn = LlamaAttention(cfg, dtype, device)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps, dtype, device)
        self.mlp = LlamaMLP(cfg, dtype, device)

    def forward(self, h, res, B: int, S: int, pos=None, cu=None):
        # q|k|v LoRA fold: RMSNorm writes y into the first H columns of the GEMM's extended operand
        y, s = self.input_layernorm(h, res, self.self_attn.qkv_proj.fold_ext())
        a = self.self_attn(y, B, S, pos, cu)
        y2, s2 = self.post_attention_layernorm(a, s)
        return self.mlp(y2), s2


class LlamaForCausalLM(nn.Module):
    """forward(input_ids [B,S], labels [B,S] already shifted (-100 = ignore), n_valid) -> loss."""

    def __init__(self, cfg: ModelConfig, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.config = cfg
        self.dtype = dtype
        H, V = cfg.hidden_size, cfg.vocab_size
        self.embed_tokens = nn.Embedding(V, H, dtype=dtype, device=device)
        self.embed_tokens.weight.requires_grad_(False)
        self.layers = nn.ModuleList([LlamaDecoderLayer(cfg, dtype, device)
                                     for _ in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(H, cfg.rms_norm_eps, dtype, device)
        self.lm_head = Linear(H, V, dtype=dtype, device=device, seg_names=["lm_head"])
        self._ckpt = "none"
        self._ckpt_layers: Optional[int] = None  # recompute only the first N layers (None: all)
        self.unit_gate = None    # engine hook run before each unit (async optimizer offload)
        self.coordinator = None  # ZeRO-3 parameter coordinator (lumen.parallel.zero)

    # --- activation checkpointing --------------------------------------------------------------
    CKPT_POLICIES = ("none", "selective", "full")

    @property
    def gradient_checkpointing(self) -> str:
        """Activation recompute policy: ``"none"``; ``"selective"`` -- every layer keeps its
        activations except the [T, 2F] gate|up output, recomputed by one GEMM in the backward
        (the layer's largest saved tensor: ~35% of its activation memory for ~one extra
        projection GEMM per layer); ``"full"`` -- the reference's per-layer recompute (HF
        ``gradient_checkpointing=True``: the layer input only, the whole forward re-run).
        Assigning True picks ``LUMEN_CKPT_POLICY`` (default ``selective``), False ``none``.
        ``"selective:N"`` / ``"full:N"``: only the first N layers recompute, the others keep
        their activations (Megatron's recompute-num-layers): recompute cost and activation
        saving both scale with N, so ``--gradient_checkpointing auto`` recomputes just the
        layers the HBM budget needs (``memory_plan.pick_checkpointing``).

        A layer whose MLP cannot use the selective recompute (trainable gate|up / down weights,
        or adapters on them) is checkpointed whole instead (``full`` for that layer), so asking
        for checkpointing never silently keeps every activation."""
        n = self._ckpt_layers
        return self._ckpt if n is None or self._ckpt == "none" else f"{self._ckpt}:{n}"

    def selective_eligible(self) -> bool:
        """True when every layer can run the ``selective`` policy as such."""
        return all(l.mlp.recompute_eligible for l in self.layers)

    def _layer_policy(self, layer, i: int = 0) -> str:
        if self._ckpt_layers is not None and i >= self._ckpt_layers:
            return "none"
        if self._ckpt == "selective" and not layer.mlp.recompute_eligible:
            if not getattr(self, "_warned_selective", False):
                self._warned_selective = True
                import sys
                print("[lumen] selective checkpointing: MLP weights are trainable or adapted, "
                      "those layers fall back to full per-layer recompute", file=sys.stderr)
            return "full"
        return self._ckpt

    @gradient_checkpointing.setter
    def gradient_checkpointing(self, v) -> None:
        import os

        if v is True or v == "true":
            v = os.environ.get("LUMEN_CKPT_POLICY", "selective")
        elif v is False or v is None or v == "false":
            v = "none"
        v, n = parse_ckpt_policy(v, self.CKPT_POLICIES)
        L = len(self.layers)
        if n is not None and n >= L:
            n = None
        self._ckpt, self._ckpt_layers = v, n
        for i, layer in enumerate(self.layers):
            layer.mlp.recompute = v == "selective" and (n is None or i < n)

    # --- ZeRO-3 units, in execution order ------------------------------------------------------
    def zero_units(self) -> List[List[nn.Module]]:
        return ([[self.embed_tokens]] + [[l] for l in self.layers] + [[self.norm, self.lm_head]])

    def lora_modules(self):
        for name, m in self.named_modules():
            if isinstance(m, Linear) and m.lora is not None:
                yield name, m

    def init_weights(self, std: float = 0.02, seed: int = 0):
        """Random init (synthetic benches: no checkpoint download): Normal(0, std) like HF,
        norms = 1.  Generated on the parameters' device (fast on GPU), identical on every rank
        for the same seed."""
        init_normal_(self, std, seed)

    def _run_unit(self, idx, fn, *args):
        g = self.unit_gate
        if g is not None:  # async ZeRO-Offload step: this unit's adapters must have landed
            g(idx)
        c = self.coordinator
        if c is None:
            return fn(*args)
        c.pre_forward(idx)
        out = fn(*args)
        return c.post_forward(idx, out)

    supports_packing = True  # forward(..., cu_seqlens=...) runs packed varlen rows

    def hidden_states(self, input_ids: torch.Tensor, pos: Optional[torch.Tensor] = None,
                      cu: Optional[tuple] = None):
        if input_ids.dim() == 1:
            input_ids = input_ids.view(1, -1)
        B, S = input_ids.shape
        if cu is not None:
            cu = tuple(int(c) for c in cu)
            if cu[0] != 0 or cu[-1] != B * S:
                raise ValueError(f"cu_seqlens must span the {B * S} packed tokens, got {cu}")
            if pos is None:
                pos = torch.cat([torch.arange(b - a, dtype=torch.int32) for a, b in
                                 zip(cu[:-1], cu[1:])]).to(input_ids.device)
            if input_ids.is_cuda:
                prepare_varlen(cu, input_ids.device)  # tile lists: one async copy per step
        h = self._run_unit(0, lambda ids: embedding(ids, self.embed_tokens.weight),
                           input_ids.reshape(-1))
        res = None
        for i, layer in enumerate(self.layers):
            if (self._ckpt != "none" and self.training and torch.is_grad_enabled()
                    and self._layer_policy(layer, i) == "full"):
                fn = lambda h_, r_, L=layer: cp.checkpoint(L, h_, r_, B, S, pos, cu, use_reentrant=False)  # noqa: E731
            else:
                fn = lambda h_, r_, L=layer: L(h_, r_, B, S, pos, cu)  # noqa: E731
            h, res = self._run_unit(i + 1, fn, h, res)
        return h, res

    def forward(self, input_ids: torch.Tensor, labels: Optional[torch.Tensor] = None,
                n_valid: Optional[int] = None, pos: Optional[torch.Tensor] = None,
                cu_seqlens: Optional[tuple] = None):
        """``cu_seqlens``: the rows of ``input_ids`` are packed sequences with these offsets
        (lumen.data.PackedCollator); ``pos`` then holds per-sequence positions."""
        if self.training and torch.is_grad_enabled():
            arena_reset(input_ids.device)  # adapter scratch of the previous micro-step is dead
        h, res = self.hidden_states(input_ids, pos, cu_seqlens)
        last = len(self.layers) + 1

        def head(h_, r_):
            y, _ = self.norm(h_, r_)
            if labels is None:
                return torch.matmul(y, self.lm_head.weight.t())
            nv = int(n_valid) if n_valid is not None else int((labels != -100).sum())
            return lm_head_cross_entropy(y, labels.reshape(-1), self.lm_head.weight_fn, nv,
                                         self.lm_head.weight, self.lm_head._wt_fn())

        return self._run_unit(last, head, h, res)


def init_normal_(model: nn.Module, std: float = 0.02, seed: int = 0):
    gens = {}
    with torch.no_grad():
        for name, p in model.named_parameters():
            if "lora_" in name or p.numel() == 0 or p.is_meta:
                continue
            if p.dim() == 1:
                if name.endswith("bias"):
                    p.zero_()
                else:
                    p.fill_(1.0)
                continue
            dev = p.device
            g = gens.get(str(dev))
            if g is None:
                g = torch.Generator(device=dev)
                g.manual_seed(seed)
                gens[str(dev)] = g
            p.normal_(0.0, std, generator=g)
