"""OPT decoder (facebook/opt-125m), the model of BASELINE.json config 1
("OPT-125m LoRA ZeRO-1 on CPU/gloo world_size=2").

Architecture per transformers' OPTForCausalLM (pre-LN variant used by opt-125m): learned
positions with offset 2, q/k/v/out_proj with bias (q|k|v fused here), LayerNorm, ReLU FFN
fc1/fc2, final LayerNorm, LM head tied to the token embedding.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.utils.checkpoint as cp

from ..ops.embedding import embedding
from ..ops.lora import arena_reset
from ..ops._native import use_native
from ..ops.attention import causal_attention, flash_attention_qkv
from ..ops.loss import lm_head_cross_entropy
from ..ops.norm import layer_norm
from .config import ModelConfig
from .layers import Linear
from .llama import init_normal_


class OPTDecoderLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype=None, device=None):
        super().__init__()
        H, Fd = cfg.hidden_size, cfg.ffn_dim or cfg.intermediate_size
        self.cfg = cfg
        self.self_attn_layer_norm = nn.LayerNorm(H, dtype=dtype, device=device)
        self.qkv_proj = Linear(H, 3 * H, bias=True, dtype=dtype, device=device,
                               seg_sizes=[H, H, H], seg_names=["q_proj", "k_proj", "v_proj"])
        self.out_proj = Linear(H, H, bias=True, dtype=dtype, device=device,
                               seg_names=["out_proj"])
        self.final_layer_norm = nn.LayerNorm(H, dtype=dtype, device=device)
        self.fc1 = Linear(H, Fd, bias=True, dtype=dtype, device=device, seg_names=["fc1"])
        self.fc2 = Linear(Fd, H, bias=True, dtype=dtype, device=device, seg_names=["fc2"])
        for p in self.parameters():
            p.requires_grad_(False)

    def forward(self, h, B: int, S: int, cu=None):
        c = self.cfg
        nh, D = c.num_attention_heads, c.head_dim
        ln1, ln2 = self.self_attn_layer_norm, self.final_layer_norm
        x = layer_norm(h, ln1.weight, ln1.bias, ln1.eps)
        qkv2d = self.qkv_proj(x)
        if qkv2d.is_cuda and use_native(qkv2d):
            # HIP flash attention straight from the fused token-major q|k|v rows (head dim 64
            # runs zero-padded to the kernels' 128, lumen.ops.attention._flash_padded)
            cu_ = cu if cu is not None else tuple(range(0, B * S + 1, S))
            o = flash_attention_qkv(qkv2d, cu_, nh, nh, D, True)
        elif cu is not None:  # packed rows, portable path: one causal block per sequence
            outs = []
            for s0, s1 in zip(cu[:-1], cu[1:]):
                t = qkv2d[s0:s1].view(1, s1 - s0, 3, nh, D)
                outs.append(causal_attention(t[:, :, 0].transpose(1, 2), t[:, :, 1].transpose(1, 2),
                                             t[:, :, 2].transpose(1, 2)))
            o = torch.cat(outs, 0)
        else:
            qkv = qkv2d.view(B, S, 3, nh, D)
            o = causal_attention(qkv[:, :, 0].transpose(1, 2), qkv[:, :, 1].transpose(1, 2),
                                 qkv[:, :, 2].transpose(1, 2))
        h = h + self.out_proj(o)
        x = layer_norm(h, ln2.weight, ln2.bias, ln2.eps)
        return h + self.fc2(F.relu(self.fc1(x)))


class OPTForCausalLM(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype=torch.float32, device=None):
        super().__init__()
        self.config = cfg
        self.dtype = dtype
        H, V = cfg.hidden_size, cfg.vocab_size
        self.embed_tokens = nn.Embedding(V, H, dtype=dtype, device=device)
        self.embed_positions = nn.Embedding(cfg.max_position_embeddings + 2, H, dtype=dtype,
                                           device=device)
        self.layers = nn.ModuleList([OPTDecoderLayer(cfg, dtype, device)
                                     for _ in range(cfg.num_hidden_layers)])
        self.final_layer_norm = nn.LayerNorm(H, dtype=dtype, device=device)
        for p in self.parameters():
            p.requires_grad_(False)
        self.gradient_checkpointing = False
        self.unit_gate = None    # engine hook run before each unit (async optimizer offload)
        self.coordinator = None

    def zero_units(self) -> List[List[nn.Module]]:
        return ([[self.embed_tokens, self.embed_positions]] + [[l] for l in self.layers]
                + [[self.final_layer_norm, self.embed_tokens]])  # tied head: depends on unit 0

    def lora_modules(self):
        for name, m in self.named_modules():
            if isinstance(m, Linear) and m.lora is not None:
                yield name, m

    def init_weights(self, std: float = 0.02, seed: int = 0):
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

    def forward(self, input_ids: torch.Tensor, labels: Optional[torch.Tensor] = None,
                n_valid: Optional[int] = None, pos: Optional[torch.Tensor] = None,
                cu_seqlens: Optional[tuple] = None):
        if self.training and torch.is_grad_enabled():
            arena_reset(input_ids.device)  # adapter scratch of the previous micro-step is dead
        if input_ids.dim() == 1:
            input_ids = input_ids.view(1, -1)
        B, S = input_ids.shape
        cu = tuple(int(c) for c in cu_seqlens) if cu_seqlens is not None else None
        if pos is None:
            if cu is not None:
                pos = torch.cat([torch.arange(b - a) for a, b in zip(cu[:-1], cu[1:])]).to(
                    input_ids.device)
            else:
                pos = torch.arange(S, device=input_ids.device).expand(B, S)
        pos = pos.long().reshape(B, S)

        def embed(ids, p):
            return (embedding(ids, self.embed_tokens.weight)
                    + embedding(p + 2, self.embed_positions.weight)).reshape(B * S, -1)

        h = self._run_unit(0, embed, input_ids, pos)
        for i, layer in enumerate(self.layers):
            if self.gradient_checkpointing and self.training and torch.is_grad_enabled():
                fn = lambda h_, L=layer: cp.checkpoint(L, h_, B, S, cu, use_reentrant=False)  # noqa: E731
            else:
                fn = lambda h_, L=layer: L(h_, B, S, cu)  # noqa: E731
            h = self._run_unit(i + 1, fn, h)
        last = len(self.layers) + 1

        def head(h_):
            fl = self.final_layer_norm
            y = layer_norm(h_, fl.weight, fl.bias, fl.eps)
            wfn = lambda: self.embed_tokens.weight  # noqa: E731  (tied head)
            if labels is None:
                return torch.matmul(y, wfn().t())
            nv = int(n_valid) if n_valid is not None else int((labels != -100).sum())
            return lm_head_cross_entropy(y, labels.reshape(-1), wfn, nv, None)

        return self._run_unit(last, head, h)
