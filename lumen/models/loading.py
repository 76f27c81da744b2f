"""HF-format checkpoint IO (safetensors only: nothing from a file is ever executed).

Load: a local HF directory (``config.json`` + ``model*.safetensors`` [+ index]) into lumen's
fused layout (q|k|v and gate|up concatenated).  Save: the inverse, used to export a merged
model (``merged_model/`` of the reference .gitignore:20) for serving.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Dict

import torch
import torch.nn as nn


def _hf_name_map(model) -> Dict[str, tuple]:
    """our param name -> list of (hf name, row slice) composing it (fused rows concatenated)."""
    cfg = model.config
    m = {}
    if cfg.arch == "llama":
        m["embed_tokens.weight"] = [("model.embed_tokens.weight", None)]
        m["norm.weight"] = [("model.norm.weight", None)]
        m["lm_head.weight"] = [("lm_head.weight", None)]
        for i in range(cfg.num_hidden_layers):
            p = f"model.layers.{i}."
            o = f"layers.{i}."
            m[o + "input_layernorm.weight"] = [(p + "input_layernorm.weight", None)]
            m[o + "post_attention_layernorm.weight"] = [(p + "post_attention_layernorm.weight", None)]
            m[o + "self_attn.qkv_proj.weight"] = [(p + f"self_attn.{n}_proj.weight", None) for n in "qkv"]
            m[o + "self_attn.o_proj.weight"] = [(p + "self_attn.o_proj.weight", None)]
            m[o + "mlp.gate_up_proj.weight"] = [(p + "mlp.gate_proj.weight", None),
                                                (p + "mlp.up_proj.weight", None)]
            m[o + "mlp.down_proj.weight"] = [(p + "mlp.down_proj.weight", None)]
    else:  # opt
        d = "model.decoder."
        m["embed_tokens.weight"] = [(d + "embed_tokens.weight", None)]
        m["embed_positions.weight"] = [(d + "embed_positions.weight", None)]
        m["final_layer_norm.weight"] = [(d + "final_layer_norm.weight", None)]
        m["final_layer_norm.bias"] = [(d + "final_layer_norm.bias", None)]
        for i in range(cfg.num_hidden_layers):
            p = f"{d}layers.{i}."
            o = f"layers.{i}."
            for ln in ("self_attn_layer_norm", "final_layer_norm"):
                m[o + ln + ".weight"] = [(p + ln + ".weight", None)]
                m[o + ln + ".bias"] = [(p + ln + ".bias", None)]
            for wb in ("weight", "bias"):
                m[o + f"qkv_proj.{wb}"] = [(p + f"self_attn.{n}_proj.{wb}", None) for n in "qkv"]
                m[o + f"out_proj.{wb}"] = [(p + f"self_attn.out_proj.{wb}", None)]
                m[o + f"fc1.{wb}"] = [(p + f"fc1.{wb}", None)]
                m[o + f"fc2.{wb}"] = [(p + f"fc2.{wb}", None)]
    return m


def _open_all(path: str):
    from safetensors import safe_open

    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    files = [f for f in files if not os.path.basename(f).startswith("adapter_")]
    handles = {}
    for f in files:
        h = safe_open(f, framework="pt", device="cpu")
        for k in h.keys():
            handles[k] = h
    return handles


@torch.no_grad()
def load_hf_weights(model: nn.Module, path: str, strict: bool = True) -> None:
    handles = _open_all(path)
    if not handles:
        raise FileNotFoundError(f"no *.safetensors in {path}")
    params = dict(model.named_parameters())
    for ours, srcs in _hf_name_map(model).items():
        if ours not in params:
            continue
        if not all(s in handles for s, _ in srcs):
            if ours == "lm_head.weight" and "model.embed_tokens.weight" in handles:
                srcs = [("model.embed_tokens.weight", None)]  # tied
            elif strict:
                raise KeyError(f"missing {srcs[0][0]} in {path}")
            else:
                continue
        t = torch.cat([handles[s].get_tensor(s) for s, _ in srcs], 0)
        dst = params[ours]
        if tuple(t.shape) != tuple(dst.shape):
            raise ValueError(f"{ours}: checkpoint {tuple(t.shape)} != model {tuple(dst.shape)}")
        dst.copy_(t.to(dst.dtype))
    from .layers import invalidate_weight_caches

    invalidate_weight_caches(model)


@torch.no_grad()
def save_hf_weights(model: nn.Module, path: str, shard_bytes: int = 5 << 30) -> None:
    """Write an HF-layout safetensors checkpoint + config.json (un-fusing q|k|v, gate|up)."""
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    cfg = model.config
    params = dict(model.named_parameters())
    out: Dict[str, torch.Tensor] = {}
    for ours, srcs in _hf_name_map(model).items():
        if ours not in params:
            continue
        t = params[ours].detach().cpu()
        if len(srcs) == 1:
            out[srcs[0][0]] = t.contiguous()
            continue
        if ours.endswith("qkv_proj.weight") or ours.endswith("qkv_proj.bias"):
            D = cfg.head_dim
            sizes = [cfg.num_attention_heads * D, cfg.num_key_value_heads * D,
                     cfg.num_key_value_heads * D]
        else:
            sizes = [t.shape[0] // 2] * 2
        for (name, _), piece in zip(srcs, torch.split(t, sizes, 0)):
            out[name] = piece.contiguous()
    shards, cur, cur_b = [], {}, 0
    for k, v in out.items():
        nb = v.numel() * v.element_size()
        if cur and cur_b + nb > shard_bytes:
            shards.append(cur)
            cur, cur_b = {}, 0
        cur[k] = v
        cur_b += nb
    if cur:
        shards.append(cur)
    index = {"metadata": {"total_size": sum(v.numel() * v.element_size() for v in out.values())},
             "weight_map": {}}
    for i, sh in enumerate(shards):
        fn = (f"model-{i + 1:05d}-of-{len(shards):05d}.safetensors" if len(shards) > 1
              else "model.safetensors")
        save_file(sh, os.path.join(path, fn), metadata={"format": "pt"})
        for k in sh:
            index["weight_map"][k] = fn
    if len(shards) > 1:
        with open(os.path.join(path, "model.safetensors.index.json"), "w") as f:
            json.dump(index, f, indent=2)
    hf_cfg = _config_to_hf(cfg)
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(hf_cfg, f, indent=2)


def _config_to_hf(cfg) -> dict:
    if cfg.arch == "opt":
        return {"model_type": "opt", "vocab_size": cfg.vocab_size, "hidden_size": cfg.hidden_size,
                "ffn_dim": cfg.ffn_dim, "num_hidden_layers": cfg.num_hidden_layers,
                "num_attention_heads": cfg.num_attention_heads,
                "max_position_embeddings": cfg.max_position_embeddings,
                "word_embed_proj_dim": cfg.word_embed_proj_dim,
                "do_layer_norm_before": True, "pad_token_id": cfg.pad_token_id,
                "bos_token_id": cfg.bos_token_id, "eos_token_id": cfg.eos_token_id}
    return {"model_type": "llama", "architectures": ["LlamaForCausalLM"],
            "vocab_size": cfg.vocab_size, "hidden_size": cfg.hidden_size,
            "intermediate_size": cfg.intermediate_size,
            "num_hidden_layers": cfg.num_hidden_layers,
            "num_attention_heads": cfg.num_attention_heads,
            "num_key_value_heads": cfg.num_key_value_heads,
            "max_position_embeddings": cfg.max_position_embeddings,
            "rms_norm_eps": cfg.rms_norm_eps, "rope_theta": cfg.rope_theta,
            "tie_word_embeddings": cfg.tie_word_embeddings, "bos_token_id": cfg.bos_token_id,
            "eos_token_id": cfg.eos_token_id, "hidden_act": "silu"}
