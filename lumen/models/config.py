"""Model configurations.

The reference fine-tunes ``meta-llama/Llama-2-7b-hf`` loaded through HF transformers
(``training/train_baseline.py:122-126``) and the north-star adds Llama-2-70B and OPT-125m
(``/root/repo/BASELINE.json`` configs).  There is no network on the build or GPU boxes, so
every architecture is described here by its published hyper-parameters and instantiated with
random weights unless a local HF checkpoint directory (``config.json`` + ``*.safetensors``) is
given.
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field, fields
from typing import Optional


@dataclass
class ModelConfig:
    arch: str = "llama"  # "llama" | "opt"
    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 32
    max_position_embeddings: int = 4096
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    tie_word_embeddings: bool = False
    # OPT specifics
    ffn_dim: int = 0
    word_embed_proj_dim: int = 0
    do_layer_norm_before: bool = True
    layer_norm_eps: float = 1e-5
    pad_token_id: int = 0
    bos_token_id: int = 1
    eos_token_id: int = 2
    name: str = "custom"

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads

    @property
    def q_size(self) -> int:
        return self.num_attention_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_key_value_heads * self.head_dim

    def num_params(self) -> int:
        """Total parameter count (base model, no adapters)."""
        h, v, L = self.hidden_size, self.vocab_size, self.num_hidden_layers
        if self.arch == "llama":
            attn = h * (self.q_size + 2 * self.kv_size) + self.q_size * h
            mlp = 3 * h * self.intermediate_size
            norms = 2 * h
            emb = v * h * (1 if self.tie_word_embeddings else 2)
            return L * (attn + mlp + norms) + emb + h
        # OPT: biases + learned positions + layernorms
        f = self.ffn_dim
        attn = 4 * h * h + 4 * h
        mlp = 2 * h * f + f + h
        norms = 4 * h
        return L * (attn + mlp + norms) + v * h + (self.max_position_embeddings + 2) * h + 2 * h

    def to_dict(self):
        return asdict(self)

    def save(self, path: str):
        with open(path, "w") as f:
            json.dump(self.to_dict(), f, indent=2)

    @classmethod
    def from_dict(cls, d: dict) -> "ModelConfig":
        names = {f.name for f in fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})


def _hf_to_config(d: dict) -> ModelConfig:
    mt = d.get("model_type", "llama")
    if mt == "opt":
        return ModelConfig(
            arch="opt", vocab_size=d["vocab_size"], hidden_size=d["hidden_size"],
            intermediate_size=d["ffn_dim"], ffn_dim=d["ffn_dim"],
            num_hidden_layers=d["num_hidden_layers"], num_attention_heads=d["num_attention_heads"],
            num_key_value_heads=d["num_attention_heads"],
            max_position_embeddings=d.get("max_position_embeddings", 2048),
            word_embed_proj_dim=d.get("word_embed_proj_dim", d["hidden_size"]),
            do_layer_norm_before=d.get("do_layer_norm_before", True),
            tie_word_embeddings=True, pad_token_id=d.get("pad_token_id", 1),
            bos_token_id=d.get("bos_token_id", 2), eos_token_id=d.get("eos_token_id", 2),
            name=d.get("_name_or_path", "opt"))
    return ModelConfig(
        arch="llama", vocab_size=d["vocab_size"], hidden_size=d["hidden_size"],
        intermediate_size=d["intermediate_size"], num_hidden_layers=d["num_hidden_layers"],
        num_attention_heads=d["num_attention_heads"],
        num_key_value_heads=d.get("num_key_value_heads", d["num_attention_heads"]),
        max_position_embeddings=d.get("max_position_embeddings", 4096),
        rms_norm_eps=d.get("rms_norm_eps", 1e-5), rope_theta=d.get("rope_theta", 10000.0),
        tie_word_embeddings=d.get("tie_word_embeddings", False),
        bos_token_id=d.get("bos_token_id", 1), eos_token_id=d.get("eos_token_id", 2),
        pad_token_id=d.get("pad_token_id", 0) or 0, name=d.get("_name_or_path", "llama"))


PRESETS = {
    # meta-llama/Llama-2-7b-hf: 6,738,415,616 params
    "llama2-7b": dict(arch="llama", vocab_size=32000, hidden_size=4096, intermediate_size=11008,
                      num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=32,
                      max_position_embeddings=4096, name="meta-llama/Llama-2-7b-hf"),
    "llama2-13b": dict(arch="llama", vocab_size=32000, hidden_size=5120, intermediate_size=13824,
                       num_hidden_layers=40, num_attention_heads=40, num_key_value_heads=40,
                       max_position_embeddings=4096, name="meta-llama/Llama-2-13b-hf"),
    # meta-llama/Llama-2-70b-hf (GQA, 8 kv heads)
    "llama2-70b": dict(arch="llama", vocab_size=32000, hidden_size=8192, intermediate_size=28672,
                       num_hidden_layers=80, num_attention_heads=64, num_key_value_heads=8,
                       max_position_embeddings=4096, name="meta-llama/Llama-2-70b-hf"),
    # Llama-2-7B layer shapes (H, F, heads, vocab) at reduced depth: multi-rank rehearsals with
    # every rank on one shared GPU (8 full 7B ranks would not fit its HBM)
    "llama2-7b-2l": dict(arch="llama", vocab_size=32000, hidden_size=4096, intermediate_size=11008,
                         num_hidden_layers=2, num_attention_heads=32, num_key_value_heads=32,
                         max_position_embeddings=4096, name="llama2-7b-2l"),
    # Llama-2-70B layer shapes (H 8192, GQA 64 / 8 heads, F 28672, vocab 32000) at depth 2:
    # world-8 rehearsals of BASELINE config 5's per-layer shapes on one shared GPU
    "llama2-70b-2l": dict(arch="llama", vocab_size=32000, hidden_size=8192,
                          intermediate_size=28672, num_hidden_layers=2, num_attention_heads=64,
                          num_key_value_heads=8, max_position_embeddings=4096,
                          name="llama2-70b-2l"),
    # facebook/opt-125m
    "opt-125m": dict(arch="opt", vocab_size=50272, hidden_size=768, intermediate_size=3072,
                     ffn_dim=3072, num_hidden_layers=12, num_attention_heads=12,
                     num_key_value_heads=12, max_position_embeddings=2048,
                     word_embed_proj_dim=768, tie_word_embeddings=True, pad_token_id=1,
                     bos_token_id=2, eos_token_id=2, name="facebook/opt-125m"),
    # small test models (CPU unit tests, smoke)
    "tiny-llama": dict(arch="llama", vocab_size=512, hidden_size=256, intermediate_size=688,
                       num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=4,
                       max_position_embeddings=512, name="tiny-llama"),
    # deeper toy model: 8 ZeRO-3 units, so the release ring / prefetch / turn-reuse logic has room
    "tiny-llama-deep": dict(arch="llama", vocab_size=512, hidden_size=128, intermediate_size=344,
                            num_hidden_layers=6, num_attention_heads=4, num_key_value_heads=2,
                            max_position_embeddings=512, name="tiny-llama-deep"),
    # head_dim 128 like Llama-2: exercises the HIP flash-attention / fused-RoPE path at toy size
    "small-llama": dict(arch="llama", vocab_size=1024, hidden_size=512, intermediate_size=1376,
                        num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
                        max_position_embeddings=1024, name="small-llama"),
    "tiny-llama-gqa": dict(arch="llama", vocab_size=512, hidden_size=256, intermediate_size=688,
                           num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
                           max_position_embeddings=512, name="tiny-llama-gqa"),
    # 8 heads / 8 kv heads / FFN and vocab divisible by 8 x 8: tensor parallelism up to 8
    "tiny-llama-tp8": dict(arch="llama", vocab_size=1024, hidden_size=512, intermediate_size=2048,
                           num_hidden_layers=2, num_attention_heads=8, num_key_value_heads=8,
                           max_position_embeddings=512, name="tiny-llama-tp8"),
    "tiny-opt": dict(arch="opt", vocab_size=512, hidden_size=64, intermediate_size=256,
                     ffn_dim=256, num_hidden_layers=2, num_attention_heads=4,
                     num_key_value_heads=4, max_position_embeddings=256, word_embed_proj_dim=64,
                     tie_word_embeddings=True, pad_token_id=1, bos_token_id=2, eos_token_id=2,
                     name="tiny-opt"),
}

# HF hub ids accepted by --model_name, mapped to presets (offline: random init).
HUB_ALIASES = {
    "meta-llama/Llama-2-7b-hf": "llama2-7b",
    "meta-llama/Llama-2-7b-chat-hf": "llama2-7b",
    "meta-llama/Llama-2-13b-hf": "llama2-13b",
    "meta-llama/Llama-2-70b-hf": "llama2-70b",
    "facebook/opt-125m": "opt-125m",
}


def get_config(name_or_path: str) -> ModelConfig:
    """Resolve a preset name, an HF hub id (offline alias) or a local HF checkpoint dir."""
    if name_or_path in PRESETS:
        return ModelConfig(**PRESETS[name_or_path])
    if name_or_path in HUB_ALIASES:
        return ModelConfig(**PRESETS[HUB_ALIASES[name_or_path]])
    if os.path.isdir(name_or_path):
        cfg_path = os.path.join(name_or_path, "config.json")
        with open(cfg_path) as f:
            d = json.load(f)
        if "arch" in d and "model_type" not in d:
            return ModelConfig.from_dict(d)
        return _hf_to_config(d)
    raise ValueError(f"unknown model '{name_or_path}' (presets: {sorted(PRESETS)})")


def checkpoint_dir(name_or_path: str) -> Optional[str]:
    """Local directory holding weights for this model, if any."""
    if os.path.isdir(name_or_path):
        return name_or_path
    return None
