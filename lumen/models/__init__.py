"""Model families: Llama / Llama-2 (7B, 13B, 70B-GQA) and OPT (125m)."""
from __future__ import annotations

from typing import Optional

import torch

from .config import PRESETS, ModelConfig, checkpoint_dir, get_config  # noqa: F401
from .llama import LlamaForCausalLM  # noqa: F401
from .opt import OPTForCausalLM  # noqa: F401


def build_model(name_or_cfg, dtype=torch.bfloat16, device=None, init: str = "auto",
                seed: int = 0):
    """Instantiate a model: from a local HF dir (weights loaded) or a preset / hub id (random
    init -- the GPU boxes are offline).  ``init``: auto | random | pretrained."""
    cfg = name_or_cfg if isinstance(name_or_cfg, ModelConfig) else get_config(name_or_cfg)
    cls = LlamaForCausalLM if cfg.arch == "llama" else OPTForCausalLM
    model = cls(cfg, dtype=dtype, device=device)
    ckpt = None if isinstance(name_or_cfg, ModelConfig) else checkpoint_dir(name_or_cfg)
    if init == "pretrained" or (init == "auto" and ckpt is not None):
        if ckpt is None:
            raise FileNotFoundError(f"no local checkpoint for {name_or_cfg}")
        from .loading import load_hf_weights

        load_hf_weights(model, ckpt)
    else:
        model.init_weights(seed=seed)
    return model
