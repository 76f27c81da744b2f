"""LoRA adapters with a PEFT-compatible on-disk format (no peft import: not installed).

Reference: ``LoraConfig(task_type=CAUSAL_LM, r=lora_r, lora_alpha=2*lora_r, lora_dropout=0.05,
target_modules=[q_proj,k_proj,v_proj,o_proj], bias="none")`` + ``get_peft_model`` +
``print_trainable_parameters`` (training/train_baseline.py:131-141) and
``trainer.save_model(final)`` which writes ``adapter_config.json`` + ``adapter_model.safetensors``
with keys ``base_model.model.model.layers.{i}.self_attn.{q,k,v,o}_proj.lora_{A,B}.weight``
(training/train_baseline.py:226-228).
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from ..models.layers import Linear

DEFAULT_TARGETS = ["q_proj", "k_proj", "v_proj", "o_proj"]
_OPT_ALIASES = {"o_proj": "out_proj"}


@dataclass
class LoraConfig:
    r: int = 16
    lora_alpha: Optional[float] = None  # reference: 2 * r
    lora_dropout: float = 0.05
    target_modules: List[str] = field(default_factory=lambda: list(DEFAULT_TARGETS))
    bias: str = "none"
    task_type: str = "CAUSAL_LM"

    def __post_init__(self):
        if self.lora_alpha is None:
            self.lora_alpha = 2 * self.r


def _hf_prefix(model) -> str:
    return "model.decoder." if model.config.arch == "opt" else "model."


def _targets_for(model, targets: List[str]) -> List[str]:
    if model.config.arch == "opt":
        return [_OPT_ALIASES.get(t, t) for t in targets]
    return list(targets)


def apply_lora(model: nn.Module, cfg: LoraConfig) -> nn.Module:
    """Freeze the base model and attach adapters to every fused linear holding a target
    segment.  Returns the model (adapters are f32 parameters, the only trainable ones)."""
    for p in model.parameters():
        p.requires_grad_(False)
    targets = set(_targets_for(model, cfg.target_modules))
    for name, m in model.named_modules():
        if not isinstance(m, Linear) or name.endswith("lm_head"):
            continue
        hit = [n for n in m.seg_names if n in targets]
        if not hit:
            # non-fused single-projection modules are addressed by their own attribute name
            leaf = name.split(".")[-1]
            if leaf in targets and len(m.seg_names) == 1:
                m.seg_names = [leaf]
                hit = [leaf]
        if hit:
            m.add_lora(hit, cfg.r, float(cfg.lora_alpha), cfg.lora_dropout)
    model.lora_config = cfg
    return model


def count_parameters(model: nn.Module):
    trainable = sum(p.numel() for p in model.parameters() if p.requires_grad)
    total = 0
    for p in model.parameters():
        total += int(torch.Size(getattr(p, "_zero_shape", p.shape)).numel())
    return trainable, total


def print_trainable_parameters(model: nn.Module, printer=print):
    t, a = count_parameters(model)
    printer(f"trainable params: {t:,d} || all params: {a:,d} || trainable%: {100 * t / a:.4f}")
    return t, a


def _peft_key(model, module_name: str, seg_name: str, which: str) -> str:
    parts = module_name.split(".")
    parts[-1] = seg_name
    if model.config.arch == "opt" and seg_name in ("q_proj", "k_proj", "v_proj", "out_proj"):
        parts.insert(-1, "self_attn")  # HF OPTAttention lives under .self_attn
    return f"base_model.model.{_hf_prefix(model)}{'.'.join(parts)}.lora_{which}.weight"


def adapter_state_dict(model: nn.Module) -> Dict[str, torch.Tensor]:
    sd = {}
    for name, m in model.named_modules():
        if isinstance(m, Linear) and m.lora is not None:
            for seg in m.lora.names:
                A, B = m.lora.segment(seg)
                sd[_peft_key(model, name, seg, "A")] = A.detach().float().cpu().contiguous()
                sd[_peft_key(model, name, seg, "B")] = B.detach().float().cpu().contiguous()
    return sd


def save_adapter(model: nn.Module, path: str, base_model_name: str = "",
                 state: Optional[Dict[str, torch.Tensor]] = None) -> None:
    """PEFT layout; ``state`` = a precomputed (e.g. host-side snapshot) adapter_state_dict."""
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    cfg: LoraConfig = getattr(model, "lora_config", LoraConfig())
    save_file(state if state is not None else adapter_state_dict(model),
              os.path.join(path, "adapter_model.safetensors"), metadata={"format": "pt"})
    conf = {
        "alpha_pattern": {}, "auto_mapping": None, "base_model_name_or_path": base_model_name,
        "bias": cfg.bias, "fan_in_fan_out": False, "inference_mode": True,
        "init_lora_weights": True, "layer_replication": None, "layers_pattern": None,
        "layers_to_transform": None, "loftq_config": {}, "lora_alpha": cfg.lora_alpha,
        "lora_dropout": cfg.lora_dropout, "megatron_config": None,
        "megatron_core": "megatron.core", "modules_to_save": None, "peft_type": "LORA",
        "r": cfg.r, "rank_pattern": {}, "revision": None,
        "target_modules": sorted(set(cfg.target_modules)), "task_type": cfg.task_type,
        "use_dora": False, "use_rslora": False,
    }
    with open(os.path.join(path, "adapter_config.json"), "w") as f:
        json.dump(conf, f, indent=2)


def read_adapter_config(path: str) -> LoraConfig:
    with open(os.path.join(path, "adapter_config.json")) as f:
        c = json.load(f)
    return LoraConfig(r=int(c["r"]), lora_alpha=float(c["lora_alpha"]),
                      lora_dropout=float(c.get("lora_dropout", 0.0)),
                      target_modules=list(c["target_modules"]), bias=c.get("bias", "none"),
                      task_type=c.get("task_type", "CAUSAL_LM"))


def load_adapter(model: nn.Module, path: str, apply: bool = True, strict: bool = True) -> nn.Module:
    """Load a PEFT adapter dir into `model` (attaching adapters first when `apply`)."""
    from safetensors.torch import load_file

    cfg = read_adapter_config(path)
    if apply and not any(isinstance(m, Linear) and m.lora is not None for m in model.modules()):
        apply_lora(model, cfg)
    sd = load_file(os.path.join(path, "adapter_model.safetensors"))
    used = set()
    with torch.no_grad():
        for name, m in model.named_modules():
            if isinstance(m, Linear) and m.lora is not None:
                for seg in m.lora.names:
                    A, B = m.lora.segment(seg)
                    ka, kb = _peft_key(model, name, seg, "A"), _peft_key(model, name, seg, "B")
                    if ka in sd:
                        A.copy_(sd[ka].to(A.dtype))
                        B.copy_(sd[kb].to(B.dtype))
                        used.update((ka, kb))
                    elif strict:
                        raise KeyError(f"adapter is missing {ka}")
    if strict and set(sd) - used:
        raise KeyError(f"unexpected adapter keys: {sorted(set(sd) - used)[:4]}")
    return model


def merge_lora(model: nn.Module) -> nn.Module:
    """Fold every adapter into its base weight (PEFT merge_and_unload)."""
    for m in model.modules():
        if isinstance(m, Linear) and m.lora is not None:
            m.merge_lora()
    return model
