"""DeepSpeed-JSON compatible config parsing with "auto" resolution.

The reference hands ``configs/ds_config_zero{1,2,3}.json`` to HF's TrainingArguments, which
fills every ``"auto"`` from its own arguments (reference training/train_deepspeed_zero1.py:233;
schema: configs/ds_config_zero1.json:1-49, zero2.json:2-42, zero3.json:1-57).  lumen parses the
same schema itself (no DeepSpeed / transformers import) and resolves "auto" from the CLI:
  train_batch_size = micro * accum * world; train_micro_batch_size_per_gpu = micro;
  gradient_accumulation_steps = accum; optimizer.lr / scheduler.warmup_max_lr = learning_rate;
  scheduler.warmup_num_steps = warmup_steps; gradient_clipping "auto" = 1.0 (HF max_grad_norm).
Precision: the JSON is authoritative (fixes reference quirk 2): ``bf16.enabled`` (MI355X
default) or ``fp16.enabled`` (dynamic loss scaling), else f32.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, Optional, Tuple


def _auto(v, default):
    return default if (v is None or v == "auto") else v


@dataclass
class DSConfig:
    stage: int = 0
    dtype: str = "bf16"               # bf16 | fp16 | fp32
    # fp16 dynamic loss scaling
    loss_scale: float = 0.0           # 0 = dynamic
    initial_scale_power: int = 16
    loss_scale_window: int = 1000
    hysteresis: int = 2
    min_loss_scale: float = 1.0
    # optimizer
    lr: float = 2e-4
    betas: Tuple[float, float] = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.0
    # scheduler (WarmupLR)
    warmup_min_lr: float = 0.0
    warmup_max_lr: float = 2e-4
    warmup_num_steps: int = 0
    warmup_type: str = "log"
    # "warmup": DeepSpeed WarmupLR (constant after the warm-up: every reference DeepSpeed config
    # has a WarmupLR section, and its ZeRO-2 run logged 'learning_rate': 0.0002 for 2,856 steps,
    # training/train.ipynb:339-644; a config without one runs at a constant LR).
    # "hf_linear": no DeepSpeed config at all (the
    # reference train_baseline.py's plain HF Trainer): linear warm-up, then linear decay to 0 at
    # ``decay_total_steps`` (transformers get_linear_schedule_with_warmup; set by the trainer
    # once the run length is known)
    lr_schedule: str = "warmup"
    decay_total_steps: int = 0
    # DeepSpeed WarmupDecayLR ("warmup_decay") / WarmupCosineLR ("warmup_cosine"): the decay
    # horizon is the scheduler's total_num_steps ("auto": the run length, set by the trainer)
    cos_min_ratio: float = 0.0
    gradient_clipping: float = 1.0
    # batch
    train_batch_size: int = 1
    micro_batch: int = 1
    grad_accum: int = 1
    # zero
    overlap_comm: bool = True
    reduce_scatter: bool = True
    contiguous_gradients: bool = True
    reduce_bucket_size: int = int(5e8)
    allgather_bucket_size: int = int(5e8)
    offload_optimizer: str = "none"
    offload_optimizer_pin: bool = True
    offload_param: str = "none"
    offload_param_pin: bool = True
    stage3_prefetch_bucket_size: int = int(5e7)
    stage3_param_persistence_threshold: int = int(1e5)
    stage3_max_live_parameters: int = int(1e9)
    stage3_max_reuse_distance: int = int(1e9)
    stage3_gather_16bit_weights_on_model_save: bool = False
    steps_per_print: int = 10
    wall_clock_breakdown: bool = False
    raw: Dict[str, Any] = field(default_factory=dict)

    @property
    def torch_dtype(self):
        import torch
        return {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[self.dtype]


def load_ds_config(src, micro_batch: int, grad_accum: int, world_size: int,
                   learning_rate: float, warmup_steps: int = 0,
                   max_grad_norm: float = 1.0, dtype_override: Optional[str] = None) -> DSConfig:
    if isinstance(src, dict):
        raw = dict(src)
    elif src is None:
        raw = {}
    else:
        with open(src) as f:
            raw = json.load(f)
    c = DSConfig(raw=raw)
    z = raw.get("zero_optimization", {}) or {}
    c.stage = int(z.get("stage", 0))
    fp16 = raw.get("fp16", {}) or {}
    bf16 = raw.get("bf16", raw.get("bfloat16", {})) or {}
    if bf16.get("enabled", False) is True:
        c.dtype = "bf16"
    elif fp16.get("enabled", False) is True:
        c.dtype = "fp16"
    elif raw:
        c.dtype = "fp32" if ("fp16" in raw or "bf16" in raw) else "bf16"
    if dtype_override:
        c.dtype = dtype_override
    c.loss_scale = float(fp16.get("loss_scale", 0))
    c.initial_scale_power = int(fp16.get("initial_scale_power", 16))
    c.loss_scale_window = int(fp16.get("loss_scale_window", 1000))
    c.hysteresis = int(fp16.get("hysteresis", 2))
    c.min_loss_scale = float(fp16.get("min_loss_scale", 1))
    opt = (raw.get("optimizer", {}) or {}).get("params", {}) or {}
    c.lr = float(_auto(opt.get("lr"), learning_rate))
    c.betas = tuple(_auto(opt.get("betas"), (0.9, 0.999)))
    c.eps = float(_auto(opt.get("eps"), 1e-8))
    c.weight_decay = float(_auto(opt.get("weight_decay"), 0.0))
    sch = raw.get("scheduler", {}) or {}
    sp = sch.get("params", {}) or {}
    c.warmup_min_lr = float(_auto(sp.get("warmup_min_lr"), 0.0))
    c.warmup_max_lr = float(_auto(sp.get("warmup_max_lr"), c.lr))
    c.warmup_num_steps = int(_auto(sp.get("warmup_num_steps"), warmup_steps))
    c.warmup_type = sp.get("warmup_type", "log")
    kind = sch.get("type", "WarmupLR")
    if kind not in ("WarmupLR", "WarmupDecayLR", "WarmupCosineLR"):
        raise ValueError(f"scheduler type {kind!r}: WarmupLR, WarmupDecayLR or WarmupCosineLR")
    if kind in ("WarmupDecayLR", "WarmupCosineLR"):
        c.lr_schedule = "warmup_decay" if kind == "WarmupDecayLR" else "warmup_cosine"
        c.decay_total_steps = int(_auto(sp.get("total_num_steps"), 0))
        if kind == "WarmupCosineLR":   # ratios of the optimizer's lr
            c.warmup_max_lr = c.lr
            c.warmup_min_lr = float(sp.get("warmup_min_ratio", 0.0)) * c.lr
            c.cos_min_ratio = float(sp.get("cos_min_ratio", 1e-4))
    if not raw:
        c.lr_schedule = "hf_linear"
        c.warmup_min_lr, c.warmup_max_lr = 0.0, c.lr
    elif not sch and not warmup_steps:
        # no "scheduler" section and no warm-up asked for: DeepSpeed builds no WarmupLR (HF's
        # default schedule with 0 warm-up steps also starts at the full rate), so the first step
        # runs at the full rate -- not WarmupLR's lr = warmup_min_lr
        c.warmup_min_lr = c.warmup_max_lr = c.lr
    c.gradient_clipping = float(_auto(raw.get("gradient_clipping"), max_grad_norm))
    c.micro_batch = int(_auto(raw.get("train_micro_batch_size_per_gpu"), micro_batch))
    c.grad_accum = int(_auto(raw.get("gradient_accumulation_steps"), grad_accum))
    c.train_batch_size = int(_auto(raw.get("train_batch_size"),
                                   c.micro_batch * c.grad_accum * world_size))
    if c.train_batch_size != c.micro_batch * c.grad_accum * world_size:
        raise ValueError(
            f"train_batch_size {c.train_batch_size} != micro {c.micro_batch} x accum "
            f"{c.grad_accum} x world {world_size}")
    c.overlap_comm = bool(z.get("overlap_comm", True))
    c.reduce_scatter = bool(z.get("reduce_scatter", True))
    c.contiguous_gradients = bool(z.get("contiguous_gradients", True))
    c.reduce_bucket_size = int(float(_auto(z.get("reduce_bucket_size"), 5e8)))
    c.allgather_bucket_size = int(float(_auto(z.get("allgather_bucket_size"), 5e8)))
    oo = z.get("offload_optimizer", {}) or {}
    op = z.get("offload_param", {}) or {}
    c.offload_optimizer = str(oo.get("device", "none") or "none")
    c.offload_optimizer_pin = bool(oo.get("pin_memory", True))
    c.offload_param = str(op.get("device", "none") or "none")
    c.offload_param_pin = bool(op.get("pin_memory", True))
    c.stage3_prefetch_bucket_size = int(float(_auto(z.get("stage3_prefetch_bucket_size"), 5e7)))
    c.stage3_param_persistence_threshold = int(float(_auto(
        z.get("stage3_param_persistence_threshold"), 1e5)))
    # "auto" (lumen extension): size the live-parameter budget from free HBM at engine start
    # (-1 here; resolved by the ZeRO-3 coordinator once the shards exist)
    c.stage3_max_live_parameters = (-1 if z.get("stage3_max_live_parameters") == "auto" else
                                    int(float(z.get("stage3_max_live_parameters", 1e9))))
    c.stage3_max_reuse_distance = int(float(_auto(z.get("stage3_max_reuse_distance"), 1e9)))
    c.stage3_gather_16bit_weights_on_model_save = bool(
        z.get("stage3_gather_16bit_weights_on_model_save", False))
    c.steps_per_print = int(raw.get("steps_per_print", 10))
    c.wall_clock_breakdown = bool(raw.get("wall_clock_breakdown", False))
    return c


def zero_stage_from_config(path: str) -> int:
    """Reference training/utils.py:36-48 (``get_zero_stage_from_config``)."""
    with open(path) as f:
        return int(json.load(f)["zero_optimization"]["stage"])


def warmup_lr(step: int, c: DSConfig) -> float:
    """DeepSpeed WarmupLR (log warm-up by default) as used by every reference config.

    DeepSpeed clamps the warm-up length to ``max(2, warmup_num_steps)`` and the first optimizer
    step runs at iteration 0, i.e. at ``warmup_min_lr`` (gamma = log(1) = 0); with the "auto"
    configs (HF fills ``warmup_num_steps`` = 0) every later step runs at ``warmup_max_lr``.
    ``hf_linear`` (no DeepSpeed config): HF's linear warm-up / linear decay to 0."""
    if c.lr_schedule == "hf_linear" and c.decay_total_steps > 0:
        w, T = c.warmup_num_steps, c.decay_total_steps
        if step < w:
            return c.warmup_max_lr * step / w
        return c.warmup_max_lr * max(0.0, (T - step) / max(1, T - w))
    n = max(2, c.warmup_num_steps)
    if c.lr_schedule in ("warmup_decay", "warmup_cosine") and c.decay_total_steps > 0 and step >= n:
        import math
        T = c.decay_total_steps
        if c.lr_schedule == "warmup_decay":
            return c.warmup_min_lr + (c.warmup_max_lr - c.warmup_min_lr) * max(
                0.0, (T - step) / max(1, T - n))
        r = 0.5 * (1 + math.cos(math.pi * (step - n + 1) / max(1, T - n)))
        return c.warmup_max_lr * max(0.0, c.cos_min_ratio + (1 - c.cos_min_ratio) * r)
    if step >= n:
        return c.warmup_max_lr
    if c.warmup_type == "linear":
        gamma = step / n
    else:
        import math
        gamma = math.log(step + 1) / math.log(n)
    return c.warmup_min_lr + (c.warmup_max_lr - c.warmup_min_lr) * gamma


def find_config(path: str) -> str:
    """Resolve a config path relative to cwd, the repo root, or configs/ (reference quirk 1)."""
    if os.path.exists(path):
        return path
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    for cand in (os.path.join(root, path), os.path.join(root, "configs", os.path.basename(path))):
        if os.path.exists(cand):
            return cand
    raise FileNotFoundError(path)
