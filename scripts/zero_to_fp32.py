#!/usr/bin/env python3
"""Consolidate a lumen ZeRO checkpoint into one f32 PEFT adapter (DeepSpeed ``zero_to_fp32.py``
equivalent; SURVEY 2.7 checkpoint layout).

    python scripts/zero_to_fp32.py <checkpoint-N dir> <output dir> [--tag global_stepN]

Reads every rank's ``zero_pp_rank_{r}_mp_rank_00_optim_states.pt`` (any world size, any ZeRO
stage), reassembles the f32 master weights by parameter name and writes
``adapter_model.safetensors`` (f32, PEFT key names) + ``adapter_config.json`` to the output dir,
and ``optimizer_fp32.pt`` (per-parameter exp_avg / exp_avg_sq, weights_only-loadable).  No GPU
and no base weights are needed: the model skeleton is built on the meta device.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("checkpoint_dir")
    ap.add_argument("output_dir")
    ap.add_argument("--tag", default=None, help="global_stepN dir (default: the 'latest' file)")
    a = ap.parse_args(argv)

    import torch
    import torch.nn as nn

    from lumen.lora import adapter_state_dict, apply_lora, read_adapter_config, save_adapter
    from lumen.models import LlamaForCausalLM, OPTForCausalLM, get_config
    from lumen.train.reshard import consolidate

    tag = a.tag
    if tag is None:
        with open(os.path.join(a.checkpoint_dir, "latest")) as f:
            tag = f.read().strip()
    params = consolidate(os.path.join(a.checkpoint_dir, tag))
    with open(os.path.join(a.checkpoint_dir, "adapter_config.json")) as f:
        base = json.load(f).get("base_model_name_or_path", "")
    lcfg = read_adapter_config(a.checkpoint_dir)
    cfg = get_config(base)
    cls = LlamaForCausalLM if cfg.arch == "llama" else OPTForCausalLM
    model = cls(cfg, dtype=torch.bfloat16, device="meta")   # skeleton only: no base weights
    apply_lora(model, lcfg)
    model.lora_config = lcfg
    for name, st in params.items():
        mod_name, pname = name.rsplit(".", 1)
        mod = model.get_submodule(mod_name)
        shape = getattr(mod, pname).shape
        setattr(mod, pname, nn.Parameter(st["master"].view(shape), requires_grad=False))
    os.makedirs(a.output_dir, exist_ok=True)
    save_adapter(model, a.output_dir, base, state=adapter_state_dict(model))
    torch.save({n: {"exp_avg": st["exp_avg"], "exp_avg_sq": st["exp_avg_sq"]}
                for n, st in params.items()}, os.path.join(a.output_dir, "optimizer_fp32.pt"))
    ts = os.path.join(a.checkpoint_dir, "trainer_state.json")
    if os.path.exists(ts):
        shutil.copy(ts, os.path.join(a.output_dir, "trainer_state.json"))
    n = sum(st["master"].numel() for st in params.values())
    print(f"[zero_to_fp32] {len(params)} tensors, {n:,} f32 params from {tag} -> {a.output_dir}")


if __name__ == "__main__":
    main()
