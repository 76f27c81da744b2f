#!/usr/bin/env python
"""Merge a trained LoRA adapter into its base model and export an HF checkpoint.

    python scripts/merge_lora.py --model meta-llama/Llama-2-7b-hf \
        --adapter checkpoints/zero3_8gpu/final --output_dir merged_model

The reference's ``.gitignore:20`` (``merged_model/``) implies PEFT ``merge_and_unload`` before
serving; lumen folds W += (alpha/r) * B @ A for every adapted fused linear in place and writes
sharded safetensors + config.json in the HF layout (q|k|v and gate|up un-fused), which
``lumen.serve`` (and transformers) load directly.  ``--model`` is a local HF dir or a preset
name (random init, offline).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main(argv=None):
    p = argparse.ArgumentParser(description="Merge a PEFT LoRA adapter into the base weights")
    p.add_argument("--model", required=True)
    p.add_argument("--adapter", required=True)
    p.add_argument("--output_dir", default="merged_model")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    p.add_argument("--device", default="cpu")
    a = p.parse_args(argv)
    import torch

    from lumen.lora import load_adapter, merge_lora
    from lumen.models import build_model
    from lumen.models.loading import save_hf_weights

    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    model = build_model(a.model, dtype=dt, device=torch.device(a.device))
    load_adapter(model, a.adapter)
    merge_lora(model)
    save_hf_weights(model, a.output_dir)
    tok_files = [f for f in ("tokenizer.json", "tokenizer.model", "tokenizer_config.json",
                             "special_tokens_map.json") if os.path.isfile(os.path.join(a.adapter, f))]
    for f in tok_files:  # the training CLIs save the tokenizer next to the adapter
        with open(os.path.join(a.adapter, f), "rb") as src, \
                open(os.path.join(a.output_dir, f), "wb") as dst:
            dst.write(src.read())
    print(f"merged {a.adapter} into {a.model} -> {a.output_dir}")
    return a.output_dir


if __name__ == "__main__":
    main()
