"""Command-line front end shared by the reference-compatible entrypoints.

``training/train_baseline.py`` and ``training/train_deepspeed_zero{1,2,3}.py`` call
``main(variant)``; flags, defaults and output-dir naming follow the reference scripts
(SURVEY 2.7):

  variant   micro accum  output_dir default                      save policy     config flag
  baseline  1     16     ./checkpoints/baseline_1gpu              epoch, keep 2   (none: stage 0)
  zero1     1     16     ./checkpoints/deepspeed_zero1 + _{N}gpu  100 steps, 3    --deepspeed_config
  zero2     1     1      ./checkpoints/zero{stage}_{N}gpu         100 steps, 3    --deepspeed_config
  zero3     2     4      ./checkpoints/zero{stage}_{N}gpu         epoch, keep 2   --deepspeed (req.)

Reference quirks fixed: zero1's default config path points at configs/ (1), the
JSON decides precision (2), every variant writes the metrics row (3), imports work from any cwd
(4), world size comes from the launcher (6), resume resolves on every rank (7), tokens/s is
recorded (8), the visible-device set is validated (12), a CPU/gloo path exists (13).
lumen extras: --synthetic, --max_steps, --max_length, --init, --device, --no_gradient_checkpointing.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

VARIANTS = {
    "baseline": dict(micro=1, accum=16, out="./checkpoints/baseline_1gpu", save="epoch", limit=2,
                     config=None),
    "zero1": dict(micro=1, accum=16, out="./checkpoints/deepspeed_zero1", save="steps", limit=3,
                  config="./configs/ds_config_zero1.json"),
    "zero2": dict(micro=1, accum=1, out=None, save="steps", limit=3,
                  config="./configs/ds_config_zero2.json"),
    "zero3": dict(micro=2, accum=4, out=None, save="epoch", limit=2, config=None),
}


def _ckpt_arg(v: str) -> str:
    """--gradient_checkpointing value: auto | true | false | selective | full, optionally ':N'."""
    base, _, n = v.partition(":")
    if base not in ("auto", "true", "false", "selective", "full") or (
            n and (base not in ("selective", "full") or not n.isdigit())):
        raise argparse.ArgumentTypeError(
            f"invalid choice {v!r}: auto, true, false, selective, full, selective:N or full:N")
    return v


def build_parser(variant: str) -> argparse.ArgumentParser:
    v = VARIANTS[variant]
    ap = argparse.ArgumentParser(description=f"LoRA fine-tuning on MI355X ({variant})")
    ap.add_argument("--model_name", default="meta-llama/Llama-2-7b-hf")
    ap.add_argument("--dataset_path", default="./data/glaive_code_full")
    ap.add_argument("--output_dir", default=v["out"])
    ap.add_argument("--num_train_epochs", type=int, default=3)
    ap.add_argument("--per_device_train_batch_size", type=int, default=v["micro"])
    ap.add_argument("--gradient_accumulation_steps", type=int, default=v["accum"])
    ap.add_argument("--learning_rate", type=float, default=2e-4)
    ap.add_argument("--lora_r", type=int, default=16)
    if variant in ("zero1", "zero2"):
        ap.add_argument("--deepspeed_config", default=v["config"])
    if variant == "zero3":
        ap.add_argument("--deepspeed", required=True, help="DeepSpeed-schema JSON config")
    if variant == "baseline":
        ap.add_argument("--deepspeed_config", default=None,
                        help="(lumen) optional config for precision / optimizer settings")
    ap.add_argument("--resume_from_checkpoint", action="store_true")
    ap.add_argument("--local_rank", type=int, default=-1)
    # lumen extensions
    ap.add_argument("--synthetic", action="store_true", help="random-token dataset (offline)")
    ap.add_argument("--synthetic_samples", type=int, default=1024)
    ap.add_argument("--synthetic_min_len", type=int, default=None,
                    help="variable-length synthetic rows: lengths uniform in [min, max_length]")
    ap.add_argument("--no_packing", action="store_true",
                    help="pad to the longest row (reference collation) instead of packing")
    ap.add_argument("--prefetch", type=int, default=2, help="batches collated ahead (0 = inline)")
    ap.add_argument("--pack_tokens", type=int, default=0,
                    help="token-budget batching: pack whole sequences up to N tokens per "
                         "micro-step (packing only; the micro-batch size is then variable)")
    ap.add_argument("--max_steps", type=int, default=-1)
    ap.add_argument("--max_length", type=int, default=512)
    ap.add_argument("--init", default="auto", choices=["auto", "random", "pretrained"])
    ap.add_argument("--device", default=None, choices=[None, "cpu", "cuda"])
    ap.add_argument("--dtype", default=None, choices=[None, "bf16", "fp16", "fp32"])
    ap.add_argument("--lora_alpha", type=float, default=None)
    ap.add_argument("--lora_dropout", type=float, default=0.05)
    ap.add_argument("--lora_targets", default="q_proj,k_proj,v_proj,o_proj")
    ap.add_argument("--logging_steps", type=int, default=10)
    ap.add_argument("--save_steps", type=int, default=100)
    ap.add_argument("--save_total_limit", type=int, default=v["limit"])
    ap.add_argument("--save_strategy", default=v["save"], choices=["steps", "epoch", "no"])
    ap.add_argument("--warmup_steps", type=int, default=0)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--gradient_checkpointing", default="auto", type=_ckpt_arg,
                    help="activation recompute (the reference always enables it): auto | true | "
                         "false | selective | full | selective:N | full:N.  true = the "
                         "model's default policy (Llama: 'selective', the gate|up output "
                         "recomputed; layers whose MLP is trainable or adapted are recomputed "
                         "whole, as 'full'); full = per-layer recompute like HF; ':N' = only the "
                         "first N layers recompute; auto: only as much recompute as the "
                         "estimated activations need to fit in free HBM (logged)")
    ap.add_argument("--no_gradient_checkpointing", action="store_true",
                    help="same as --gradient_checkpointing false")
    ap.add_argument("--no_fuse_accumulation", action="store_true",
                    help="run every accumulation micro-batch as its own forward / backward")
    ap.add_argument("--metrics_csv", default="results/training_metrics.csv")
    return ap


def main(variant: str, argv=None) -> dict:
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    if root not in sys.path:
        sys.path.insert(0, root)
    args = build_parser(variant).parse_args(argv)
    if args.local_rank >= 0 and "LOCAL_RANK" not in os.environ:
        os.environ["LOCAL_RANK"] = str(args.local_rank)

    from lumen.parallel.dist import init
    from lumen.train.config import find_config, load_ds_config
    from lumen.train.trainer import TrainArgs, Trainer
    from lumen.utils.metrics import (create_experiment_name, print_metrics_summary,
                                     save_training_metrics)

    env = init(device=args.device)
    world = env.world_size
    cfg_path = getattr(args, "deepspeed", None) or getattr(args, "deepspeed_config", None)
    cfg_src = find_config(cfg_path) if cfg_path else None
    dtype = args.dtype
    if dtype is None and env.device.type == "cpu":
        dtype = "fp32"  # CPU/gloo path: no 16-bit GEMM kernels on the host
    ds = load_ds_config(cfg_src, args.per_device_train_batch_size,
                        args.gradient_accumulation_steps, world, args.learning_rate,
                        args.warmup_steps, dtype_override=dtype)
    if variant == "baseline":
        ds.stage = 0
    stage = ds.stage
    experiment = create_experiment_name(world, stage)
    out = args.output_dir
    if variant == "zero1":
        out = f"{out}_{world}gpu"
    elif out is None:
        out = f"./checkpoints/{experiment}"
    if env.is_main:
        print("=" * 70)
        print(f"lumen {variant}: experiment={experiment} world={world} ZeRO-{stage} "
              f"device={env.device} dtype={ds.dtype}")
        print(f"effective batch = {ds.micro_batch} x {ds.grad_accum} x {world} = "
              f"{ds.train_batch_size}")
        print("=" * 70, flush=True)
    targs = TrainArgs(
        model_name=args.model_name, dataset_path=args.dataset_path, output_dir=out,
        num_train_epochs=args.num_train_epochs,
        per_device_train_batch_size=args.per_device_train_batch_size,
        gradient_accumulation_steps=args.gradient_accumulation_steps,
        learning_rate=args.learning_rate, lora_r=args.lora_r, lora_alpha=args.lora_alpha,
        lora_dropout=args.lora_dropout, lora_targets=args.lora_targets.split(","),
        max_length=args.max_length, seed=args.seed, logging_steps=args.logging_steps,
        save_strategy=args.save_strategy, save_steps=args.save_steps,
        save_total_limit=args.save_total_limit,
        gradient_checkpointing=("false" if args.no_gradient_checkpointing
                                else args.gradient_checkpointing),
        resume_from_checkpoint=args.resume_from_checkpoint, max_steps=args.max_steps,
        warmup_steps=args.warmup_steps, synthetic=args.synthetic,
        synthetic_samples=args.synthetic_samples, init=args.init, experiment=experiment,
        synthetic_min_len=args.synthetic_min_len, pack_sequences=not args.no_packing,
        prefetch=args.prefetch, pack_tokens=args.pack_tokens,
        fuse_accumulation=not args.no_fuse_accumulation)
    t0 = time.time()
    trainer = Trainer(targs, ds, env)
    result = trainer.train()
    metrics = {
        "experiment": experiment if variant != "baseline" else "baseline",
        "num_gpus": world,
        "zero_stage": stage,
        "strategy": "pytorch_lora" if variant == "baseline" else f"deepspeed_zero{stage}",
        "training_time_hours": result["training_time_hours"],
        "samples_per_second": result["samples_per_second"],
        "peak_memory_gb": result["peak_memory_gb"],
        "final_loss": result["final_loss"],
        "tokens_per_second": result["tokens_per_second"],
        "tflops_per_gpu": result["tflops_per_gpu"],
    }
    if env.is_main:
        print_metrics_summary(metrics)
        save_training_metrics(metrics, args.metrics_csv)
        print(f"total wall time {time.time() - t0:.1f}s; checkpoints in {out}", flush=True)
    from lumen.parallel.dist import shutdown

    shutdown()
    return metrics
