"""DS-config parsing, scheduler, loss scaler, collator, sampler, metrics CSV, dataset prep."""
import csv
import json
import math
import os

import pytest
import torch

from lumen.data import CausalLMCollator, ShardedSampler
from lumen.parallel.zero import DynamicLossScaler
from lumen.train.config import load_ds_config, warmup_lr
from lumen.utils.metrics import create_experiment_name, save_training_metrics

# Schema of the reference's configs/ds_config_zero{1,3}.json (values as published there)
REF_Z1 = {"train_batch_size": "auto", "train_micro_batch_size_per_gpu": "auto",
          "gradient_accumulation_steps": "auto",
          "optimizer": {"type": "AdamW", "params": {"lr": "auto", "betas": [0.9, 0.999],
                                                    "eps": 1e-8, "weight_decay": 0.0}},
          "scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0,
                                                       "warmup_max_lr": "auto",
                                                       "warmup_num_steps": "auto"}},
          "fp16": {"enabled": True, "loss_scale": 0, "loss_scale_window": 1000,
                   "initial_scale_power": 16, "hysteresis": 2, "min_loss_scale": 1},
          "zero_optimization": {"stage": 1, "allgather_partitions": True,
                                "allgather_bucket_size": 5e8, "overlap_comm": True,
                                "reduce_scatter": True, "reduce_bucket_size": 5e8,
                                "contiguous_gradients": True},
          "gradient_clipping": 1.0, "steps_per_print": 10, "wall_clock_breakdown": False}
REF_Z3 = {"train_batch_size": "auto", "train_micro_batch_size_per_gpu": "auto",
          "gradient_accumulation_steps": "auto", "gradient_clipping": 1.0,
          "fp16": REF_Z1["fp16"],
          "zero_optimization": {"stage": 3,
                                "offload_optimizer": {"device": "cpu", "pin_memory": True},
                                "offload_param": {"device": "cpu", "pin_memory": True},
                                "overlap_comm": True, "contiguous_gradients": True,
                                "reduce_bucket_size": 5e7, "stage3_prefetch_bucket_size": 5e7,
                                "stage3_param_persistence_threshold": 1e5,
                                "stage3_max_live_parameters": 1e9,
                                "stage3_max_reuse_distance": 1e9,
                                "stage3_gather_16bit_weights_on_model_save": True},
          "optimizer": REF_Z1["optimizer"], "scheduler": REF_Z1["scheduler"]}


def test_reference_zero1_schema_auto_resolution():
    c = load_ds_config(REF_Z1, micro_batch=1, grad_accum=16, world_size=4, learning_rate=2e-4)
    assert c.stage == 1 and c.dtype == "fp16"
    assert c.train_batch_size == 64 and c.micro_batch == 1 and c.grad_accum == 16
    assert c.lr == 2e-4 and c.warmup_max_lr == 2e-4 and c.warmup_num_steps == 0
    assert c.betas == (0.9, 0.999) and c.eps == 1e-8 and c.gradient_clipping == 1.0
    assert c.reduce_bucket_size == 500_000_000 and c.initial_scale_power == 16


def test_reference_zero3_schema():
    c = load_ds_config(REF_Z3, 2, 4, 8, 2e-4)
    assert c.stage == 3 and c.offload_optimizer == "cpu" and c.offload_param == "cpu"
    assert c.stage3_param_persistence_threshold == 100_000
    assert c.stage3_max_live_parameters == 1_000_000_000
    assert c.stage3_gather_16bit_weights_on_model_save
    assert c.train_batch_size == 64


def test_zero2_gradient_clipping_auto_and_bf16(tmp_path):
    p = tmp_path / "c.json"
    p.write_text(json.dumps({"zero_optimization": {"stage": 2}, "bf16": {"enabled": True},
                             "gradient_clipping": "auto"}))
    c = load_ds_config(str(p), 1, 1, 2, 1e-4)
    assert c.dtype == "bf16" and c.gradient_clipping == 1.0 and c.lr == 1e-4


def test_batch_mismatch_raises():
    with pytest.raises(ValueError):
        load_ds_config({"train_batch_size": 7}, 1, 1, 2, 1e-4)


def test_shipped_configs_parse():
    import glob
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for f in glob.glob(os.path.join(root, "configs", "*.json")):
        c = load_ds_config(f, 2, 4, 8, 2e-4)
        assert c.stage in (1, 2, 3)


def test_warmup_lr_log():
    c = load_ds_config({"scheduler": {"params": {"warmup_num_steps": 10}}}, 1, 1, 1, 1.0)
    assert warmup_lr(0, c) == 0.0
    assert abs(warmup_lr(4, c) - math.log(5) / math.log(10)) < 1e-9
    assert warmup_lr(10, c) == 1.0 and warmup_lr(100, c) == 1.0


def test_warmup_lr_auto_matches_deepspeed():
    """The reference configs' "auto" warm-up (HF fills warmup_num_steps = 0): DeepSpeed clamps
    to 2 steps, so optimizer step 0 runs at warmup_min_lr and step 1 on at the full LR."""
    raw = {"scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0,
                                                         "warmup_max_lr": "auto",
                                                         "warmup_num_steps": "auto"}}}
    c = load_ds_config(raw, 1, 1, 1, 2e-4)
    assert warmup_lr(0, c) == 0.0
    assert warmup_lr(1, c) == 2e-4 and warmup_lr(5, c) == 2e-4
    lin = load_ds_config({"scheduler": {"params": {"warmup_num_steps": 1,
                                                   "warmup_type": "linear"}}}, 1, 1, 1, 1.0)
    assert warmup_lr(0, lin) == 0.0 and warmup_lr(1, lin) == 0.5 and warmup_lr(2, lin) == 1.0


def test_lr_schedules_hf_linear_and_deepspeed_constant(tmp_path):
    """No DeepSpeed config (reference train_baseline.py: plain HF Trainer) -> HF's default
    linear schedule: warm-up from 0, then linear decay to 0 at the last step.  DeepSpeed
    configs run WarmupLR, constant after the warm-up, as the reference's ZeRO-2 run logged
    (training/train.ipynb:339-644: 'learning_rate': 0.0002 for 2,856 steps)."""
    c = load_ds_config(None, 1, 1, 1, 2e-4, warmup_steps=0)
    assert c.lr_schedule == "hf_linear"
    c.decay_total_steps = 100
    assert warmup_lr(0, c) == pytest.approx(2e-4)
    assert warmup_lr(50, c) == pytest.approx(1e-4)
    assert warmup_lr(99, c) == pytest.approx(2e-6)
    w = load_ds_config(None, 1, 1, 1, 2e-4, warmup_steps=10)
    w.decay_total_steps = 110
    assert warmup_lr(0, w) == 0.0 and warmup_lr(5, w) == pytest.approx(1e-4)
    assert warmup_lr(10, w) == pytest.approx(2e-4) and warmup_lr(60, w) == pytest.approx(1e-4)
    ds2 = load_ds_config({"zero_optimization": {"stage": 2}}, 1, 1, 1, 2e-4)
    assert ds2.lr_schedule == "warmup"
    assert warmup_lr(0, ds2) == 2e-4 and warmup_lr(5000, ds2) == 2e-4
    # end to end through the trainer (host path on CPU): the logged LR decays to ~0
    from lumen.parallel.dist import init
    from lumen.train.trainer import TrainArgs, Trainer

    a = TrainArgs(model_name="tiny-llama", dataset_path=None, output_dir=str(tmp_path),
                  synthetic=True, synthetic_samples=16, max_length=32, max_steps=4,
                  logging_steps=1, save_strategy="no", init="random", save_final=False)
    ds = load_ds_config(None, 1, 1, 1, 2e-4, dtype_override="fp32")
    tr = Trainer(a, ds, init(), printer=lambda *x, **k: None)
    tr.train()
    lrs = [r["learning_rate"] for r in tr.log_history]
    assert lrs == pytest.approx([2e-4, 1.5e-4, 1e-4, 5e-5])


def test_loss_scaler_deepspeed_semantics():
    s = DynamicLossScaler(2 ** 16, window=3, hysteresis=2)
    s.update(True)  # first overflow absorbed by hysteresis
    assert s.scale == 2 ** 16
    s.update(True)
    assert s.scale == 2 ** 15
    for _ in range(3):
        s.update(False)
    assert s.scale == 2 ** 16
    s2 = DynamicLossScaler(4.0, window=1000, hysteresis=1, min_scale=2.0)
    s2.update(True)
    s2.update(True)
    assert s2.scale == 2.0


def test_collator_pad_eos_and_shift():
    col = CausalLMCollator(pad_id=2)
    b = col([{"input_ids": [1, 5, 6, 2]}, {"input_ids": [1, 7]}])
    assert b["input_ids"].tolist() == [[1, 5, 6, 2], [1, 7, 2, 2]]
    # labels = ids with pad(=eos) masked, then shifted left by one
    assert b["labels"].tolist() == [[5, 6, -100, -100], [7, -100, -100, -100]]
    assert b["n_valid"] == 3 and b["n_tokens"] == 6


def test_sharded_sampler_partition():
    n, W = 11, 3
    parts = [ShardedSampler(n, r, W, seed=42).indices(0) for r in range(W)]
    assert all(len(p) == 4 for p in parts)
    assert set(sum(parts, [])) == set(range(n))
    assert ShardedSampler(n, 0, W, seed=42).indices(1) != parts[0]


def test_experiment_name_and_metrics_csv(tmp_path):
    assert create_experiment_name(1, 0) == "baseline"
    assert create_experiment_name(2, 2) == "zero2_2gpu"
    assert create_experiment_name(4, 3) == "zero3_4gpu"
    p = str(tmp_path / "m.csv")
    base = dict(experiment="baseline", num_gpus=1, zero_stage=0, strategy="pytorch_lora",
                training_time_hours=1.0, samples_per_second=2.0, peak_memory_gb=3.0,
                final_loss=0.5)
    save_training_metrics(base, p)
    save_training_metrics(dict(base, experiment="zero3_8gpu", tokens_per_second=9.0), p)
    rows = list(csv.DictReader(open(p)))
    hdr = list(rows[0].keys())
    assert hdr[:8] == ["experiment", "num_gpus", "zero_stage", "strategy", "training_time_hours",
                       "samples_per_second", "peak_memory_gb", "final_loss"]
    assert rows[1]["tokens_per_second"] == "9.0" and rows[0]["tokens_per_second"] == ""


def test_dropout_mask_rate_and_determinism():
    from lumen.ops.lora import dropout_mask_ref

    m1 = dropout_mask_ref(123, 64, 512, 0.05)
    m2 = dropout_mask_ref(123, 64, 512, 0.05)
    assert torch.equal(m1, m2)
    assert abs(1 - m1.float().mean().item() - 0.05) < 0.005
    assert not torch.equal(m1, dropout_mask_ref(124, 64, 512, 0.05))


def test_stage3_max_live_auto():
    """lumen extension: "auto" live-parameter budget (sized from free HBM by the coordinator)."""
    from lumen.train.config import load_ds_config

    c = load_ds_config({"zero_optimization": {"stage": 3, "stage3_max_live_parameters": "auto"}},
                       1, 1, 1, 1e-4)
    assert c.stage3_max_live_parameters == -1
    c = load_ds_config(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "ds_config_zero3_mi355x.json"), 8, 1, 8, 1e-4)
    assert c.stage3_max_live_parameters == -1 and c.stage == 3


def test_no_scheduler_section_means_constant_lr():
    """A DeepSpeed config without a "scheduler" section builds no WarmupLR: the first optimizer
    step already runs at the full rate (a WarmupLR config starts at warmup_min_lr)."""
    from lumen.train.config import load_ds_config, warmup_lr

    c = load_ds_config({"zero_optimization": {"stage": 1}}, 2, 1, 1, 3e-4)
    assert warmup_lr(0, c) == warmup_lr(1, c) == warmup_lr(100, c) == 3e-4
    w = load_ds_config({"zero_optimization": {"stage": 1},
                        "scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0,
                                                                     "warmup_max_lr": "auto",
                                                                     "warmup_num_steps": "auto"}}},
                       2, 1, 1, 3e-4)
    assert warmup_lr(0, w) == 0.0 and warmup_lr(1, w) == 3e-4


def test_deepspeed_warmup_decay_and_cosine_schedules():
    """DeepSpeed WarmupDecayLR (linear decay to warmup_min_lr at total_num_steps) and
    WarmupCosineLR (ratios of the optimizer lr; cosine to cos_min_ratio), both after the
    WarmupLR warm-up; "auto" total steps come from the trainer's run length."""
    d = load_ds_config({"scheduler": {"type": "WarmupDecayLR", "params": {
        "warmup_min_lr": 1e-5, "warmup_max_lr": 1e-3, "warmup_num_steps": 10,
        "warmup_type": "linear", "total_num_steps": 110}}}, 1, 1, 1, 1e-3)
    assert d.lr_schedule == "warmup_decay" and d.decay_total_steps == 110
    assert warmup_lr(0, d) == pytest.approx(1e-5) and warmup_lr(5, d) == pytest.approx(5.05e-4)
    assert warmup_lr(10, d) == pytest.approx(1e-3)
    assert warmup_lr(60, d) == pytest.approx(1e-5 + (1e-3 - 1e-5) * 0.5)
    assert warmup_lr(110, d) == pytest.approx(1e-5) and warmup_lr(500, d) == pytest.approx(1e-5)
    c = load_ds_config({"optimizer": {"type": "AdamW", "params": {"lr": 2e-4}},
                        "scheduler": {"type": "WarmupCosineLR", "params": {
                            "total_num_steps": "auto", "warmup_min_ratio": 0.1,
                            "warmup_num_steps": 4, "cos_min_ratio": 0.05,
                            "warmup_type": "linear"}}}, 1, 1, 1, 2e-4)
    assert c.lr_schedule == "warmup_cosine" and c.decay_total_steps == 0
    assert warmup_lr(0, c) == pytest.approx(2e-5)
    c.decay_total_steps = 104
    assert warmup_lr(4, c) == pytest.approx(2e-4 * (0.05 + 0.95 * 0.5 * (1 + math.cos(math.pi / 100))))
    assert warmup_lr(53, c) == pytest.approx(2e-4 * (0.05 + 0.95 * 0.5), rel=1e-3)
    assert warmup_lr(103, c) == pytest.approx(2e-4 * 0.05)
    with pytest.raises(ValueError):
        load_ds_config({"scheduler": {"type": "OneCycle"}}, 1, 1, 1, 1e-3)
