"""The device-side LR schedule of the fused AdamW (kernels/adamw.hip OptSched) equals the host
formula (lumen.train.config.warmup_lr) step by step for every schedule kind: DeepSpeed WarmupLR,
WarmupDecayLR, WarmupCosineLR and HF's linear warm-up + decay.  With beta1 = beta2 = 0 and a
unit gradient an Adam update moves a parameter by exactly -lr, so the per-step parameter deltas
read the device LR back."""
import pytest
import torch

from lumen.train.config import load_ds_config, warmup_lr

pytestmark = pytest.mark.gpu

KINDS = {"hf_linear": 0, "warmup_decay": 1, "warmup_cosine": 2}


def _cfgs():
    yield load_ds_config({"scheduler": {"type": "WarmupLR", "params": {
        "warmup_min_lr": 1e-5, "warmup_max_lr": 1e-3, "warmup_num_steps": 6}}}, 1, 1, 1, 1e-3)
    yield load_ds_config({"scheduler": {"type": "WarmupDecayLR", "params": {
        "warmup_min_lr": 1e-5, "warmup_max_lr": 1e-3, "warmup_num_steps": 5,
        "warmup_type": "linear", "total_num_steps": 30}}}, 1, 1, 1, 1e-3)
    c = load_ds_config({"optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
                        "scheduler": {"type": "WarmupCosineLR", "params": {
                            "total_num_steps": 30, "warmup_min_ratio": 0.1,
                            "warmup_num_steps": 5, "cos_min_ratio": 0.05}}}, 1, 1, 1, 1e-3)
    yield c
    h = load_ds_config(None, 1, 1, 1, 1e-3, warmup_steps=4)
    h.decay_total_steps = 30
    yield h


@pytest.mark.parametrize("cfg", list(_cfgs()), ids=["WarmupLR", "WarmupDecayLR",
                                                     "WarmupCosineLR", "hf_linear"])
def test_device_lr_matches_host_schedule(cfg):
    from lumen.ops._native import native

    dev = torch.device("cuda")
    n = 64
    p = torch.zeros(n, device=dev)
    g = torch.ones(n, device=dev)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    state = torch.zeros(8, dtype=torch.float32, device=dev)
    state[2] = 1.0
    kind = KINDS.get(cfg.lr_schedule, 0)
    decay = cfg.decay_total_steps if cfg.lr_schedule in KINDS else 0
    sched = [cfg.warmup_min_lr, cfg.warmup_max_lr, float(cfg.warmup_num_steps),
             1.0 if cfg.warmup_type == "linear" else 0.0, 1.0, 0.0, 1000.0, 2.0, 1.0,
             float(decay), float(kind), float(cfg.cos_min_ratio)]
    got = []
    for _ in range(34):
        before = p.clone()
        native().adamw(p, g, m, v, None, 0.0, 0.0, 0.0, 1e-12, 0.0, 1.0, 1.0, 1.0, None, 0.0,
                       state, sched)
        got.append(float((before - p).mean()))
    want = [warmup_lr(k, cfg) for k in range(34)]
    assert got == pytest.approx(want, rel=2e-5, abs=1e-9)
