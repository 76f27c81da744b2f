"""Checkpoint rotation / resume equivalence and the reference-compatible CLIs (CPU)."""
import csv
import os
import socket
import subprocess
import sys

import torch

from lumen.lora import adapter_state_dict
from lumen.parallel.dist import init
from lumen.train.checkpoint import latest_checkpoint, list_checkpoints
from lumen.train.config import load_ds_config
from lumen.train.trainer import TrainArgs, Trainer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trainer(out, max_steps, resume=False, save_steps=2, limit=None):
    env = init(device="cpu")
    ds = load_ds_config({"zero_optimization": {"stage": 1}}, 2, 2, 1, 5e-3, dtype_override="fp32")
    a = TrainArgs(model_name="tiny-llama", synthetic=True, synthetic_samples=40, max_length=16,
                  per_device_train_batch_size=2, gradient_accumulation_steps=2,
                  max_steps=max_steps, logging_steps=1, lora_r=4, lora_dropout=0.05,
                  save_strategy="steps", save_steps=save_steps, save_total_limit=limit,
                  resume_from_checkpoint=resume, output_dir=out, seed=3, save_final=False)
    return Trainer(a, ds, env, printer=lambda *x, **k: None)


def test_resume_is_bit_exact(tmp_path):
    full = _trainer(str(tmp_path / "full"), 6, save_steps=100)
    full.train()
    ref = adapter_state_dict(full.model)

    first = _trainer(str(tmp_path / "part"), 4, save_steps=2)
    first.train()
    assert latest_checkpoint(str(tmp_path / "part")).endswith("checkpoint-4")
    second = _trainer(str(tmp_path / "part"), 6, resume=True, save_steps=100)
    assert second.engine.global_step == 0
    second.train()
    assert second.engine.global_step == 6
    got = adapter_state_dict(second.model)
    for k in ref:
        assert torch.allclose(ref[k], got[k], atol=1e-6), k


def test_checkpoint_layout_and_rotation(tmp_path):
    t = _trainer(str(tmp_path), 6, save_steps=2, limit=2)
    t.train()
    steps = [s for s, _ in list_checkpoints(str(tmp_path))]
    assert steps == [4, 6]
    ck = os.path.join(str(tmp_path), "checkpoint-6")
    for f in ("adapter_model.safetensors", "adapter_config.json", "trainer_state.json",
              "latest", "rng_state_0.pth",
              "global_step6/zero_pp_rank_0_mp_rank_00_optim_states.pt"):
        assert os.path.exists(os.path.join(ck, f)), f
    sd = torch.load(os.path.join(ck, "global_step6/zero_pp_rank_0_mp_rank_00_optim_states.pt"),
                    weights_only=True)
    assert sd["global_step"] == 6


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_cli_opt125m_zero1_gloo_world2(tmp_path):
    """BASELINE.json config 1: OPT-125m LoRA ZeRO-1 on CPU/gloo world_size=2, through the
    reference-compatible entrypoint and launcher."""
    out = str(tmp_path / "ck")
    csvp = str(tmp_path / "metrics.csv")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}",
           os.path.join(ROOT, "training", "train_deepspeed_zero1.py"),
           "--model_name", "facebook/opt-125m", "--synthetic", "--synthetic_samples", "16",
           "--max_length", "32", "--max_steps", "2", "--logging_steps", "1",
           "--per_device_train_batch_size", "1", "--gradient_accumulation_steps", "2",
           "--device", "cpu", "--output_dir", out, "--metrics_csv", csvp,
           "--deepspeed_config", os.path.join(ROOT, "configs", "ds_config_zero1.json")]
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "trainable params: 1,179,648 || all params: 126,418,944" in r.stdout  # 125,239,296 base
    rows = list(csv.DictReader(open(csvp)))
    assert rows[-1]["experiment"] == "zero1_2gpu" and rows[-1]["num_gpus"] == "2"
    assert os.path.exists(os.path.join(out + "_2gpu", "final", "adapter_model.safetensors"))


def test_cli_baseline_single_process(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "training", "train_baseline.py"),
           "--model_name", "tiny-llama", "--synthetic", "--synthetic_samples", "8",
           "--max_length", "16", "--max_steps", "2", "--device", "cpu",
           "--output_dir", str(tmp_path / "b"), "--metrics_csv", str(tmp_path / "m.csv")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT), cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    rows = list(csv.DictReader(open(tmp_path / "m.csv")))
    assert rows[-1]["experiment"] == "baseline" and rows[-1]["strategy"] == "pytorch_lora"


def _zero2_cmd(out, csvp, steps, resume=False):
    cmd = [sys.executable, "-m", "lumen.launch", "--nproc_per_node", "2", "--master_port",
           str(_port()), "--grace", "5", os.path.join(ROOT, "training", "train_deepspeed_zero2.py"),
           "--model_name", "tiny-llama", "--synthetic", "--synthetic_samples", "64",
           "--max_length", "16", "--max_steps", str(steps), "--logging_steps", "1",
           "--per_device_train_batch_size", "2", "--gradient_accumulation_steps", "2",
           "--lora_r", "4", "--save_steps", "2", "--device", "cpu", "--output_dir", out,
           "--metrics_csv", csvp, "--seed", "5",
           "--deepspeed_config", os.path.join(ROOT, "configs", "ds_config_zero2.json")]
    if resume:
        cmd.append("--resume_from_checkpoint")
    return cmd


def test_fault_injection_kill_and_resume_matches(tmp_path):
    """Rank 1 dies after step 3 (LUMEN_FAULT_STEP), the launcher tears rank 0 down, and a resumed
    run from checkpoint-2 ends with the same adapter as an uninterrupted run."""
    from safetensors.torch import load_file

    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    env.pop("HIP_VISIBLE_DEVICES", None)
    csvp = str(tmp_path / "m.csv")
    full = str(tmp_path / "full")
    r = subprocess.run(_zero2_cmd(full, csvp, 6), capture_output=True, text=True, timeout=600,
                       env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]

    part = str(tmp_path / "part")
    fenv = dict(env, LUMEN_FAULT_STEP="3", LUMEN_FAULT_RANK="1")
    r = subprocess.run(_zero2_cmd(part, csvp, 6), capture_output=True, text=True, timeout=600,
                       env=fenv, cwd=ROOT)
    assert r.returncode == 17, (r.returncode, r.stderr[-3000:])
    assert "rank 1 exited with code 17" in r.stderr
    assert latest_checkpoint(part).endswith("checkpoint-2")
    assert not os.path.exists(os.path.join(part, "final"))

    r = subprocess.run(_zero2_cmd(part, csvp, 6, resume=True), capture_output=True, text=True,
                       timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "resumed from" in r.stdout
    a = load_file(os.path.join(full, "final", "adapter_model.safetensors"))
    b = load_file(os.path.join(part, "final", "adapter_model.safetensors"))
    assert a.keys() == b.keys()
    for k in a:
        torch.testing.assert_close(a[k], b[k], rtol=0, atol=1e-6)


def test_async_checkpoint_layout_and_resume(tmp_path):
    """The side-thread writer produces the same layout and resumes bit-exactly."""
    from lumen.train.checkpoint import AsyncCheckpointer

    full = _trainer(str(tmp_path / "full"), 6, save_steps=100)
    full.args.async_save = False
    full.train()
    ref = adapter_state_dict(full.model)
    part = _trainer(str(tmp_path / "part"), 4, save_steps=2, limit=1)
    assert isinstance(part.ckpt, AsyncCheckpointer)
    part.train()
    steps = [s for s, _ in list_checkpoints(str(tmp_path / "part"))]
    assert steps == [4], steps
    ck = latest_checkpoint(str(tmp_path / "part"))
    assert not [f for f in os.listdir(os.path.join(ck, "global_step4")) if f.startswith(".done")]
    second = _trainer(str(tmp_path / "part"), 6, resume=True, save_steps=100)
    second.train()
    got = adapter_state_dict(second.model)
    for k in ref:
        assert torch.allclose(ref[k], got[k], atol=1e-6), k


def test_accumulation_fusion_matches_micro_steps(tmp_path):
    """grad_accum micro-batches with equal valid-token counts run as ONE forward/backward
    (trainer ``fuse_accumulation``): same adapters and logged losses as accumulating them one by
    one (dropout off: the fused forward draws its masks differently)."""
    env = init(device="cpu")
    res = {}
    for fuse in (False, True):
        ds = load_ds_config({"zero_optimization": {"stage": 2}}, 2, 4, 1, 5e-3,
                            dtype_override="fp32")
        a = TrainArgs(model_name="tiny-llama", synthetic=True, synthetic_samples=64, max_length=16,
                      per_device_train_batch_size=2, gradient_accumulation_steps=4, max_steps=3,
                      logging_steps=1, lora_r=4, lora_dropout=0.0, save_strategy="no",
                      output_dir=str(tmp_path / str(fuse)), seed=3, save_final=False,
                      fuse_accumulation=fuse)
        tr = Trainer(a, ds, env, printer=lambda *x, **k: None)
        calls = []
        orig = tr.engine.forward
        tr.engine.forward = lambda b: (calls.append(b.get("micro_steps", 1)), orig(b))[1]
        tr.train()
        res[fuse] = (adapter_state_dict(tr.model), [r["loss"] for r in tr.log_history], calls)
    (a0, l0, c0), (a1, l1, c1) = res[False], res[True]
    assert c0 == [1] * 12 and c1 == [4] * 3
    assert l0 == l1
    # f32 summation order differs (one batch vs four); Adam turns a rounding difference in a
    # near-zero gradient into an update of up to ~lr, so bound outliers by lr and the bulk tightly
    for k in a0:
        d = (a0[k] - a1[k]).abs()
        assert d.max().item() < 5e-3, (k, d.max().item())
        assert (d > 1e-5 + 1e-3 * a0[k].abs()).float().mean().item() < 0.02, k
