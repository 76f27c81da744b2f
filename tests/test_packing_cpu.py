"""Sequence packing (lumen.data.PackedCollator + varlen model path) against the padded batch:
same labels, same loss, same adapter gradients; background collation; trainer end to end."""
import math

import torch

from lumen.data import CausalLMCollator, PackedCollator, PrefetchLoader


def _examples():
    g = torch.Generator().manual_seed(0)
    lens = [7, 3, 12, 1, 9]
    ex = [{"input_ids": torch.randint(3, 50, (n,), generator=g).tolist()} for n in lens]
    ex[2]["input_ids"][4] = 2  # a genuine eos == pad inside a sequence: never a target
    return ex


def test_packed_labels_match_padded():
    ex = _examples()
    pad = 2
    p = PackedCollator(pad_id=pad, pad_to_multiple_of=24)(ex)
    q = CausalLMCollator(pad_id=pad)(ex)
    cu = p["cu_seqlens"]
    assert cu[:6] == (0, 7, 10, 22, 23, 32) and cu[-1] == p["n_padded"] == 48
    assert p["n_tokens"] == 32 and p["n_valid"] == q["n_valid"]
    for i, (a, b) in enumerate(zip(cu[:5], cu[1:6])):
        n = b - a
        assert p["input_ids"][0, a:b].tolist() == q["input_ids"][i, :n].tolist()
        assert p["labels"][0, a:b].tolist() == q["labels"][i, :n].tolist()
        assert p["pos"][a:b].tolist() == list(range(n))
    assert (p["labels"][0, 32:] == -100).all()


def test_packed_forward_backward_matches_padded():
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model

    torch.manual_seed(0)
    m = build_model("tiny-llama", dtype=torch.float32, device=torch.device("cpu"), init="random",
                    seed=1)
    apply_lora(m, LoraConfig(r=8, lora_dropout=0.0))
    with torch.no_grad():
        for _, mod in m.lora_modules():
            mod.lora.lora_B.normal_(0, 0.02)
    m.train()
    ex = _examples()
    p = PackedCollator(pad_id=2, pad_to_multiple_of=16)(ex)
    q = CausalLMCollator(pad_id=2)(ex)
    lp = m(p["input_ids"], p["labels"], p["n_valid"], p["pos"], cu_seqlens=p["cu_seqlens"])
    lp.backward()
    gp = {n: t.grad.clone() for n, t in m.named_parameters() if t.requires_grad}
    m.zero_grad(set_to_none=True)
    # padded reference, one sequence at a time (left-aligned rows, no attention mask needed for
    # causal attention since padding is only ever to the right)
    lq = m(q["input_ids"], q["labels"], q["n_valid"])
    lq.backward()
    gq = {n: t.grad.clone() for n, t in m.named_parameters() if t.requires_grad}
    assert math.isclose(lp.item(), lq.item(), rel_tol=1e-5)
    for n in gp:
        torch.testing.assert_close(gp[n], gq[n], rtol=1e-4, atol=1e-6)


def test_prefetch_loader_order_and_errors():
    src = [[{"input_ids": [3, 4, 5]}] * 2 for _ in range(5)]
    ld = PrefetchLoader(src, PackedCollator(pad_id=2, pad_to_multiple_of=8), depth=2, pin=False)
    got = [b["n_tokens"] for _, b in ld]
    assert got == [6] * 5

    def bad(raw):
        raise RuntimeError("boom")

    ld = PrefetchLoader(src, bad, depth=1, pin=False)
    try:
        list(ld)
        raise AssertionError("producer error was swallowed")
    except RuntimeError as e:
        assert "boom" in str(e)


def test_trainer_packed_variable_length(tmp_path):
    from lumen.parallel.dist import init
    from lumen.train.config import load_ds_config
    from lumen.train.trainer import TrainArgs, Trainer

    env = init()
    ds = load_ds_config({"zero_optimization": {"stage": 0}, "bf16": {"enabled": False}}, 4, 1, 1,
                        1e-3)
    a = TrainArgs(model_name="tiny-llama", dataset_path=None, output_dir=str(tmp_path),
                  synthetic=True, synthetic_samples=32, synthetic_min_len=8, max_length=64,
                  max_steps=4, logging_steps=2, save_strategy="no", init="random",
                  per_device_train_batch_size=4, save_final=False)
    tr = Trainer(a, ds, env, printer=lambda *x, **k: None)
    assert tr.packed
    res = tr.train()
    assert res["global_step"] == 4 and math.isfinite(res["final_loss"])


def test_trainer_token_budget_batches(tmp_path):
    from lumen.parallel.dist import init
    from lumen.train.config import load_ds_config
    from lumen.train.trainer import TrainArgs, Trainer

    env = init()
    ds = load_ds_config({"zero_optimization": {"stage": 0}, "bf16": {"enabled": False}}, 4, 1, 1,
                        1e-3)
    a = TrainArgs(model_name="tiny-llama", dataset_path=None, output_dir=str(tmp_path),
                  synthetic=True, synthetic_samples=64, synthetic_min_len=8, max_length=64,
                  max_steps=3, logging_steps=1, save_strategy="no", init="random",
                  per_device_train_batch_size=4, save_final=False, pack_tokens=200)
    tr = Trainer(a, ds, env, printer=lambda *x, **k: None)
    sizes = [sum(len(e["input_ids"]) for e in b) for b in tr._batches(0, 0)]
    assert all(n <= 200 for n in sizes) and sum(sizes) > 0.8 * 200 * len(sizes)
    res = tr.train()
    assert res["global_step"] == 3


def test_token_budget_world2_epoch_end(tmp_path):
    """--pack_tokens at world 2 with ZeRO-3 over a whole epoch: each rank's shard has its own
    length mix, so the token-budget plans differ in length; the ranks agree on the MIN and the
    run reaches the epoch end (an extra micro-step on one rank would hang its ZeRO-3 gathers).
    Resume from a mid-epoch checkpoint continues at the same micro-batch on both ranks."""
    import os
    import socket
    import subprocess
    import sys

    from lumen.data.datasets import SyntheticTokenDataset
    from lumen.data.sampler import ShardedSampler

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n, budget, maxlen = 48, 120, 64
    ds = SyntheticTokenDataset(n, maxlen, 256, seed=42, min_len=8)

    def count(rank):
        c, cur = 0, 0
        for j in ShardedSampler(n, rank, 2, seed=42).indices(0):
            L = ds.length(j)
            if cur and cur + L > budget:
                c, cur = c + 1, 0
            cur += L
        return c + (cur > 0)

    assert count(0) != count(1)  # the case the MIN agreement exists for

    def run(out, extra):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr=127.0.0.1", f"--master-port={port}",
               os.path.join(root, "training", "train_deepspeed_zero3.py"),
               "--model_name", "tiny-llama", "--synthetic", "--synthetic_samples", str(n),
               "--synthetic_min_len", "8", "--max_length", str(maxlen), "--pack_tokens",
               str(budget), "--num_train_epochs", "1", "--logging_steps", "1",
               "--per_device_train_batch_size", "1", "--gradient_accumulation_steps", "1",
               "--device", "cpu", "--output_dir", out, "--metrics_csv",
               os.path.join(out, "m.csv"), "--save_strategy", "steps", "--save_steps", "3",
               "--deepspeed", os.path.join(root, "configs", "ds_config_zero3_mi355x.json"),
               *extra]
        env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=root, LUMEN_WATCHDOG_S="120")
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env,
                           cwd=str(tmp_path))
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
        return r.stdout

    out = str(tmp_path / "ck")
    log = run(out, [])
    steps = min(count(0), count(1))
    assert f'"step": {steps}' in log
    # resume from checkpoint-3 (delete later ones): finishes the same epoch at the same step
    import shutil

    for d in os.listdir(out):
        if d.startswith("checkpoint-") and int(d.split("-")[1]) > 3:
            shutil.rmtree(os.path.join(out, d))
    log2 = run(out, ["--resume_from_checkpoint"])
    assert "resumed from" in log2 and f'"step": {steps}' in log2
    assert '"step": 4' in log2


def test_opt_packed_matches_padded():
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model

    torch.manual_seed(0)
    m = build_model("tiny-opt", dtype=torch.float32, device=torch.device("cpu"), init="random",
                    seed=1)
    apply_lora(m, LoraConfig(r=4, lora_dropout=0.0, target_modules=["q_proj", "v_proj"]))
    m.train()
    ex = _examples()
    p = PackedCollator(pad_id=2, pad_to_multiple_of=16)(ex)
    q = CausalLMCollator(pad_id=2)(ex)
    lp = m(p["input_ids"], p["labels"], p["n_valid"], p["pos"], cu_seqlens=p["cu_seqlens"])
    lq = m(q["input_ids"], q["labels"], q["n_valid"])
    assert math.isclose(lp.item(), lq.item(), rel_tol=1e-5)
