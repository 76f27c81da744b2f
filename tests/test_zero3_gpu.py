"""ZeRO-3 parameter coordinator on the GPU path (native kernels read the gathered weights at
backward time through ``weight_fn``), on a one-GPU box: ``LUMEN_ZERO3_SINGLE=1`` partitions at
world size 1, where a gather is an async copy on a side stream with the same stream ordering
as RCCL's.  Every schedule (release / keep), with accumulation and activation checkpointing,
must give the stage-0 trajectory."""
import math

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(monkeypatch, stage, schedule=None, ckpt=False, steps=4, accum=2, bwd_wt="none",
           config=None, max_live=None, fold=False):
    from lumen.lora import LoraConfig, adapter_state_dict, apply_lora
    from lumen.models import build_model
    from lumen.parallel.dist import init
    from lumen.train.config import load_ds_config
    from lumen.train.engine import ZeroEngine

    import lumen.ops.lora as lora_mod

    monkeypatch.setenv("LUMEN_ZERO3_SINGLE", "1")
    # same backward GEMM layout on both sides (persistent weights would otherwise use cached
    # W^T while gathered ones do not: bf16 rounding differences that Adam amplifies); for the
    # same reason no LoRA fold here (a folded gathered weight is a row-strided [N, K + 64] view,
    # a persistent one contiguous: different GEMM algorithms) -- the fold on gathered weights
    # has its own test below
    monkeypatch.setenv("LUMEN_BWD_WT", bwd_wt)
    monkeypatch.setattr(lora_mod, "FOLD", fold)
    if schedule:
        monkeypatch.setenv("LUMEN_ZERO3_SCHEDULE", schedule)
    torch.manual_seed(0)
    m = build_model("small-llama", dtype=torch.bfloat16, device=torch.device("cuda"), seed=3)
    apply_lora(m, LoraConfig(r=16, lora_dropout=0.1))
    m.gradient_checkpointing = ckpt
    m.train()
    env = init()
    if config is not None:
        ds = load_ds_config(config, 2, accum, 1, 1e-3, dtype_override="bf16")
        ds.stage3_param_persistence_threshold = int(1e4)
    else:
        z = {"stage": stage, "stage3_param_persistence_threshold": 1e4}
        if max_live is not None:
            z["stage3_max_live_parameters"] = max_live
        # WarmupLR like the reference configs (first step at warmup_min_lr), so the dict runs
        # and the configs/ds_config_zero3.json run follow the same schedule
        ds = load_ds_config({"zero_optimization": z,
                             "scheduler": {"type": "WarmupLR",
                                           "params": {"warmup_min_lr": 0, "warmup_max_lr": "auto",
                                                      "warmup_num_steps": "auto"}}},
                            2, accum, 1, 1e-3)
    eng = ZeroEngine(m, ds, env)
    g = torch.Generator(device="cpu").manual_seed(5)
    losses = []
    for _ in range(steps * accum):
        ids = torch.randint(3, m.config.vocab_size, (2, 64), generator=g).cuda()
        labels = torch.roll(ids, -1, 1)
        loss = eng.forward({"input_ids": ids, "labels": labels})
        eng.backward(loss)
        eng.step()
        losses.append(float(loss))
    eng.sync_params()  # an offloaded optimizer step may still be in flight (async offload)
    torch.cuda.synchronize()
    return adapter_state_dict(m), losses, eng.coordinator


def _layer_numel(name="small-llama"):
    from lumen.models import get_config

    c = get_config(name)
    H, D = c.hidden_size, c.head_dim
    return (H * (c.num_attention_heads + 2 * c.num_key_value_heads) * D
            + c.num_attention_heads * D * H + 3 * H * c.intermediate_size)


# live budgets: release -> 1 element (a ring of 2 buffers); hybrid -> a 2-buffer ring + one of
# the two decoder layers resident
_LIVE = {"release": lambda: 1, "hybrid": lambda: int(3.02 * _layer_numel()), "keep": lambda: None}


@pytest.mark.parametrize("schedule,ckpt", [("release", False), ("keep", False),
                                           ("keep", True), ("release", True),
                                           ("hybrid", False), ("hybrid", True)])
def test_zero3_schedules_match_stage0_on_gpu(schedule, ckpt, monkeypatch):
    ref, ref_losses, _ = _train(monkeypatch, 0, ckpt=ckpt)
    # release: a live budget of one unit -> a ring of 2 buffers, nothing kept across the turn,
    # every layer gathered twice per micro-step
    # (hybrid forced: a 2-layer model has no budget that is below the model and still holds a
    # two-buffer ring plus a layer -- the auto rule is covered by the gloo world-4/8 tests)
    got, losses, coord = _train(monkeypatch, 3, schedule, ckpt=ckpt, max_live=_LIVE[schedule]())
    assert coord is not None and coord.schedule == schedule
    n_units = sum(1 for u in coord.units if u.params)
    if schedule == "release":
        assert coord.pool_size == 2 and coord.turn_keep == 0 and coord.pool_overflows == 0
        # forward: every unit; backward: every layer (the head is consumed at the turn)
        assert coord.gathers == 8 * (n_units + n_units - 2)
    elif schedule == "hybrid":
        # the last decoder layer resident (gathered once); embedding, layer 1 and the head go
        # through a 2-buffer ring: 3 forward gathers + layer 1 again in the backward
        assert [u.idx for u in coord.units if u.resident] == [2]
        assert coord.pool_size == 2 and coord.pool_overflows == 0
        assert coord.gathers == 8 * 4 + 1
    else:
        # keep: every unit gathered once, then resident (frozen weights never go stale)
        assert coord.gathers == n_units
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 2e-2 * max(1.0, abs(b))
    for k in ref:
        torch.testing.assert_close(got[k], ref[k], rtol=2e-3, atol=2e-5)


@pytest.mark.parametrize("schedule", ["release", "hybrid"])
def test_zero3_transposed_backward_gathers(schedule, monkeypatch):
    """Ring units gather their TRANSPOSED shard for the backward (W^T [K, N] per projection),
    so the input-gradient GEMMs run in the TN form straight from the gathered buffer: same
    trajectory as stage 0 with persistent W^T copies (the same GEMM form)."""
    ref, _, _ = _train(monkeypatch, 0, bwd_wt="all")
    got, _, coord = _train(monkeypatch, 3, schedule, bwd_wt="all", max_live=_LIVE[schedule]())
    assert coord.schedule == schedule
    ring = [u for u in coord.units[1:-1] if not u.resident]
    assert ring and all(u.shard_t is not None for u in ring)
    assert all(u.shard_t is None for u in coord.units if u.resident)
    # every ring decoder layer is gathered transposed once per backward (8 micro-steps)
    assert coord.gathers_t == 8 * len(ring)
    for k in ref:
        torch.testing.assert_close(got[k], ref[k], rtol=2e-3, atol=2e-5)
    # a recompute policy needs the forward layout in the backward: no transposed gathers
    got2, _, coord2 = _train(monkeypatch, 3, schedule, bwd_wt="all", max_live=_LIVE[schedule](),
                             ckpt="full")
    assert coord2.gathers_t == 0


def test_zero3_offpath_transposes_match_persistent_layout(monkeypatch):
    """keep: W^T of every gathered projection is written once, on a side stream right after its
    gather, so the backward runs the same TN GEMMs as with persistent weights."""
    ref, _, _ = _train(monkeypatch, 0, bwd_wt="all", ckpt=True)
    got, _, coord = _train(monkeypatch, 3, "keep", bwd_wt="all", ckpt=True)
    assert coord.transposed_numel > 0
    # 4 projections per decoder unit, plus the LM head's W^T in the last unit (LUMEN_LMHEAD_WT)
    head = int(os.environ.get("LUMEN_LMHEAD_WT", "1") != "0")
    assert sum(len(u.tn) for u in coord.units) == 4 * sum(1 for u in coord.units[1:-1]) + head
    for k in ref:
        torch.testing.assert_close(got[k], ref[k], rtol=2e-3, atol=2e-5)


def test_reference_zero3_config_with_cpu_offload(monkeypatch):
    """The reference's configs/ds_config_zero3.json (params AND optimizer offloaded to CPU,
    pinned) on the GPU path:
    shards stream H2D per gather, the C++ AdamW updates the host master copy."""
    import os

    from lumen.train.config import load_ds_config

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    raw = load_ds_config(os.path.join(root, "configs", "ds_config_zero3.json"), 2, 2, 1, 1e-3)
    assert raw.offload_param == "cpu" and raw.offload_optimizer == "cpu"
    ref, ref_losses, _ = _train(monkeypatch, 0)
    got, losses, coord = _train(monkeypatch, 3, config=os.path.join(root, "configs",
                                                                      "ds_config_zero3.json"))
    assert coord.offload and coord.units[1].shard.device.type == "cpu"
    assert coord.units[1].shard.is_pinned()
    # host AdamW vs the fused HIP AdamW: same math, different rounding order.  Adam turns a
    # rounding difference in a near-zero gradient into a flipped update of size ~lr (1e-3), so
    # bound the few outliers by 4 lr and require the bulk to agree tightly.
    for k in ref:
        d = (got[k] - ref[k]).abs()
        assert d.max().item() < 4e-3, k
        assert (d > 3e-4 + 5e-3 * ref[k].abs()).float().mean().item() < 5e-3, k


@pytest.mark.parametrize("schedule", ["keep", "release", "hybrid"])
def test_zero3_schedules_race_free_under_nan_poison(schedule, monkeypatch):
    """Race detector: with LUMEN_ZERO3_POISON every buffer is NaN-filled right before each
    (re-)gather.  A read outside a buffer's live window would make the loss NaN; the run must
    match the unpoisoned one."""
    ml = _LIVE[schedule]()   # release: a 2-buffer ring, re-used every unit
    ref, ref_losses, _ = _train(monkeypatch, 3, schedule, ckpt=True, steps=3, max_live=ml)
    monkeypatch.setenv("LUMEN_ZERO3_POISON", "1")
    got, losses, coord = _train(monkeypatch, 3, schedule, ckpt=True, steps=3, max_live=ml)
    assert coord.poison
    assert all(math.isfinite(x) for x in losses)
    # (not bitwise: the LoRA kernels' split-K f32 atomics make run-to-run rounding differ)
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 1e-3 * max(1.0, abs(b))
    for k in ref:
        assert torch.isfinite(got[k]).all(), k
        torch.testing.assert_close(got[k], ref[k], rtol=2e-3, atol=2e-5)


@pytest.mark.parametrize("schedule", ["keep", "release"])
def test_zero3_gathered_lora_fold(schedule, monkeypatch):
    """LoRA fold on ZeRO-3-gathered weights: the partitioned layout reserves the [N, K + 64]
    adapter tail, it is (re)filled with s * lora_B after every gather and whenever lora_B
    changes, and one micro-step's loss and adapter gradients equal the unfolded UP write-back's
    (gradients compared before any optimizer step, where bf16 rounding is not amplified).
    keep: after an optimizer step the resident weights' tails hold the NEW lora_B."""
    import lumen.ops.lora as lora_mod
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model
    from lumen.parallel.dist import init
    from lumen.train.config import load_ds_config
    from lumen.train.engine import ZeroEngine

    monkeypatch.setenv("LUMEN_ZERO3_SINGLE", "1")
    monkeypatch.setenv("LUMEN_ZERO3_SCHEDULE", schedule)
    out = []
    for fold in (True, False):
        monkeypatch.setattr(lora_mod, "FOLD", fold)
        torch.manual_seed(0)
        m = build_model("small-llama", dtype=torch.bfloat16, device=torch.device("cuda"), seed=3)
        apply_lora(m, LoraConfig(r=16, lora_dropout=0.0))
        with torch.no_grad():
            for _, mod in m.lora_modules():
                mod.lora.lora_B.normal_(0, 0.02, generator=torch.Generator(
                    device="cuda").manual_seed(11))
        m.train()
        z = {"stage": 3, "stage3_param_persistence_threshold": 1e4}
        if schedule == "release":
            z["stage3_max_live_parameters"] = 1
        eng = ZeroEngine(m, load_ds_config({"zero_optimization": z}, 2, 1, 1, 1e-3), init())
        coord = eng.coordinator
        assert coord is not None and coord.schedule == schedule
        if fold:
            assert all(len(u.folds) == 2 for u in coord.units[1:-1])  # q|k|v and o per layer
        g = torch.Generator(device="cpu").manual_seed(5)
        ids = torch.randint(3, m.config.vocab_size, (2, 64), generator=g).cuda()
        loss = eng.forward({"input_ids": ids, "labels": torch.roll(ids, -1, 1)})
        eng.backward(loss)
        torch.cuda.synchronize()
        grads = {n: p.grad.float().clone() for n, p in m.named_parameters() if p.requires_grad}
        out.append((float(loss), grads))
        eng.step()
        if fold:
            eng.sync_params()
            loss = eng.forward({"input_ids": ids, "labels": torch.roll(ids, -1, 1)})
            eng.backward(loss)
            torch.cuda.synchronize()
            KP = lora_mod.FOLD_KP
            for u in coord.units[1:-1]:
                for lin in u.folds:
                    W = lin.weight
                    if W.numel() == 0:   # release: unit handed back to the ring
                        continue
                    K = lin.in_features
                    tail = W.as_strided((W.shape[0], K + KP), (K + KP, 1))[:, K:]
                    want = torch.zeros(W.shape[0], K + KP, dtype=W.dtype, device=W.device)
                    lin._fill_tail(want)
                    torch.testing.assert_close(tail, want[:, K:], rtol=0, atol=0)
        eng.close()
    (l1, g1), (l2, g2) = out
    assert abs(l1 - l2) < 2e-3 * abs(l2)
    for n in g1:
        r = ((g1[n] - g2[n]).norm() / g2[n].norm().clamp_min(1e-12)).item()
        assert r < 3e-2, (n, r)


@pytest.mark.parametrize("schedule", ["keep", "release"])
def test_async_offloaded_optimizer_matches_sync(schedule, monkeypatch):
    """offload_optimizer: cpu with the asynchronous step (D2H on a copy stream, C++ AdamW on a
    host thread in forward order, per-unit H2D events gating the next forward) == the
    synchronous offloaded step (same host kernel on the same gradients)."""
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = os.path.join(root, "configs", "ds_config_zero3_offload_opt_mi355x.json")
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("LUMEN_OFFLOAD_ASYNC", mode)
        res[mode] = _train(monkeypatch, 3, schedule, config=cfg)
    (sync, sl, _), (asy, al, coord) = res["0"], res["1"]
    assert coord is not None and coord.schedule == schedule
    for a, b in zip(sl, al):
        assert abs(a - b) < 1e-2 * max(1.0, abs(a)), (sl, al)
    for k in sync:
        d = (asy[k] - sync[k]).abs()
        assert d.max().item() < 4e-3, k
        assert (d > 3e-4 + 5e-3 * sync[k].abs()).float().mean().item() < 5e-3, k
    assert any(v.abs().sum() > 0 for k, v in asy.items() if "lora_B" in k)
