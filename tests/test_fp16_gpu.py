"""fp16 training on the GPU path with the reference's dynamic loss scaling
(reference configs/ds_config_zero2.json:17-24 -- fp16, loss_scale 0 = dynamic, initial scale
2^16, hysteresis 2, window 1000; the only published run is fp16 ZeRO-2, training/train.ipynb:442).

The loss scaler, Adam bias correction and WarmupLR run on the device (kernels/adamw.hip
OptSched), so an fp16 step must not synchronise the host; a forced overflow must skip the
update, halve the scale only after ``hysteresis`` overflows, and leave the trajectory equal to
one in which those batches never happened."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FP16_CFG = os.path.join(ROOT, "configs", "ds_config_zero2.json")  # the reference config: fp16


def _engine(dtype_cfg=FP16_CFG, seed=3):
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model
    from lumen.parallel.dist import init
    from lumen.train.config import load_ds_config
    from lumen.train.engine import ZeroEngine

    ds = load_ds_config(dtype_cfg, 2, 1, 1, 1e-3)
    torch.manual_seed(0)
    m = build_model("small-llama", dtype=ds.torch_dtype, device=torch.device("cuda"), seed=seed)
    apply_lora(m, LoraConfig(r=16, lora_dropout=0.0))
    m.train()
    return ZeroEngine(m, ds, init()), m, ds


def _batches(n, vocab):
    g = torch.Generator(device="cpu").manual_seed(11)
    out = []
    for _ in range(n):
        ids = torch.randint(3, vocab, (2, 64), generator=g).cuda()
        out.append({"input_ids": ids, "labels": torch.roll(ids, -1, 1), "n_valid": 2 * 64})
    return out


def test_fp16_config_is_dynamic_loss_scaled():
    eng, m, ds = _engine()
    assert ds.dtype == "fp16" and ds.stage == 2
    assert eng.device_sched and eng.scaler is not None
    assert eng.loss_scale == 2.0 ** 16
    assert next(m.parameters()).dtype == torch.float16


def test_fp16_steps_do_not_sync_host():
    eng, m, _ = _engine()
    bs = _batches(3, m.config.vocab_size)
    loss = eng.forward(bs[0])
    eng.backward(loss)
    eng.step()
    torch.cuda.synchronize()
    for b in bs[1:]:
        loss = eng.forward(b)
        eng.backward(loss)
        torch.cuda.set_sync_debug_mode("error")
        try:
            eng.step()   # unscale / clip / overflow skip / scaler update / LR all on device
        finally:
            torch.cuda.set_sync_debug_mode(0)
    assert eng.skipped_steps == 0 and eng.opt.step_count == 3


def test_fp16_forced_overflow_skips_and_backs_off(monkeypatch):
    """Run A: batches 0..5 with +inf injected into the gradient at steps 2 and 3.  Run B: the
    same engine on batches 0, 1, 4, 5 with the loss scale set to what A's scaler reached.  Step
    2 (first overflow) only spends hysteresis; step 3 halves the scale; neither advances Adam's
    step counter or the LR schedule, so A's adapters equal B's (the adapter reductions are
    deterministic, kernels/det.h): the A-B distance must be tiny next to the distance either run
    moved from the initial adapters."""
    import lumen.ops.lora as L
    from lumen.lora import adapter_state_dict

    monkeypatch.setattr(L, "DETERMINISTIC", True)  # order-independent adapter sums
    engA, mA, _ = _engine()
    init = {k: v.clone() for k, v in adapter_state_dict(mA).items()}
    bs = _batches(6, mA.config.vocab_size)
    scales = []
    snap = None
    for i, b in enumerate(bs):
        loss = engA.forward(b)
        engA.backward(loss)
        if i in (2, 3):
            engA.flat.grad[5] = float("inf")
        if i == 2:  # the optimizer's whole state before the two overflowing steps
            o = engA.opt
            snap = [t.clone() for t in (o.master, o.m, o.v)] + [
                {k: v.clone() for k, v in adapter_state_dict(mA).items()}, o.state[0].item()]
        engA.step()
        scales.append(engA.loss_scale)
        if i == 3:
            # the skip itself, asserted directly: master weights, both Adam moments, the
            # published adapters and the device step counter are exactly as before step 2
            o = engA.opt
            for before, now in zip(snap[:3], (o.master, o.m, o.v)):
                assert torch.equal(before, now)
            now_ad = adapter_state_dict(mA)
            assert all(torch.equal(v, now_ad[k]) for k, v in snap[3].items())
            assert o.state[0].item() == snap[4]
    assert scales[:3] == [2.0 ** 16] * 3          # first overflow: hysteresis 2 -> 1
    assert scales[3:] == [2.0 ** 15] * 3          # second: halve
    assert engA.skipped_steps == 2 and engA.opt.step_count == 4
    assert engA.global_step == 6                  # HF counts every optimizer step

    engB, mB, _ = _engine()
    for j, i in enumerate((0, 1, 4, 5)):
        if j == 2:
            engB.opt.state[2] = 2.0 ** 15
        loss = engB.forward(bs[i])
        engB.backward(loss)
        engB.step()
    a, b = adapter_state_dict(mA), adapter_state_dict(mB)
    for k in a:
        assert torch.isfinite(a[k]).all(), k
        moved = (a[k].float() - init[k].float()).norm()
        diff = (a[k].float() - b[k].float()).norm()
        # 1 %: the adapter reductions are deterministic (kernels/det.h), so A and B differ only
        # by what the skipped steps' forwards did to the RNG streams; a wrong skip would move A
        # away from B by O(moved) itself (the skip is asserted directly above)
        assert diff <= 1e-2 * moved + 1e-7, (k, float(diff), float(moved))
    assert any(v.abs().sum() > 0 for k, v in a.items() if "lora_B" in k)


def test_fp16_trajectory_tracks_bf16():
    """Same data and init in fp16 (dynamic scaling) and bf16: the losses agree to rounding."""
    cfg_bf16 = os.path.join(ROOT, "configs", "ds_config_zero2_mi355x.json")
    res = {}
    for name, cfg in (("fp16", FP16_CFG), ("bf16", cfg_bf16)):
        eng, m, _ = _engine(cfg)
        losses = []
        for b in _batches(5, m.config.vocab_size):
            loss = eng.forward(b)
            eng.backward(loss)
            eng.step()
            losses.append(float(loss))
        res[name] = losses
    for a, b in zip(res["fp16"], res["bf16"]):
        assert abs(a - b) < 2e-2 * max(1.0, abs(b)), res
    assert res["fp16"][-1] < res["fp16"][0]
