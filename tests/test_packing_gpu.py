"""Packed varlen rows on the GPU path (HIP flash attention over cu_seqlens, per-sequence RoPE
positions fused into the adapter write-back) vs the padded batch."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def test_packed_matches_padded_gpu():
    from lumen.data import CausalLMCollator, PackedCollator
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model

    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = build_model("small-llama", dtype=torch.bfloat16, device=dev, init="random", seed=2)
    apply_lora(m, LoraConfig(r=16, lora_dropout=0.0))
    with torch.no_grad():
        for _, mod in m.lora_modules():
            mod.lora.lora_B.normal_(0, 0.02)
    m.train()
    g = torch.Generator().manual_seed(1)
    V = m.config.vocab_size
    ex = [{"input_ids": torch.randint(3, V, (n,), generator=g).tolist()} for n in (100, 37, 256, 5, 130)]
    p = PackedCollator(pad_id=2, pad_to_multiple_of=256)(ex)
    q = CausalLMCollator(pad_id=2)(ex)
    lp = m(p["input_ids"].to(dev), p["labels"].to(dev), p["n_valid"], p["pos"].to(dev),
           cu_seqlens=p["cu_seqlens"])
    lp.backward()
    gp = {n: t.grad.clone() for n, t in m.named_parameters() if t.requires_grad}
    m.zero_grad(set_to_none=True)
    lq = m(q["input_ids"].to(dev), q["labels"].to(dev), q["n_valid"])
    lq.backward()
    gq = {n: t.grad.clone() for n, t in m.named_parameters() if t.requires_grad}
    assert abs(lp.item() - lq.item()) < 1e-2 * abs(lq.item())
    for n in gp:
        assert _rel(gp[n], gq[n]) < 3e-2, n
