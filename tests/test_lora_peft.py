"""LoRA attach / PEFT adapter format / merge (CPU)."""
import json
import os

import pytest
import torch

from lumen.lora import (LoraConfig, adapter_state_dict, apply_lora, count_parameters,
                        load_adapter, merge_lora, save_adapter)
from lumen.models import build_model


def test_llama2_7b_trainable_counts_match_reference():
    # reference notebook: "trainable params: 16,777,216 || all params: 6,755,192,832 ||
    # trainable%: 0.2484" (training/train.ipynb:307)
    m = build_model("llama2-7b", dtype=torch.bfloat16, device="meta", init="random")
    apply_lora(m, LoraConfig(r=16))
    t, a = count_parameters(m)
    assert t == 16_777_216
    assert a == 6_755_192_832
    assert round(100 * t / a, 4) == 0.2484


def test_llama2_70b_gqa_lora_counts():
    m = build_model("llama2-70b", dtype=torch.bfloat16, device="meta", init="random")
    apply_lora(m, LoraConfig(r=16))
    t, _ = count_parameters(m)
    # q: 16*(8192+8192), k/v: 16*(8192+1024), o: 16*(8192+8192) per layer, 80 layers
    assert t == 80 * 16 * ((8192 + 8192) * 2 + (8192 + 1024) * 2) == 65_536_000


def test_peft_keys_shapes_and_roundtrip(tmp_path):
    torch.manual_seed(0)
    m = build_model("tiny-llama", dtype=torch.float32, init="random")
    apply_lora(m, LoraConfig(r=4))
    for p in m.parameters():
        if p.requires_grad:
            p.data.normal_()
    sd = adapter_state_dict(m)
    H = m.config.hidden_size
    k = "base_model.model.model.layers.0.self_attn.q_proj.lora_A.weight"
    assert k in sd and tuple(sd[k].shape) == (4, H)
    kb = "base_model.model.model.layers.1.self_attn.o_proj.lora_B.weight"
    assert kb in sd and tuple(sd[kb].shape) == (H, 4)
    assert len(sd) == 2 * 4 * m.config.num_hidden_layers
    assert all(v.dtype == torch.float32 for v in sd.values())
    save_adapter(m, str(tmp_path), "tiny-llama")
    cfg = json.load(open(tmp_path / "adapter_config.json"))
    assert cfg["peft_type"] == "LORA" and cfg["r"] == 4 and cfg["lora_alpha"] == 8
    assert sorted(cfg["target_modules"]) == ["k_proj", "o_proj", "q_proj", "v_proj"]
    m2 = build_model("tiny-llama", dtype=torch.float32, init="random")
    load_adapter(m2, str(tmp_path))
    sd2 = adapter_state_dict(m2)
    for kk in sd:
        assert torch.equal(sd[kk], sd2[kk])


def test_opt_peft_keys():
    m = build_model("tiny-opt", dtype=torch.float32, init="random")
    apply_lora(m, LoraConfig(r=4))
    sd = adapter_state_dict(m)
    assert "base_model.model.model.decoder.layers.0.self_attn.out_proj.lora_A.weight" in sd
    assert "base_model.model.model.decoder.layers.0.self_attn.v_proj.lora_B.weight" in sd


def test_merge_equals_adapter_forward():
    torch.manual_seed(0)
    m = build_model("tiny-llama", dtype=torch.float32, init="random")
    apply_lora(m, LoraConfig(r=4, lora_dropout=0.0, target_modules=["q_proj", "v_proj", "o_proj",
                                                                     "gate_proj", "down_proj"]))
    for p in m.parameters():
        if p.requires_grad:
            p.data.normal_(0, 0.1)
    m.eval()
    ids = torch.randint(3, 512, (2, 16))
    with torch.no_grad():
        a = m(ids)
        merge_lora(m)
        b = m(ids)
    assert torch.allclose(a, b, atol=1e-4)


def test_sparse_segments_q_v_only():
    """Adapters on q and v of a fused q|k|v (PEFT's default llama targets) == unfused math."""
    from lumen.ops.lora import lora_linear_ref

    torch.manual_seed(0)
    m = build_model("tiny-llama-gqa", dtype=torch.float32, init="random")
    apply_lora(m, LoraConfig(r=4, lora_dropout=0.0, target_modules=["q_proj", "v_proj"]))
    lin = m.layers[0].self_attn.qkv_proj
    for p in lin.lora.parameters():
        p.data.normal_()
    x = torch.randn(5, lin.in_features)
    y = lin(x)
    W = lin.weight
    qA, qB = lin.lora.segment("q_proj")
    vA, vB = lin.lora.segment("v_proj")
    ref = x @ W.t()
    q_off, q_len = lin.seg_offset("q_proj")
    v_off, v_len = lin.seg_offset("v_proj")
    ref[:, q_off:q_off + q_len] += lin.lora.scale * (x @ qA.t()) @ qB.t()
    ref[:, v_off:v_off + v_len] += lin.lora.scale * (x @ vA.t()) @ vB.t()
    assert torch.allclose(y, ref, atol=1e-5)


def test_checkpointing_true_never_silently_off(monkeypatch):
    """``gradient_checkpointing=True`` picks ``selective``, which can only
    recompute frozen, unadapted MLPs.  With adapters on gate/up/down every layer must fall back
    to a whole-layer recompute instead of keeping every activation."""
    import lumen.models.llama as L

    calls = []
    real = L.cp.checkpoint

    def counting(fn, *a, **k):
        calls.append(fn)
        return real(fn, *a, **k)

    monkeypatch.setattr(L.cp, "checkpoint", counting)
    torch.manual_seed(0)
    ids = torch.randint(0, 100, (2, 16))
    labels = ids.clone()
    for targets, eligible in ((["q_proj", "v_proj"], True),
                              (["q_proj", "gate_proj", "down_proj"], False)):
        m = build_model("tiny-llama", dtype=torch.float32, init="random")
        apply_lora(m, LoraConfig(r=4, target_modules=targets))
        m.gradient_checkpointing = True
        m.train()
        assert m.gradient_checkpointing == "selective"
        assert m.selective_eligible() is eligible
        calls.clear()
        m(ids, labels).backward()
        # eligible: the MLP recomputes its gate|up itself, no whole-layer checkpoint;
        # not eligible: one whole-layer checkpoint per layer
        assert len(calls) == (0 if eligible else m.config.num_hidden_layers)


def test_partial_layer_checkpointing_matches_no_recompute(monkeypatch):
    """``"selective:N"`` / ``"full:N"``: only the first N layers recompute; the loss and every
    adapter gradient equal the run without recompute."""
    import lumen.models.llama as L

    calls = []
    real = L.cp.checkpoint

    def counting(fn, *a, **k):
        calls.append(fn)
        return real(fn, *a, **k)

    monkeypatch.setattr(L.cp, "checkpoint", counting)
    torch.manual_seed(0)
    ids = torch.randint(0, 100, (2, 16))
    labels = ids.clone()
    ref = None
    for pol in ("none", "selective:1", "full:1", "full"):
        torch.manual_seed(1)  # identical weights and adapter init for every policy
        m = build_model("tiny-llama", dtype=torch.float32, init="random")
        apply_lora(m, LoraConfig(r=4, target_modules=["q_proj", "v_proj"]))
        m.gradient_checkpointing = pol
        m.train()
        nl = m.config.num_hidden_layers
        assert m.gradient_checkpointing == (pol if pol != f"full:{nl}" else "full")
        recomputing = [l.mlp.recompute for l in m.layers]
        assert recomputing == [pol == "selective:1" and i == 0 for i in range(nl)]
        calls.clear()
        loss = m(ids, labels)
        loss.backward()
        assert len(calls) == {"none": 0, "selective:1": 0, "full:1": 1, "full": nl}[pol]
        grads = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
        if ref is None:
            ref = (loss.item(), grads)
        else:
            assert abs(loss.item() - ref[0]) < 1e-6
            for n, g in grads.items():
                assert torch.allclose(g, ref[1][n], atol=1e-6, rtol=1e-5), (pol, n)
    m.gradient_checkpointing = "selective:0"
    assert m.gradient_checkpointing == "none"
    with pytest.raises(ValueError):
        m.gradient_checkpointing = "selective:x"
