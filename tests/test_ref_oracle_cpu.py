"""The fp32 oracle of the production-shape GPU tests (tests/_ref_llama.py) agrees with lumen's
CPU model (torch reference ops) on a toy Llama with GQA: loss and adapter gradients, dropout on
(same seeds from the CPU generator), LoRA on attention AND MLP projections."""
import torch

from _ref_llama import ref_loss, ref_params


def test_oracle_matches_lumen_cpu_model():
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model

    m = build_model("tiny-llama-gqa", dtype=torch.float32, device="cpu", init="random", seed=2)
    apply_lora(m, LoraConfig(r=4, lora_alpha=8, lora_dropout=0.1,
                             target_modules=["q_proj", "k_proj", "v_proj", "o_proj",
                                             "gate_proj", "down_proj"]))
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for _, mod in m.lora_modules():
            mod.lora.lora_B.copy_(torch.randn(mod.lora.lora_B.shape, generator=g) * 0.05)
    m.train()
    P = ref_params(m, "cpu")
    B, S = 3, 40
    ids = torch.randint(3, m.config.vocab_size, (B, S), generator=g)
    labels = torch.full_like(ids, -100)
    labels[:, :-1] = ids[:, 1:]
    torch.manual_seed(9)
    loss = m(ids, labels)
    loss = loss[0] if isinstance(loss, tuple) else loss
    loss.backward()
    n_calls = 4 * m.config.num_hidden_layers      # q|k|v, o, gate|up, down per layer
    torch.manual_seed(9)
    seeds = [int(torch.randint(0, 2**62, (1,)).item()) for _ in range(n_calls)]
    lref = ref_loss(P, m.config, ids.reshape(-1), labels.reshape(-1), [S] * B, 0.1, seeds)
    lref.backward()
    assert abs(loss.item() - lref.item()) < 1e-5 * abs(lref.item())
    for i, L in enumerate(P["layers"]):
        for key, name in (("qkv", "self_attn.qkv_proj"), ("o", "self_attn.o_proj"),
                          ("gu", "mlp.gate_up_proj"), ("down", "mlp.down_proj")):
            A, Bm = L[key + "_lora"][:2]
            mod = m.get_submodule(f"layers.{i}.{name}").lora
            for leaf, prm in ((A, mod.lora_A), (Bm, mod.lora_B)):
                e = ((leaf.grad - prm.grad).norm() / prm.grad.norm()).item()
                assert e < 1e-4, (i, key, e)
