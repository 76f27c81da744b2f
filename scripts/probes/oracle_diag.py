"""Per-tensor error of the 7B-shaped training step against the fp32 oracle, for the shipped
HIP path and for the torch bf16 fallback path (the bf16 noise floor of the same math)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from _ref_llama import ref_loss, ref_params  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def main():
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model, get_config

    cfg = get_config("llama2-7b-2l")
    B, S, p = 8, 512, float(os.environ.get("P", "0.05"))
    dev = torch.device("cuda")
    m = build_model("llama2-7b-2l", dtype=torch.bfloat16, device=dev, init="random", seed=0)
    apply_lora(m, LoraConfig(r=16, lora_alpha=32, lora_dropout=p))
    g = torch.Generator(device="cpu").manual_seed(11)
    with torch.no_grad():
        for _, mod in m.lora_modules():
            mod.lora.lora_B.copy_(torch.randn(mod.lora.lora_B.shape, generator=g) * 0.02)
    m.train()
    P = ref_params(m, dev)
    ids = torch.randint(3, cfg.vocab_size, (B, S), generator=g)
    labels = torch.full_like(ids, -100)
    labels[:, :-1] = ids[:, 1:]
    torch.manual_seed(7)
    seeds = [int(torch.randint(0, 2**62, (1,)).item()) for _ in range(2 * cfg.num_hidden_layers)]
    lref = ref_loss(P, cfg, ids.reshape(-1).to(dev), labels.reshape(-1).to(dev), [S] * B, p, seeds)
    lref.backward()
    refg = {}
    for i, L in enumerate(P["layers"]):
        for key, name in (("qkv", "self_attn.qkv_proj"), ("o", "self_attn.o_proj")):
            A, Bm = L[key + "_lora"][:2]
            refg[f"layers.{i}.{name}.lora.lora_A"] = A.grad
            refg[f"layers.{i}.{name}.lora.lora_B"] = Bm.grad
    for mode in ("native", "torch"):
        if mode == "torch":
            os.environ["LUMEN_DISABLE_NATIVE"] = "1"
            os.environ["LUMEN_ALLOW_TORCH_FALLBACK"] = "1"
        m.zero_grad(set_to_none=True)
        torch.manual_seed(7)
        loss = m(ids.to(dev), labels.to(dev))
        loss.backward()
        torch.cuda.synchronize()
        print(f"{mode}: loss {loss.item():.6f} ref {lref.item():.6f} "
              f"rel {abs(loss.item() - lref.item()) / lref.item():.2e}")
        for n, prm in m.named_parameters():
            if prm.requires_grad:
                print(f"  {n:45s} {rel(prm.grad, refg[n]):.4f}")
    os.environ.pop("LUMEN_DISABLE_NATIVE")


if __name__ == "__main__":
    main()
