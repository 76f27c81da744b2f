"""Where does run-to-run nondeterminism enter a training step?  Two identical forward+backward
passes of small-llama + LoRA (same seeds); every module's forward output and every module's
output gradient are recorded and compared bitwise; prints the first ones that differ (in
execution order) and checks the LoRA kernels alone on fixed inputs."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

DEV = "cuda"


def run():
    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model

    torch.manual_seed(0)
    m = build_model("small-llama", dtype=torch.bfloat16, device=torch.device(DEV), seed=3)
    apply_lora(m, LoraConfig(r=16, lora_dropout=0.05))
    m.train()
    for prm in m.parameters():
        if prm.requires_grad:
            with torch.no_grad():
                prm.normal_(0, 0.02, generator=torch.Generator(DEV).manual_seed(11))
    rec = []

    def fh(name):
        def f(mod, inp, out):
            o = out[0] if isinstance(out, tuple) else out
            if torch.is_tensor(o):
                rec.append(("fwd " + name, o.detach().clone()))
        return f

    def bh(name):
        def f(mod, gin, gout):
            for i, g in enumerate(gout):
                if torch.is_tensor(g):
                    rec.append((f"bwd {name} gout{i}", g.detach().clone()))
        return f

    for n, mod in m.named_modules():
        if n and len(list(mod.children())) == 0:
            mod.register_forward_hook(fh(n))
            mod.register_full_backward_hook(bh(n))
    g = torch.Generator(device="cpu").manual_seed(7)
    ids = torch.randint(3, m.config.vocab_size, (2, 512), generator=g).to(DEV)
    torch.manual_seed(5)
    loss = m(input_ids=ids, labels=torch.roll(ids, -1, 1))
    rec.append(("loss", loss.detach().clone()))
    loss.backward()
    torch.cuda.synchronize()
    for n, p in m.named_parameters():
        if p.requires_grad:
            rec.append(("grad " + n, p.grad.detach().clone()))
    return rec


def main():
    a, b = run(), run()
    bad = [(na, float((ta.float() - tb.float()).abs().max())) for (na, ta), (nb, tb) in zip(a, b)
           if not torch.equal(ta, tb)]
    print(f"{len(a)} records, {len(bad)} differ")
    for n, d in bad[:25]:
        print(f"  DIFF {n}: max abs {d:.3e}")


if __name__ == "__main__":
    main()
