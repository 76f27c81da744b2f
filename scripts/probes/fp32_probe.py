"""fp32 model on the GPU vs the same weights on the CPU, module by module: names the first module
whose output is non-finite or off by > 1e-3 relative (forward), then the same for the adapter
gradients.  Also SDPA with enable_gqa in fp32 vs repeat_interleave.

    python scripts/probes/fp32_probe.py [--model tiny-llama-deep] [--batch 8] [--seq 16]
"""
import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch
import torch.nn.functional as F

from lumen.lora import LoraConfig, apply_lora
from lumen.models import build_model


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="tiny-llama-deep")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--seq", type=int, default=16)
    a = ap.parse_args()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    q = torch.randn(8, 4, 16, 32, device=dev)
    k = torch.randn(8, 2, 16, 32, device=dev)
    v = torch.randn(8, 2, 16, 32, device=dev)
    o1 = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
    o2 = F.scaled_dot_product_attention(q, k.repeat_interleave(2, 1), v.repeat_interleave(2, 1),
                                        is_causal=True)
    print("sdpa_gqa_fp32 finite", bool(o1.isfinite().all()), "max_diff",
          float((o1 - o2).abs().max()), flush=True)

    cpu = build_model(a.model, dtype=torch.float32, device="cpu", init="random", seed=7)
    apply_lora(cpu, LoraConfig(r=4, lora_alpha=8, lora_dropout=0.0))
    for n, p in cpu.named_parameters():
        if "lora_B" in n:
            p.data.normal_(0, 0.02)
    gpu = copy.deepcopy(cpu).to(dev)
    outs = {}

    def hook(tag):
        def f(mod, inp, out):
            t = out[0] if isinstance(out, tuple) else out
            if torch.is_tensor(t):
                if t.requires_grad:
                    t.retain_grad()
                outs.setdefault(tag, []).append((mod._probe_name, t))
        return f

    for tag, m in (("cpu", cpu), ("gpu", gpu)):
        for n, mod in m.named_modules():
            mod._probe_name = n
            mod.register_forward_hook(hook(tag))
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, 500, (a.batch, a.seq), generator=g)
    lc = cpu(ids, labels=ids)
    lg = gpu(ids.to(dev), labels=ids.to(dev))
    lc = lc[0] if isinstance(lc, tuple) else lc
    lg = lg[0] if isinstance(lg, tuple) else lg
    print("loss cpu", float(lc), "gpu", float(lg), flush=True)
    reported = 0
    for (n1, t1), (n2, t2) in zip(outs["cpu"], outs["gpu"]):
        t1, t2 = t1.detach().float().cpu(), t2.detach().float().cpu()
        if t1.shape != t2.shape:
            continue
        fin = bool(t2.isfinite().all())
        rel = float((t1 - t2).norm() / max(float(t1.norm()), 1e-12)) if fin else float("nan")
        if not fin or rel > 1e-3:
            print("FWD", n2 or "<model>", tuple(t2.shape), "finite", fin, "rel", rel, flush=True)
            reported += 1
            if reported > 12:
                break
    lc.backward()
    lg.backward()
    # gradients w.r.t. module outputs, from the loss backwards: the first mismatch names the
    # op whose backward is wrong (the module AFTER it in forward order consumed a good gradient)
    for (n1, t1), (n2, t2) in reversed(list(zip(outs["cpu"], outs["gpu"]))):
        if t1.grad is None or t2.grad is None:
            continue
        g1, g2 = t1.grad.float(), t2.grad.float().cpu()
        rel = float((g1 - g2).norm() / max(float(g1.norm()), 1e-20))
        print("DOUT", n2 or "<model>", tuple(g2.shape), "rel", round(rel, 6), flush=True)
    gc = {n: p.grad for n, p in cpu.named_parameters() if p.grad is not None}
    bad = 0
    for n, p in gpu.named_parameters():
        if p.grad is None or n not in gc:
            continue
        t2 = p.grad.float().cpu()
        fin = bool(t2.isfinite().all())
        rel = float((gc[n] - t2).norm() / max(float(gc[n].norm()), 1e-12)) if fin else float("nan")
        if not fin or rel > 1e-3:
            print("GRAD", n, "finite", fin, "rel", rel, flush=True)
            bad += 1
    print("done bad_grads", bad, flush=True)


if __name__ == "__main__":
    main()
