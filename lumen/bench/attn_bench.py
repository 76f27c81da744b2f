"""Micro-benchmark: HIP flash attention vs torch SDPA (fwd / fwd+bwd) at training shapes."""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import torch.nn.functional as F

    from lumen.ops.attention import flash_attention_qkv

    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--S", type=int, default=512)
    ap.add_argument("--nh", type=int, default=32)
    ap.add_argument("--nkv", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="all")
    a = ap.parse_args()
    D = 128
    res = {"B": a.B, "S": a.S, "nh": a.nh, "nkv": a.nkv}
    dev = "cuda"
    T = a.B * a.S
    qkv = (torch.randn(T, (a.nh + 2 * a.nkv) * D, device=dev) * 0.5).to(torch.bfloat16)
    cu = list(range(0, T + 1, a.S))
    flops_f = 4 * a.B * a.nh * a.S * a.S * D / 2  # causal

    def timeit(fn, n):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n

    q = qkv[:, :a.nh * D].view(a.B, a.S, a.nh, D).transpose(1, 2).contiguous()
    k = qkv[:, a.nh * D:(a.nh + a.nkv) * D].view(a.B, a.S, a.nkv, D).transpose(1, 2).contiguous()
    v = qkv[:, (a.nh + a.nkv) * D:].view(a.B, a.S, a.nkv, D).transpose(1, 2).contiguous()
    if a.only in ("all", "fwd"):
        t = timeit(lambda: flash_attention_qkv(qkv, cu, a.nh, a.nkv, D, True), a.iters)
        res["lumen_fwd_us"] = round(t * 1e6, 1)
        res["lumen_fwd_tflops"] = round(flops_f / t / 1e12, 1)
        t = timeit(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True,
                                                           enable_gqa=a.nkv != a.nh), a.iters)
        res["sdpa_fwd_us"] = round(t * 1e6, 1)
    if a.only in ("all", "bwd"):
        x = qkv.clone().requires_grad_(True)
        o = flash_attention_qkv(x, cu, a.nh, a.nkv, D, True)
        g = torch.randn_like(o)
        t = timeit(lambda: torch.autograd.grad(o, x, g, retain_graph=True), a.iters)
        res["lumen_bwd_us"] = round(t * 1e6, 1)
        res["lumen_bwd_tflops"] = round(2.5 * flops_f / t / 1e12, 1)
        q2, k2, v2 = (t_.clone().requires_grad_(True) for t_ in (q, k, v))
        o2 = F.scaled_dot_product_attention(q2, k2, v2, is_causal=True, enable_gqa=a.nkv != a.nh)
        g2 = torch.randn_like(o2)
        t = timeit(lambda: torch.autograd.grad(o2, (q2, k2, v2), g2, retain_graph=True), a.iters)
        res["sdpa_bwd_us"] = round(t * 1e6, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
