"""Flash-attention forward/backward shape probe: where the per-tile cost goes.

Times lumen's attention at several (B, S, causal) shapes with the same total token count so the
tile count per workgroup changes while the work per tile does not.  Output: one JSON line per
shape with us / TF/s for the forward and forward+backward.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from lumen.ops.attention import flash_attention_qkv

    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="8x512c,8x512n,2x2048c,2x2048n,32x128c")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--bwd", action="store_true")
    a = ap.parse_args()
    nh = 32
    D = 128
    for spec in a.shapes.split(","):
        bs, rest = spec.split("x")
        B, S, causal = int(bs), int(rest[:-1]), rest[-1] == "c"
        T = B * S
        qkv = (torch.randn(T, 3 * nh * D, device="cuda") * 0.5).to(torch.bfloat16)
        cu = list(range(0, T + 1, S))
        fl = 4 * B * nh * S * S * D * (0.5 if causal else 1.0)

        def fwd():
            return flash_attention_qkv(qkv, cu, nh, nh, D, causal)

        def run(fn):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / a.iters

        res = {"shape": spec, "fwd_us": round(run(fwd), 1)}
        res["fwd_tflops"] = round(fl / res["fwd_us"] / 1e6, 1)
        if a.bwd:
            x = qkv.clone().requires_grad_(True)
            o = flash_attention_qkv(x, cu, nh, nh, D, causal)
            g = torch.randn_like(o)
            res["bwd_us"] = round(run(lambda: torch.autograd.grad(o, x, g, retain_graph=True)), 1)
            res["bwd_tflops"] = round(2.5 * fl / res["bwd_us"] / 1e6, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
