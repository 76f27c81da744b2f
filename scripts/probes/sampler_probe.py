"""Decode-step sampler timing (kernels/sampling.hip): 256 rows x V = 32000, greedy / top-k only /
top-p only / both, logits ~ N(0, s^2) for a few spreads.  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from lumen.ops._native import native  # noqa: E402

C = native()
dev = torch.device("cuda")
R, V = 256, 32000
out = {}
for spread in (1.0, 3.0, 8.0):
    logits = (torch.randn(R, V, device=dev) * spread).to(torch.bfloat16)
    for name, t, p, k in (("greedy", 0.0, 1.0, 0), ("topk50", 0.8, 1.0, 50),
                          ("topp0.95", 0.8, 0.95, 0), ("both", 0.8, 0.95, 50)):
        args = (logits, torch.full((R,), t, device=dev), torch.full((R,), p, device=dev),
                torch.full((R,), k, device=dev, dtype=torch.int32))
        o = torch.empty(R, device=dev, dtype=torch.int64)
        for _ in range(3):
            C.sample(*args, 1, 0, o, None)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for i in range(50):
            C.sample(*args, 1, i, o, None)
        e.record()
        torch.cuda.synchronize()
        out[f"s{spread:g}_{name}"] = round(s.elapsed_time(e) * 1000 / 50, 1)
print(json.dumps(out), flush=True)
