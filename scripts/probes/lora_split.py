"""Sweep the LoRA kernels' split target (blocks per launch) at the training shapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import lumen.ops.lora as L  # noqa: E402
from lumen.bench.lora_bench import _time  # noqa: E402

dev = torch.device("cuda")
T, K, r = 4096, 4096, 16
shapes = {"qkv": [(0, 4096, 0, 0), (4096, 4096, 16, 4096), (8192, 4096, 32, 8192)],
          "o": [(0, 4096, 0, 0)]}
for tgt in (256, 512, 1024, 2048, 4096):
    L.SPLIT_TARGET = tgt
    out = [f"target {tgt:5d}"]
    for name, segs in shapes.items():
        N = segs[-1][0] + segs[-1][1]
        R = r * len(segs)
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        y = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        dx = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        A = torch.randn(R, K, device=dev) * 0.01
        B = torch.randn(N, r, device=dev) * 0.01
        fwd = _time(lambda: L.lora_fwd_native(x, y, A, B, segs, r, 2.0, 0.05, 123))
        Z = L.lora_fwd_native(x, y, A, B, segs, r, 2.0, 0.05, 123)[0]
        bwd = _time(lambda: L.lora_bwd_native(dy, x, A, B, Z, dx, segs, r, 2.0, 0.05, 123))
        out.append(f"{name} fwd {fwd:6.1f} bwd {bwd:6.1f}")
    print(" | ".join(out), flush=True)
