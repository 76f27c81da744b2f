"""Kernel durations of the decode-path small ops at batch 1 (run under rocprofv3 --kernel-trace)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from lumen.ops.norm import rms_norm  # noqa: E402
from lumen.ops.activation import swiglu  # noqa: E402

dev = "cuda"
for T in (1, 16, 256):
    x = torch.randn(T, 4096, device=dev, dtype=torch.bfloat16)
    r = torch.randn(T, 4096, device=dev, dtype=torch.bfloat16)
    w = torch.ones(4096, device=dev, dtype=torch.bfloat16)
    gu = torch.randn(T, 22016, device=dev, dtype=torch.bfloat16)
    for _ in range(200):
        rms_norm(x, w, 1e-5, r)
        rms_norm(x, w, 1e-5)
        swiglu(gu)
        x + r
    torch.cuda.synchronize()
print("ok")
