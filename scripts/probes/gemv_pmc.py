"""Batch-1 GEMV kernels at the Llama-2-7B projection shapes, 20 calls each, for a rocprofv3
--pmc run (FETCH_SIZE per dispatch -> HBM bytes actually read)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from lumen.ops._native import native  # noqa: E402

dev = "cuda"
for name, (N, K) in {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096),
                     "down": (4096, 11008)}.items():
    ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(2)]
    x = torch.randn(1, K, device=dev).to(torch.bfloat16)
    y = torch.empty(1, N, device=dev, dtype=torch.bfloat16)
    for i in range(20):
        native().skinny_gemm(x, ws[i % 2], y)
    torch.cuda.synchronize()
    del ws
print("ok")
