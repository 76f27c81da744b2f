"""The training step's library GEMMs (Llama-2-7B, T = 4096 tokens) run back to back for a
counter pass: clock (GRBM_GUI_ACTIVE over the kernel time) and MFMA busy
(SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x cycles) per shape.

    rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -- \
        python3 scripts/probes/gemm_pmc.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lumen.utils.gemm_tuning import load_tuned_gemms  # noqa: E402

SHAPES = [("qkv fwd", 4096, 12288, 4096), ("o fwd", 4096, 4096, 4096),
          ("gate|up fwd", 4096, 22016, 4096), ("down fwd", 4096, 4096, 11008),
          ("gate|up dX", 4096, 4096, 22016), ("square 8192", 8192, 8192, 8192)]


def main():
    load_tuned_gemms()
    dev = torch.device("cuda")
    for name, M, N, K in SHAPES:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        for _ in range(3):
            torch.matmul(x, w.t())
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            torch.matmul(x, w.t())
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 10 * 1e3
        print(f"{name:12s} M={M} N={N} K={K}: {us:8.1f} us  {2 * M * N * K / us / 1e9:6.3f} PF/s",
              flush=True)


if __name__ == "__main__":
    main()
