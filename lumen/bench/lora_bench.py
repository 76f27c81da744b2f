"""LoRA adapter-kernel timing at the Llama-2-7B training shapes (T = 8 x 512 tokens).

    python -m lumen.bench.lora_bench

Times the forward adapter products (Z = drop(x) A^T, y += s Z B^T) and the backward ones
(dZ, dA, dB, dx += drop'(dZ A)) for the fused q|k|v (3 segments, R = 48) and o_proj (R = 16)
linears, with the f32-MFMA kernel and with the 16-bit-MFMA kernels.
"""
from __future__ import annotations

import torch


def _time(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    import lumen.ops.lora as L

    dev = torch.device("cuda")
    T, K, r = 4096, 4096, 16
    shapes = {"qkv": [(0, 4096, 0, 0), (4096, 4096, 16, 4096), (8192, 4096, 32, 8192)],
              "o": [(0, 4096, 0, 0)]}
    for name, segs in shapes.items():
        N = segs[-1][0] + segs[-1][1]
        R = r * len(segs)
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        y = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        dx = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        A = torch.randn(R, K, device=dev) * 0.01
        B = torch.randn(N, r, device=dev) * 0.01
        for impl in ("f32", "v2"):
            L.USE_V2 = impl == "v2"
            fwd = _time(lambda: L.lora_fwd_native(x, y, A, B, segs, r, 2.0, 0.05, 123))
            Z = L.lora_fwd_native(x, y, A, B, segs, r, 2.0, 0.05, 123)[0]
            bwd = _time(lambda: L.lora_bwd_native(dy, x, A, B, Z, dx, segs, r, 2.0, 0.05, 123))
            print(f"{name:4s} {impl:4s} fwd {fwd:7.1f} us  bwd {bwd:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
