"""LoRA adapter passes at the Llama-2-7B training shapes (T = 8 x 512), as the model calls them:
q|k|v with the fused RoPE write-back and o_proj; forward (Z, y += s Z B^T) and backward
(dZ, dA, dB, dx += drop'(dZ A)).  Prints one JSON line of microseconds per call."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import lumen.ops.lora as L  # noqa: E402
from lumen.ops.rope import rope_tables  # noqa: E402


def _time(fn, iters=40):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1000.0, 1)


dev = torch.device("cuda")
T, K, r, D = 4096, 4096, 16, 128
cos, sin = rope_tables(D, 4096, 10000.0, dev)
pos = (torch.arange(T, device=dev) % 512).to(torch.int32)
out = {"v3": L.USE_V3, "dy_tw": L.DY_TW}
for name, segs, rope_cols in (("qkv", [(0, 4096, 0, 0), (4096, 4096, 16, 1), (8192, 4096, 32, 2)], 8192),
                              ("o", [(0, 4096, 0, 0)], 0)):
    N = segs[-1][0] + segs[-1][1]
    R = r * len(segs)
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    y = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
    dx = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    A = torch.randn(R, K, device=dev) * 0.01
    B = torch.randn(N, r, device=dev) * 0.01
    rope = (pos, cos, sin, rope_cols) if rope_cols else None
    out[name + "_fwd"] = _time(lambda: L.lora_fwd_native(x, y, A, B, segs, r, 2.0, 0.05, 123,
                                                         rope=rope))
    Z = L.lora_fwd_native(x, y, A, B, segs, r, 2.0, 0.05, 123)[0]
    out[name + "_bwd"] = _time(lambda: L.lora_bwd_native(dy, x, A, B, Z, dx, segs, r, 2.0, 0.05,
                                                         123))
print(json.dumps(out), flush=True)
