"""Per-kernel timing of the LoRA adapter passes at the Llama-2-7B training shapes (T = 8 x 512,
r = 16, p = 0.05): lora_v2 vs lora_v3 for DOWN (Z = drop(x) A^T), UP (y += s Z B^T with RoPE),
the backward dY products (v2: DOWN mode 2 + WGRAD dB; v3: fused dy3) and dx += drop'(dZ A).
Prints one JSON line of microseconds per call and effective GB/s."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import lumen.ops.lora as L  # noqa: E402
from lumen.ops._native import native  # noqa: E402
from lumen.ops.rope import rope_tables  # noqa: E402


def _time(fn, iters=50):
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
nat = native()
T, K, r, D, p = 4096, 4096, 16, 128, 0.05
seed = 1234
th, ds = L.drop_threshold(p), 1.0 / (1.0 - p)
cos, sin = rope_tables(D, 4096, 10000.0, dev)
pos = (torch.arange(T, device=dev) % 512).to(torch.int32)
tw_env = int(os.environ.get("TW", "0"))
out = {}
for name, segs, rope_cols in (("qkv", [(0, 4096, 0, 0), (4096, 4096, 16, 4096), (8192, 4096, 32, 8192)], 8192),
                              ("o", [(0, 4096, 0, 0)], 0)):
    N = segs[-1][0] + segs[-1][1]
    R = r * len(segs)
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    y = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
    dx = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    A = torch.randn(R, K, device=dev) * 0.01
    B = torch.randn(N, r, device=dev) * 0.01
    Z = torch.zeros(T, R, device=dev)
    dZ = torch.zeros(T, R, device=dev)
    dA = torch.zeros(R, K, device=dev)
    dB = torch.zeros(N, r, device=dev)
    mb = 1e6
    # DOWN
    t2 = _time(lambda: L._lora2(0, 1, x, A, Z, R, 1, 1.0, T, R, L._split(math.ceil(T / 64), K, 256),
                                [(0, 0, 0, K)], seed, p, K))
    t3 = _time(lambda: nat.lora3_down(x, K, A, Z, R, T, K, R, 1.0, seed, th, ds, K, 0))
    out[name + "_down"] = (t2, t3, round(x.numel() * 2 / t3 / 1e3, 0))
    # UP (+ RoPE on q|k)
    mask = sum(1 << j for j, sg in enumerate(segs) if sg[0] + sg[1] <= rope_cols) if rope_cols else 0
    rp2 = (cos, sin, pos, mask) if rope_cols else None
    t2 = _time(lambda: L._lora2(2, 1, B, Z, y, y.stride(0), 1, 2.0, T, r, 1,
                                [(b_off * r, r_off, n_off, n_len) for (n_off, n_len, r_off, b_off) in segs],
                                rope=rp2))
    rp3 = (cos, sin, pos) if rope_cols else (None, None, None)
    t3 = _time(lambda: nat.lora3_up(1, y, N, Z, R, B, r, T, r, 2.0, 0, 0, 1.0, 0, 0,
                                    [(n_off, r_off, b_off, n_len) for (n_off, n_len, r_off, b_off) in segs],
                                    *rp3, mask))
    out[name + "_up"] = (t2, t3, round(y.numel() * 4 / t3 / 1e3, 0))
    # dY products

    def v2_dy():
        L._lora2(0, 0, dy, B, dZ, R, 1, 2.0, T, r, L._split(math.ceil(T / 64) * len(segs), K, 256),
                 [(n_off, b_off * r, r_off, n_len) for (n_off, n_len, r_off, b_off) in segs])
        L._lora2(1, 0, dy, Z, dB, r, 1, 2.0, T, r,
                 L._split(sum(math.ceil(s[1] / 128) for s in segs), T, 128),
                 [(n_off, r_off, b_off * r, n_len) for (n_off, n_len, r_off, b_off) in segs])
    t2 = _time(v2_dy)
    t3 = _time(lambda: nat.lora3_dy(dy, N, B, r, Z, R, dZ, R, dB, T, tw_env or L._dy_tw(segs, T), 2.0,
                                    [(n_off, r_off, b_off, n_len) for (n_off, n_len, r_off, b_off) in segs]))
    out[name + "_dy"] = (t2, t3, round(dy.numel() * 2 / t3 / 1e3, 0))
    # dA (shared) and dx
    out[name + "_dA_v2"] = _time(lambda: L._lora2(1, 1, x, dZ, dA, 1, K, 1.0, T, R,
                                                  L._split(math.ceil(K / 128), T, 128), [(0, 0, 0, K)], seed, p, K))
    t2 = _time(lambda: L._lora2(2, 0, A, dZ, dx, K, 1, 1.0, T, R, 1, [(0, 0, 0, K)], seed, p, K))
    t3 = _time(lambda: nat.lora3_up(0, dx, K, dZ, R, A, K, T, R, 1.0, seed, th, ds, K, 0,
                                    [(0, 0, 0, K)], None, None, None, 0))
    out[name + "_dx"] = (t2, t3, round(dx.numel() * 4 / t3 / 1e3, 0))
    tw = 256 if math.ceil(K / 128) * math.ceil(T / 256) >= 512 else 128
    t4 = _time(lambda: nat.lora3_dxa(x, dx, dZ, A, dA, tw, seed, th, ds, K, 0))
    out[name + "_dxa_fused"] = (t4, round((x.numel() * 2 + dx.numel() * 4) / t4 / 1e3, 0))
out["note"] = "(v2 us, v3 us, v3 GB/s)"
print(json.dumps(out), flush=True)
