"""lora3_dy (fused dZ / dB pass over dY) timed per dtype and dY magnitude at the Llama-2-7B
q|k|v shape: the fp16 training step showed it at 54.8 us/call vs 29.3 us in bf16
(profiles/r3d/fp16).  One JSON line per (dtype, scale, B magnitude)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from lumen.ops._native import native
    from lumen.ops.lora import _dy_tw

    nat = native()
    dev = torch.device("cuda")
    T, r = 4096, 16
    segs = [(0, 4096, 0, 0), (4096, 4096, 16, 4096), (8192, 4096, 32, 8192)]
    N, R = 12288, 48

    def run(dt, scale, bmag, zmag=1.0):
        dy = (torch.randn(T, N, device=dev) * scale).to(dt)
        B = torch.randn(N, r, device=dev) * bmag
        Z = torch.randn(T, R, device=dev) * zmag
        dZ = torch.zeros(T, R, device=dev)
        dB = torch.zeros(N, r, device=dev)
        tw = _dy_tw(segs, T)

        def f():
            nat.lora3_dy(dy, dy.stride(0), B, r, Z, R, dZ, R, dB, T, tw, 2.0,
                         [(n_off, r_off, b_off, n_len) for (n_off, n_len, r_off, b_off) in segs])
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            f()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / 50

    for dt in (torch.bfloat16, torch.float16):
        for scale, bmag, zmag in ((1e-3, 1e-2, 1.0), (1.0, 1e-2, 1.0), (1e-3, 0.0, 1.0),
                                  (1e-3, 1e-2, 0.0), (64.0, 1e-2, 1.0)):
            print(json.dumps({"dtype": str(dt), "dy_scale": scale, "B_mag": bmag, "Z_mag": zmag,
                              "us": round(run(dt, scale, bmag, zmag), 1)}), flush=True)


if __name__ == "__main__":
    main()
