"""Sustained-GEMM probe: per-batch timing of the q|k|v forward GEMM over ~12 s to expose clock
throttling (compare with rocm-smi samples taken alongside)."""
import time

import torch


def main():
    dev = torch.device("cuda")
    x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    w = torch.randn(12288, 4096, device=dev, dtype=torch.bfloat16) * 0.02
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_end = time.time() + 12
    i = 0
    while time.time() < t_end:
        s.record()
        for _ in range(100):
            y = x @ w.t()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 10.0
        print(f"batch {i:3d} t={time.time():.1f} {us:7.1f} us/gemm {2*4096*12288*4096/us/1e6:7.1f} TF/s",
              flush=True)
        i += 1
    # bursty: one GEMM then idle 1 ms
    for j in range(5):
        torch.cuda.synchronize()
        time.sleep(0.05)
        s.record(); y = x @ w.t(); e.record(); torch.cuda.synchronize()
        print(f"isolated {j}: {s.elapsed_time(e)*1000:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
