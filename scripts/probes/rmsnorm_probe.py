"""RMSNorm forward / backward at the training shape (4096 rows x 4096, bf16, fused residual)
under different occupancy caps (``set_rms_lds``: dynamic LDS bytes per workgroup).  Prints us per
call and effective TB/s (fwd: x + residual in, y + sum out; bwd: dy + s + residual grad in, dx
out).    PYTHONPATH=. python scripts/probes/rmsnorm_probe.py"""
from __future__ import annotations

import json

import torch


def timeit(fn, iters=50, warm=10):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1000.0


def main():
    from lumen.ops._native import native

    C = native()
    dev = torch.device("cuda")
    T, H = 4096, 4096
    x = torch.randn(T, H, device=dev).bfloat16()
    res = torch.randn(T, H, device=dev).bfloat16()
    w = torch.rand(H, device=dev).bfloat16()
    y = torch.empty_like(x)
    s = torch.empty_like(x)
    rstd = torch.empty(T, device=dev)
    dy = torch.randn(T, H, device=dev).bfloat16()
    dres = torch.randn(T, H, device=dev).bfloat16()
    dx = torch.empty_like(x)
    nbytes = T * H * 2
    out = []
    for lds in (0, 20480, 32768, 40960, 54272):
        C.set_rms_lds(lds, lds)
        tf = timeit(lambda: C.rmsnorm_fwd(x, res, w, y, s, rstd, 1e-5))
        tb = timeit(lambda: C.rmsnorm_bwd(dy, s, w, rstd, dres, dx, None))
        r = {"lds": lds, "fwd_us": round(tf, 2), "fwd_TBs": round(4 * nbytes / tf / 1e6, 2),
             "bwd_us": round(tb, 2), "bwd_TBs": round(4 * nbytes / tb / 1e6, 2)}
        print(json.dumps(r), flush=True)
        out.append(r)
    C.set_rms_lds(0, 0)


if __name__ == "__main__":
    main()
