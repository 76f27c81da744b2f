"""Wave-quantisation probe for the frozen-weight GEMMs at the training shape (T = 8 x 512).

hipBLASLt runs the big MLP GEMMs with 256 x 256 macro tiles, one per CU at a time.  Two of them
leave a partly idle last wave on the 256-CU chip:

* gate|up forward  y[T, 22016] = x W_gu^T   16 x 86 = 1376 tiles = 5.375 waves
* down input-grad  dx[T, 11008] = dy W_dn   16 x 43 =  688 tiles = 2.69 waves

Splitting the output columns at a whole-wave boundary (20480 + 1536, 8192 + 2816) and writing the
two parts into column views of one buffer (ldc = full width, no copy) lets the tail run as its
own, separately tuned GEMM.  This probe times one-piece vs split back to back (power-capped, as
in a step) and prints the kernels a split call launches (no copy kernels expected).

    PYTHONPATH=. python scripts/probes/split_gemm_probe.py --tune OUT.csv [--dtype fp16]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil

import torch


def timeit(fn, iters=40, warm=8):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune", default=None, help="tune new shapes into this table copy")
    ap.add_argument("--T", type=int, default=4096)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    args = ap.parse_args()
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    from lumen.utils.gemm_tuning import DEFAULT_TABLE, load_tuned_gemms, start_gemm_tuning

    if args.tune:
        if not os.path.isfile(args.tune):
            shutil.copy(DEFAULT_TABLE, args.tune)
        start_gemm_tuning(args.tune)
    else:
        load_tuned_gemms()
    dev = torch.device("cuda")
    T, H, I = args.T, 4096, 11008
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(T, H, device=dev, generator=g).to(dt)
    Wgu = (torch.randn(2 * I, H, device=dev, generator=g) * 0.02).to(dt)
    WdnT = (torch.randn(I, H, device=dev, generator=g) * 0.02).to(dt)  # cached W_down^T
    y = torch.empty(T, 2 * I, device=dev, dtype=dt)
    dx = torch.empty(T, I, device=dev, dtype=dt)
    res = {}

    def gu_one():
        torch.mm(x, Wgu.t(), out=y)

    def make_split(W, out, n1):
        W1, W2 = W[:n1], W[n1:]
        o1, o2 = out[:, :n1], out[:, n1:]

        def f():
            torch.mm(x, W1.t(), out=o1)
            torch.mm(x, W2.t(), out=o2)
        return f

    def dx_one():
        torch.mm(x, WdnT.t(), out=dx)

    ref_y = torch.mm(x, Wgu.t())
    ref_dx = torch.mm(x, WdnT.t())
    variants = {"gate_up_one": gu_one, "down_dx_one": dx_one}
    for n1 in (20480, 16384):
        variants[f"gate_up_split{n1}"] = make_split(Wgu, y, n1)
    # (down input-grad split at 8192 + 2816: the 2816-column tail GEMM fails with "invalid
    # argument" inside TunableOp tuning, with and without rotating buffers -- not pursued)
    for name, fn in variants.items():
        y.zero_()
        dx.zero_()
        fn()
        torch.cuda.synchronize()
        err = ((y - ref_y).abs().max() if name.startswith("gate") else (dx - ref_dx).abs().max())
        res[name] = {"us": round(timeit(fn), 1), "max_err": float(err)}
        print(name, res[name], flush=True)
    # sustained interleaved with a filler GEMM (power state of a training step)
    filler_w = (torch.randn(H, I, device=dev, generator=g) * 0.02).to(dt)
    h = torch.randn(T, I, device=dev, generator=g).to(dt)
    out_f = torch.empty(T, H, device=dev, dtype=dt)

    def filler():
        torch.mm(h, filler_w.t(), out=out_f)
    base = timeit(filler)
    for name, fn in variants.items():
        def both(fn=fn):
            fn()
            filler()
        res[name]["us_with_filler_minus_filler"] = round(timeit(both) - base, 1)
        print(name, res[name], flush=True)
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        variants["gate_up_split20480"]()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    res["split_kernels"] = names
    print(json.dumps(res))
    # (with --tune, TunableOp writes the table named by start_gemm_tuning at process exit)


if __name__ == "__main__":
    main()
