"""Decode-batch projection GEMMs (serving, Llama-2-7B, TP=1): where hipBLASLt stands at M = 64..256.

For every projection shape and decode batch M: y = x @ W^T with the shipped TunableOp table (what
the serving engine runs), the same after fresh tuning, and the transposed orientation y^T = W @ x^T
(fresh tuning).  Prints one JSON line per case: microseconds and the weight-streaming rate.

    python -m lumen.bench.decode_gemm_probe [--ms 64,128,192,256]
"""
from __future__ import annotations

import argparse
import json

import torch

SHAPES = (("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096),
          ("down", 4096, 11008), ("lm_head", 32000, 4096))


def _time(fn, iters=30):
    for _ in range(5):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="64,128,192,256")
    a = ap.parse_args()
    import torch.cuda.tunable as tn

    from lumen.utils.gemm_tuning import load_tuned_gemms

    dev = torch.device("cuda")
    ms = [int(x) for x in a.ms.split(",")]
    # weights: distinct buffers per shape, 13 GB total is not needed -- one per shape
    Ws = {n: torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for n, N, K in SHAPES}
    xs = {(m, K): torch.randn(m, K, device=dev, dtype=torch.bfloat16)
          for m in ms for K in {k for _, _, k in SHAPES}}
    res = {}
    for mode in ("table", "fresh"):
        if mode == "table":
            load_tuned_gemms()
        else:
            tn.enable(True)
            tn.tuning_enable(True)
            tn.set_max_tuning_duration(30)
            tn.set_filename("/tmp/decode_probe_tunableop.csv", False)
        for n, N, K in SHAPES:
            W = Ws[n]
            for m in ms:
                x = xs[(m, K)]
                us = _time(lambda: torch.matmul(x, W.t()))
                res[(mode, "xWt", n, m)] = us
                if mode == "fresh":
                    res[(mode, "Wxt", n, m)] = _time(lambda: torch.matmul(W, x.t()))
    for (mode, form, n, m), us in sorted(res.items()):
        N, K = next((N, K) for nn, N, K in SHAPES if nn == n)
        print(json.dumps({"mode": mode, "form": form, "shape": n, "M": m, "N": N, "K": K,
                          "us": round(us, 2), "weight_TBps": round(N * K * 2 / us / 1e6, 2),
                          "TFps": round(2 * m * N * K / us / 1e6, 1)}), flush=True)
    # per-M totals of one decode step's projections (32 layers + lm_head)
    for mode, form in (("table", "xWt"), ("fresh", "xWt"), ("fresh", "Wxt")):
        for m in ms:
            tot = sum(res[(mode, form, n, m)] * (1 if n == "lm_head" else 32) for n, _, _ in SHAPES)
            print(json.dumps({"mode": mode, "form": form, "M": m, "step_ms": round(tot / 1e3, 3)}))


if __name__ == "__main__":
    main()
