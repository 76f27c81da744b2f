"""GEMM layout study for the frozen-weight linears (training shapes, T = 8 x 512 tokens).

Times torch.matmul for the forward (x @ W^T) and the input-gradient (dy @ W) GEMMs in both
weight layouts, plus the K-extended variants used to fold the LoRA up/down projections into the
base GEMM, with hipBLASLt's default heuristic and after TunableOp selection.

    python -m lumen.bench.gemm_bench [--tokens 4096] [--out gpurun_out/gemm_bench.json]
"""
from __future__ import annotations

import argparse
import json

import torch


def _time(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0  # us


def cases(T):
    H, F, nh = 4096, 11008, 32
    out = []
    for name, N, K in (("qkv", 3 * H, H), ("o", H, H), ("gate_up", 2 * F, H), ("down", H, F)):
        out.append((f"{name}.fwd", "tn", T, N, K))          # x[T,K] @ W[N,K]^T
        out.append((f"{name}.dx_nn", "nn", T, K, N))         # dy[T,N] @ W[N,K]
        out.append((f"{name}.dx_tn", "tn", T, K, N))         # dy[T,N] @ Wt[K,N]^T
    for name, N, K, ext in (("qkv", 3 * H, H, 48), ("o", H, H, 16)):
        for e in (ext, 64):
            out.append((f"{name}.fwd_ext{e}", "tn", T, N, K + e))
            out.append((f"{name}.dx_tn_ext{e}", "tn", T, K + e, N))
    return out


def run(T: int):
    dev = torch.device("cuda")
    res = {}
    import torch.cuda.tunable as tn

    for tune in (False, True):
        tn.enable(tune)
        tn.tuning_enable(tune)
        if tune:
            tn.set_max_tuning_duration(40)
            tn.set_filename("/tmp/gemm_bench_tunableop.csv", False)
        for name, lay, M, N, K in cases(T):
            a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            if lay == "tn":
                b = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
                fn = lambda a=a, b=b: torch.matmul(a, b.t())  # noqa: E731
            else:
                b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
                fn = lambda a=a, b=b: torch.matmul(a, b)  # noqa: E731
            us = _time(fn)
            tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
            res.setdefault(name, {})["tuned" if tune else "heuristic"] = {"us": round(us, 1),
                                                                          "tflops": round(tf, 1)}
            print(f"{name:18s} {'tuned' if tune else 'heur ':5s} M={M} N={N} K={K}: "
                  f"{us:8.1f} us {tf:7.1f} TF/s", flush=True)
            del a, b
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = run(a.tokens)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
