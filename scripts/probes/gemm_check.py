"""Correctness + timing of one TN GEMM shape under a given TunableOp table (no tuning):
max abs error vs an fp32 matmul, and us per call.

    PYTHONPATH=. python scripts/probes/gemm_check.py TABLE M N K"""
from __future__ import annotations

import sys

import torch


def main(table, M, N, K):
    import torch.cuda.tunable as tn

    tn.enable(True)
    tn.tuning_enable(False)
    tn.read_file(table)
    dev = torch.device("cuda")
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
    ref = x.float() @ w.float().t()
    y = torch.mm(x, w.t())
    torch.cuda.synchronize()
    err = (y.float() - ref).abs().max().item()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        torch.mm(x, w.t())
    a.record()
    for _ in range(20):
        torch.mm(x, w.t())
    b.record()
    torch.cuda.synchronize()
    print(f"{table} M={M} N={N} K={K}: max_err {err:.4f} (ref max {ref.abs().max().item():.2f}), "
          f"{a.elapsed_time(b) / 20 * 1000:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], *map(int, sys.argv[2:5]))
