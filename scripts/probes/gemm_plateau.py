"""Sustained vs. burst bf16 GEMM throughput on one MI355X (is ~1.5 PF/s the training plateau?).

For the eight frozen-weight GEMMs of one Llama-2-7B layer at T = 8 x 512 tokens (the shapes and
layouts the training step runs, with the tuned table loaded) this times each shape twice:

* burst: 5 calls after a 1 s idle gap, the regime TunableOp's candidate timing sees;
* sustained: the whole layer's GEMM sequence repeated back to back for ~2 s, as in a step.

Plus two large square shapes with the library heuristic.  Output: one JSON line per case and
``gpurun_out/s4_gemm/plateau.json``.

    python scripts/probes/gemm_plateau.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from lumen.utils.gemm_tuning import load_tuned_gemms  # noqa: E402

T, H, F = 4096, 4096, 11008
# (name, out_features, in_features, layout): fwd = x[T,K] @ W[N,K]^T, dx = dy[T,N] @ Wt[K,N]^T
# (the step keeps transposed copies of the frozen weights for the input gradients), o.dx = NN
LAYER = [("qkv.fwd", 3 * H, H, "tn"), ("o.fwd", H, H, "tn"), ("gate_up.fwd", 2 * F, H, "tn"),
         ("down.fwd", H, F, "tn"), ("qkv.dx", H, 3 * H, "tn"), ("o.dx", H, H, "nn"),
         ("gate_up.dx", H, 2 * F, "tn"), ("down.dx", F, H, "tn")]


def ev_time(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / n


def main():
    os.makedirs("gpurun_out/s4_gemm", exist_ok=True)
    tuned = load_tuned_gemms()
    dev = torch.device("cuda")
    fns = []
    for name, N, K, lay in LAYER:
        a = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        if lay == "tn":
            b = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
            fn = (lambda a=a, b=b: torch.matmul(a, b.t()))
        else:
            b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
            fn = (lambda a=a, b=b: torch.matmul(a, b))
        fns.append((name, 2.0 * T * N * K, fn))
    res = {"tuned_table": tuned, "burst": {}, "sustained": {}}
    for name, fl, fn in fns:
        fn()
        torch.cuda.synchronize()
        time.sleep(1.0)
        us = ev_time(fn, 5)
        res["burst"][name] = {"us": round(us, 1), "tflops": round(fl / us / 1e6, 1)}
        print(json.dumps({"case": name, "mode": "burst", **res["burst"][name]}), flush=True)
    # sustained: the layer's sequence back to back, per-shape time from per-shape event pairs
    total_fl = sum(fl for _, fl, _ in fns)
    acc = {name: 0.0 for name, _, _ in fns}
    reps = 0
    t0 = time.time()
    while time.time() - t0 < 2.0:
        for name, _, fn in fns:
            acc[name] += ev_time(fn, 1)
        reps += 1
    for name, fl, _ in fns:
        us = acc[name] / reps
        res["sustained"][name] = {"us": round(us, 1), "tflops": round(fl / us / 1e6, 1)}
        print(json.dumps({"case": name, "mode": "sustained", **res["sustained"][name]}), flush=True)
    layer_us = sum(acc.values()) / reps
    res["sustained_layer"] = {"us": round(layer_us, 1), "tflops": round(total_fl / layer_us / 1e6, 1),
                              "reps": reps}
    print(json.dumps({"case": "layer", "mode": "sustained", **res["sustained_layer"]}), flush=True)
    torch.cuda.tunable.enable(False)
    for M in (8192, 16384):
        a = torch.randn(M, M, device=dev, dtype=torch.bfloat16)
        b = torch.randn(M, M, device=dev, dtype=torch.bfloat16)
        fn = (lambda a=a, b=b: torch.matmul(a, b.t()))
        ev_time(fn, 3)
        us = ev_time(fn, 20 if M == 8192 else 5)
        res[f"square{M}"] = {"us": round(us, 1), "tflops": round(2.0 * M ** 3 / us / 1e6, 1)}
        print(json.dumps({"case": f"square{M}", "mode": "heuristic", **res[f"square{M}"]}),
              flush=True)
        del a, b
    with open("gpurun_out/s4_gemm/plateau.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
