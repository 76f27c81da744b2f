"""Micro-benchmark: weight-streaming decode GEMM vs torch.matmul (hipBLASLt, tuned table) at the
Llama-2-7B projection shapes for decode batches 1..16."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _time(fn, ws, reps=20):
    import torch

    for w in ws:
        fn(w)
    torch.cuda.synchronize()
    it = reps * len(ws)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(it):
        fn(ws[i % len(ws)])
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / it, 2)


def m1_forms():
    """Decode batches 1..4: row-group (form 0) vs rows-per-lane (form 1) weight-streaming kernels
    vs hipBLASLt; at M = 1 also the SwiGLU-fused down projection (vs swiglu kernel + GEMV)."""
    import torch

    from lumen.ops._native import native
    from lumen.ops.activation import swiglu
    from lumen.utils.gemm_tuning import load_tuned_gemms

    load_tuned_gemms()
    dev = "cuda"
    shapes = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096),
              "down": (4096, 11008), "lm_head": (32000, 4096)}
    for M in (1, 2, 3, 4):
        for name, (N, K) in shapes.items():
            copies = max(2, int(600e6 // (N * K * 2)))
            ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            row = {"M": M, "shape": name, "N": N, "K": K}
            for form in (0, 1):
                native().set_gemv_form(form)
                row[f"form{form}_us"] = _time(lambda w: native().skinny_gemm(x, w, y), ws)
                row[f"form{form}_TBps"] = round(N * K * 2 / (row[f"form{form}_us"] * 1e-6) / 1e12, 2)
            row["hipblaslt_us"] = _time(lambda w: torch.matmul(x, w.t()), ws)
            native().set_gemv_form(1)
            print(json.dumps(row), flush=True)
            del ws


def main():
    import torch

    if "--m1-forms" in sys.argv:
        return m1_forms()

    from lumen.ops._native import native
    from lumen.utils.gemm_tuning import load_tuned_gemms

    load_tuned_gemms()
    dev = "cuda"
    shapes = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096),
              "down": (4096, 11008)}
    # rotate over enough weight copies that every call streams from HBM (> 256 MB MALL)
    for M in (1, 2, 4, 8, 16):
        row = {"M": M}
        for name, (N, K) in shapes.items():
            copies = max(2, int(600e6 // (N * K * 2)))
            ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            res = {}
            for impl in ("lumen", "hipblaslt"):
                fn = (lambda w: native().skinny_gemm(x, w, y)) if impl == "lumen" else \
                    (lambda w: torch.matmul(x, w.t()))
                for w in ws:
                    fn(w)
                torch.cuda.synchronize()
                it = 20 * len(ws)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(it):
                    fn(ws[i % len(ws)])
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / it
                res[impl] = round(us, 2)
            res["lumen_TBps"] = round(N * K * 2 / (res["lumen"] * 1e-6) / 1e12, 2)
            row[name] = res
            del ws
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
