"""(Probe: needs scripts/probes/batch_gemm.hip built into the extension with a `batch_gemm`
binding; it is not part of the shipped build.)

Decode-batch projections: the MFMA batch GEMM (kernels/batch_gemm.hip) vs hipBLASLt with the
tuned table, Llama-2-7B shapes (q|k|v, o, gate|up, down, lm_head) at M = 8..256.

    python -m lumen.bench.batch_gemm_bench [--ms 8,16,...] > out.jsonl

One JSON line per (shape, M): both times (CUDA events over --iters back-to-back calls, weights
rotated through a set larger than the 256 MB Infinity Cache so W streams from HBM as in a
decode step), the weight bandwidth, and the max abs error of each against an f32 reference."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096),
          "down": (4096, 11008), "lm_head": (32000, 4096)}


def main():
    import torch

    from lumen.ops._native import native
    from lumen.utils.gemm_tuning import load_tuned_gemms

    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="8,16,32,64,96,128,160,192,224,256")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    load_tuned_gemms()
    C = native()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        nrot = max(2, int(600e6 // (N * K * 2)) + 1)  # > 256 MB MALL: W streams from HBM
        ws = [torch.randn(N, K, device=dev, generator=g).mul_(0.02).bfloat16() for _ in range(nrot)]
        for M in (int(v) for v in a.ms.split(",")):
            x = torch.randn(M, K, device=dev, generator=g).bfloat16()
            ref = x.float() @ ws[0].float().t()
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            C.batch_gemm(x, ws[0], y)
            err_b = (y.float() - ref).abs().max().item()
            err_h = (torch.matmul(x, ws[0].t()).float() - ref).abs().max().item()

            def timed(fn):
                for i in range(3):
                    fn(ws[i % nrot])
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(a.iters):
                    fn(ws[i % nrot])
                e1.record()
                torch.cuda.synchronize()
                return e0.elapsed_time(e1) * 1e3 / a.iters

            t_b = timed(lambda w: C.batch_gemm(x, w, y))
            t_h = timed(lambda w: torch.matmul(x, w.t()))
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "batch_us": round(t_b, 1),
                              "hipblaslt_us": round(t_h, 1),
                              "batch_tb_s": round(N * K * 2 / t_b / 1e6, 2),
                              "speedup": round(t_h / t_b, 2), "err_batch": err_b,
                              "err_hipblaslt": err_h}), flush=True)
        del ws


if __name__ == "__main__":
    main()
