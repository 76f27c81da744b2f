"""Decode GEMM at M = 256 (the full decode bucket): hipBLASLt vs kernels/decode_gemm.hip with
the k-rotated loop (flags 1) and the k-tiled x layout (flags 2), every (BN, waves, split-K).
Weights rotate over > 512 MB so they stream from HBM as in a decode step.

    python scripts/probes/dgemm_variants.py [--m 256]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from lumen.bench.decode_gemm_probe import SHAPES, _time  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=256)
    a = ap.parse_args()
    from lumen.ops.gemm import decode_gemm, x_ktiled
    from lumen.utils.gemm_tuning import load_tuned_gemms

    load_tuned_gemms()
    dev = torch.device("cuda")
    M = a.m
    tot = {}
    for name, N, K in SHAPES[:4]:
        n_w = max(2, -(-512 * 2**20 // (N * K * 2)))
        Ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(n_w)]
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        xt = x_ktiled(x)
        lib = _time(lambda i: torch.matmul(x, Ws[i].t()), n_w)
        best = {}
        for fl in (0, 1, 2, 3):
            xin = xt if fl & 2 else x
            for bn in (64, 128):
                for nw in (4, 8):
                    for s in (1, 2, 3, 4, 6):
                        if s > K // 64 or -(-N // bn) * s > 4 * 256:
                            continue
                        try:
                            us = _time(lambda i: decode_gemm(xin, Ws[i], 256, bn, s, nw,
                                                             flags=fl, m=M), n_w)
                        except Exception as e:  # noqa: BLE001
                            print(json.dumps({"shape": name, "err": repr(e)[:160]}), flush=True)
                            continue
                        if fl not in best or us < best[fl][0]:
                            best[fl] = (us, bn, nw, s)
        rec = {"shape": name, "M": M, "lib_us": round(lib, 2),
               **{f"f{fl}": {"us": round(b[0], 2), "BN": b[1], "NW": b[2], "S": b[3],
                             "vs_lib": round(lib / b[0], 3)} for fl, b in best.items()}}
        print(json.dumps(rec), flush=True)
        t = tot.setdefault("lib", 0.0)
        tot["lib"] = t + lib * 32
        for fl, b in best.items():
            tot[f"f{fl}"] = tot.get(f"f{fl}", 0.0) + min(b[0], lib) * 32
        del Ws
        torch.cuda.empty_cache()
    print(json.dumps({"M": M, "step_ms": {k: round(v / 1e3, 3) for k, v in tot.items()}}))


if __name__ == "__main__":
    main()
