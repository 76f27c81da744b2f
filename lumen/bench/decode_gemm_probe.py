"""Decode-batch projection GEMMs (serving, Llama-2-7B, TP=1): hipBLASLt vs the decode MFMA GEMM.

For every projection shape and decode batch M (the serving graph buckets' block heights): the
library GEMM y = x @ W^T with the shipped TunableOp table (what the serving engine ran so far),
and every (BN, split-K) plan of ``kernels/decode_gemm.hip`` for the batch's block height.  The
weights rotate over copies totalling > 512 MB, so each launch reads W from HBM as in a decode
step (13 GB of weights per step; a repeated 100 MB matrix would be served by the 256 MB Infinity
Cache).  Writes the plans that beat the library by > 3% to ``--plans`` (the serving engine's
table, configs/kernels/decode_gemm_plans.json).

    python -m lumen.bench.decode_gemm_probe [--ms 64,128,192,256] [--plans out.json]
"""
from __future__ import annotations

import argparse
import json

import torch

SHAPES = (("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096),
          ("down", 4096, 11008), ("lm_head", 32000, 4096))


def _time(fn, n_w, iters=40):
    for i in range(6):
        fn(i % n_w)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i % n_w)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="64,128,192,256")
    ap.add_argument("--plans", default=None, help="write winning plans here (JSON)")
    ap.add_argument("--win", type=float, default=0.97, help="plan kept if dgemm < win x library")
    a = ap.parse_args()
    from lumen.ops.gemm import DG_BNS, DG_BNS8, decode_gemm, dg_bucket
    from lumen.utils.gemm_tuning import load_tuned_gemms

    load_tuned_gemms()
    dev = torch.device("cuda")
    ms = [int(x) for x in a.ms.split(",")]
    plans, rows = [], []
    tot = {}
    for name, N, K in SHAPES:
        n_w = max(2, -(-512 * 2**20 // (N * K * 2)))
        Ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(n_w)]
        for m in ms:
            x = torch.randn(m, K, device=dev, dtype=torch.bfloat16)
            lib = _time(lambda i: torch.matmul(x, Ws[i].t()), n_w)
            bm = dg_bucket(m)
            best = None
            cands = [(b, 4) for b in DG_BNS[bm]] + [(b, 8) for b in DG_BNS8.get(bm, ())]
            for bn, nw in cands:
                for s in (1, 2, 3, 4, 6, 8):
                    if s > K // 64 or -(-N // bn) * s > 4 * 256:
                        continue
                    try:
                        us = _time(lambda i: decode_gemm(x, Ws[i], bm, bn, s, nw), n_w)
                    except Exception as e:  # noqa: BLE001
                        print(json.dumps({"shape": name, "M": m, "BN": bn, "S": s, "NW": nw,
                                          "error": repr(e)[:200]}), flush=True)
                        continue
                    rows.append({"shape": name, "M": m, "BM": bm, "BN": bn, "S": s, "NW": nw,
                                 "us": round(us, 2)})
                    if best is None or us < best[0]:
                        best = (us, bn, s, nw)
            ref = x.float() @ Ws[0].float().t()
            err = ((decode_gemm(x, Ws[0], bm, best[1], best[2], best[3]).float() - ref).norm()
                   / ref.norm()).item()
            rec = {"shape": name, "M": m, "N": N, "K": K, "lib_us": round(lib, 2),
                   "dgemm_us": round(best[0], 2), "BM": bm, "BN": best[1], "S": best[2],
                   "NW": best[3],
                   "speedup": round(lib / best[0], 3), "rel_err": round(err, 5),
                   "lib_TBps": round(N * K * 2 / lib / 1e6, 2),
                   "dgemm_TBps": round(N * K * 2 / best[0] / 1e6, 2)}
            print(json.dumps(rec), flush=True)
            layers = 1 if name == "lm_head" else 32
            t = tot.setdefault(m, [0.0, 0.0])
            t[0] += lib * layers
            t[1] += min(lib, best[0]) * layers
            if best[0] < a.win * lib:
                plans.append({"N": N, "K": K, "BM": bm, "BN": best[1], "S": best[2],
                              "NW": best[3], "M_measured": m, "us": round(best[0], 2), "lib_us": round(lib, 2)})
        del Ws
        torch.cuda.empty_cache()
    for m, (l, d) in sorted(tot.items()):
        print(json.dumps({"M": m, "step_projections_ms_library": round(l / 1e3, 3),
                          "step_projections_ms_planned": round(d / 1e3, 3)}), flush=True)
    for r in rows:
        print(json.dumps(dict(r, sweep=True)))
    if a.plans:
        # one plan per (N, K, BM): the measured M of each bucket is its block height
        with open(a.plans, "w") as f:
            json.dump({"source": "lumen/bench/decode_gemm_probe.py (weights rotated over "
                                 "> 512 MB: HBM-resident like a decode step)",
                       "plans": plans}, f, indent=1)


if __name__ == "__main__":
    main()
