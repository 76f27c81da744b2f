"""Where the decode GEMM's time goes at M = 256: every (BN, waves, split-K) plan timed
  * as shipped (flags 0),
  * with the k loop's ds_reads + MFMAs skipped (flags 4: the load pipeline alone),
  * with one weight matrix re-used (Infinity-Cache resident: HBM taken out),
plus hipBLASLt for reference.  Every time is graph-replayed GPU time.  Per-CU L2->CU traffic of a plan: (BM + BN) * K / S * 2 bytes.

    python scripts/probes/dgemm_costprobe.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from lumen.bench.decode_gemm_probe import SHAPES  # noqa: E402


def _time(fn, n_w, iters=40):
    """GPU time per call: the calls are captured in a hipGraph and replayed (a Python-issued
    loop of ~20-50 us kernels is host-bound and measures the launch path, not the kernel)."""
    for i in range(6):
        fn(i % n_w)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        fn(0)
        with torch.cuda.graph(g, stream=st):
            for i in range(iters):
                fn(i % n_w)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * iters) * 1000.0


def main():
    from lumen.ops.gemm import decode_gemm
    from lumen.utils.gemm_tuning import load_tuned_gemms

    load_tuned_gemms()
    dev = torch.device("cuda")
    M = 256
    for name, N, K in SHAPES[:4]:
        n_w = max(2, -(-512 * 2**20 // (N * K * 2)))
        Ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(n_w)]
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        lib = _time(lambda i: torch.matmul(x, Ws[i].t()), n_w)
        lib_hot = _time(lambda i: torch.matmul(x, Ws[0].t()), n_w)
        print(json.dumps({"shape": name, "lib_us": round(lib, 2), "lib_hot_us": round(lib_hot, 2)}),
              flush=True)
        for bn in (64, 128):
            for nw in (4, 8):
                for s in (1, 2, 3, 4):
                    blocks = -(-N // bn) * s
                    if blocks > 2 * 256 or blocks < 96:
                        continue
                    try:
                        t0 = _time(lambda i: decode_gemm(x, Ws[i], 256, bn, s, nw), n_w)
                        t4 = _time(lambda i: decode_gemm(x, Ws[i], 256, bn, s, nw, flags=4), n_w)
                        th = _time(lambda i: decode_gemm(x, Ws[0], 256, bn, s, nw), n_w)
                    except Exception as e:  # noqa: BLE001
                        print(json.dumps({"shape": name, "err": repr(e)[:120]}), flush=True)
                        continue
                    per_cu = (256 + bn) * K // s * 2
                    print(json.dumps({"shape": name, "BN": bn, "NW": nw, "S": s, "blocks": blocks,
                                      "us": round(t0, 2), "no_compute_us": round(t4, 2),
                                      "w_hot_us": round(th, 2),
                                      "per_block_MB": round(per_cu / 2**20, 2),
                                      "GBps_per_block_no_compute": round(per_cu / t4 / 1e3, 1)}),
                          flush=True)
        del Ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
