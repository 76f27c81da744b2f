"""Whole-wave column splits for the serving prefill / mixed-step projections (Llama-2-7B, M =
2048 and 4096 tokens per step): tune the two parts of every split with TunableOp (written to
``--out``, the shipped table plus the new rows), then time split vs single GEMM, graph-replayed,
weights rotating over > 512 MB.

    python scripts/probes/tune_serve_splits.py --out gpurun_out/x/gemms.csv [--max_tail 0.75]"""
import argparse
import json
import os
import shutil
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

SHAPES = (("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096),
          ("down", 4096, 11008),
          # training: the down projection's input gradient dY @ W (TN against the cached W^T)
          ("down_dx", 11008, 4096))


def _time(fn, n_w, iters=20):
    for i in range(4):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--ms", default="2048,4096")
    ap.add_argument("--max_tail", type=float, default=0.75)
    ap.add_argument("--phase", default="both", choices=["both", "tune", "time"])
    ap.add_argument("--only", default="", help="comma list of shape names (default: all)")
    a = ap.parse_args()
    if a.phase == "both":  # TunableOp writes its file at process exit: tune in a child first
        import subprocess
        rc = subprocess.call([sys.executable, "-u", __file__, "--out", a.out, "--ms", a.ms,
                              "--max_tail", str(a.max_tail), "--phase", "tune", "--only", a.only])
        if rc:
            sys.exit(rc)
        a.phase = "time"
    import lumen.ops.gemm as G
    from lumen.utils.gemm_tuning import DEFAULT_TABLE, load_tuned_gemms, start_gemm_tuning

    G.SPLIT_MAX_TAIL = a.max_tail
    dev = torch.device("cuda")
    ms = [int(m) for m in a.ms.split(",")]
    cases = []
    for name, N, K in SHAPES:
        if a.only and name not in a.only.split(","):
            continue
        for M in ms:
            cases.append((name, N, K, M, G.split_cols(M, N)))
    if a.phase == "tune":
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        shutil.copy(DEFAULT_TABLE, a.out)
        # rotating buffers off: they copy ldc * n elements from C's pointer, which overruns the
        # column-view outputs of the parts
        start_gemm_tuning(a.out, rotating_mb=0)
        for name, N, K, M, n1 in cases:
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            torch.matmul(x, w.t())                       # the single GEMM (tuned if new)
            if n1:
                y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                torch.mm(x, w[:n1].t(), out=y[:, :n1])   # the two parts
                torch.mm(x, w[n1:].t(), out=y[:, n1:])
            torch.cuda.synchronize()
            print(json.dumps({"tuned": name, "M": M, "n1": n1}), flush=True)
        return
    assert load_tuned_gemms(a.out), a.out
    for name, N, K, M, n1 in cases:
        if not n1:
            continue
        n_w = max(2, -(-512 * 2**20 // (N * K * 2)))
        Ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(n_w)]
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        one = _time(lambda i: torch.matmul(x, Ws[i].t()), n_w)
        ys = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

        def split(i):
            torch.mm(x, Ws[i][:n1].t(), out=ys[:, :n1])
            torch.mm(x, Ws[i][n1:].t(), out=ys[:, n1:])

        two = _time(split, n_w)
        ref = torch.matmul(x, Ws[0].t())
        split(0)
        err = ((ys.float() - ref.float()).norm() / ref.float().norm()).item()
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "n1": n1,
                          "single_us": round(one, 2), "split_us": round(two, 2),
                          "speedup": round(one / two, 3), "rel_diff": round(err, 6),
                          "plan_taken": G._split_plan(x, Ws[0])}), flush=True)
        del Ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
