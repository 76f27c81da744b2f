"""The LM head's input gradient dH = dlogits [T, V] @ W [V, H] (Llama-2-7B: T 4096, V 32000,
H 4096): NN as today vs TN against a cached W^T (the frozen linears' form), heuristic and
TunableOp-tuned.  Graph-free event timing, 20 launches each.

    python scripts/probes/lm_head_dx_probe.py --out gpurun_out/x/gemms.csv"""
import argparse
import json
import os
import shutil
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
T, V, H = 4096, 32000, 4096


def _t(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--phase", default="both")
    a = ap.parse_args()
    from lumen.utils.gemm_tuning import DEFAULT_TABLE, load_tuned_gemms, start_gemm_tuning

    dev = torch.device("cuda")
    if a.phase == "both":
        rc = subprocess.call([sys.executable, "-u", __file__, "--out", a.out, "--phase", "tune"])
        if rc:
            sys.exit(rc)
    if a.phase == "tune":
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        shutil.copy(DEFAULT_TABLE, a.out)
        start_gemm_tuning(a.out, rotating_mb=0)
        d = torch.randn(T, V, device=dev, dtype=torch.bfloat16)
        wt = torch.randn(H, V, device=dev, dtype=torch.bfloat16) * 0.02
        torch.matmul(d, wt.t())
        torch.cuda.synchronize()
        return
    d = torch.randn(T, V, device=dev, dtype=torch.bfloat16)
    W = torch.randn(V, H, device=dev, dtype=torch.bfloat16) * 0.02
    Wt = W.t().contiguous()
    res = {}
    load_tuned_gemms()
    res["nn_shipped_table_us"] = round(_t(lambda: torch.matmul(d, W)), 1)
    res["tn_shipped_table_us"] = round(_t(lambda: torch.matmul(d, Wt.t())), 1)
    ref = torch.matmul(d.float()[:64], W.float())
    load_tuned_gemms(a.out)
    res["tn_tuned_us"] = round(_t(lambda: torch.matmul(d, Wt.t())), 1)
    res["rel_diff"] = ((torch.matmul(d, Wt.t())[:64].float() - ref).norm() / ref.norm()).item()
    res["pf_s_nn"] = round(2 * T * V * H / res["nn_shipped_table_us"] / 1e9, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
