"""Decode-batch GEMM layouts on the library: y = x W^T as matmul(x, W^T) (the serving path, tuned
table) vs y^T = matmul(W, x^T) (weights as the left operand, tuned here by TunableOp) plus the
transpose back.  One JSON line per (M, shape)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.cuda.tunable as tn  # noqa: E402


def _time(fn, ws, reps=20):
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


from lumen.utils.gemm_tuning import DEFAULT_TABLE  # noqa: E402

tn.enable(True)
tn.tuning_enable(True)
tn.set_max_tuning_duration(30)
tn.set_max_tuning_iterations(50)
tn.set_rotating_buffer_size(1024)
tn.set_filename("/tmp/lumen_layout_probe.csv", False)
tn.read_file(DEFAULT_TABLE)
dev = "cuda"
shapes = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008)}
for M in (64, 128, 256):
    for name, (N, K) in shapes.items():
        copies = max(2, int(600e6 // (N * K * 2)))
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        xt = x.t().contiguous()
        a = _time(lambda w: torch.matmul(x, w.t()), ws)
        b = _time(lambda w: torch.matmul(w, xt), ws)
        c = _time(lambda w: torch.matmul(w, xt).t().contiguous(), ws)
        print(json.dumps({"M": M, "shape": name, "x_Wt_us": a, "W_xt_us": b,
                          "W_xt_plus_transpose_us": c}), flush=True)
        del ws
