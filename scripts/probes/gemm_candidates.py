"""List every TunableOp candidate for the training-step GEMM shapes with its tuning-time
duration (PYTORCH_TUNABLEOP_VERBOSE log), fastest first: the runner-ups are what
``scripts/gpu/insitu_gemm.sh`` then times inside the power-capped training step.

    PYTORCH_TUNABLEOP_VERBOSE=3 PYTHONPATH=. python scripts/probes/gemm_candidates.py OUT.json"""
from __future__ import annotations

import json
import os
import re
import sys
import tempfile

import torch

# (name, M (tokens), N (out features), K): forward y = x W^T and input-grad dX = dY (W^T)^T
SHAPES = [
    ("qkv_fold_fwd", 4096, 12288, 4160), ("o_fold_fwd", 4096, 4096, 4160),
    ("gate_up_fwd_part", 4096, 20480, 4096), ("down_fwd", 4096, 4096, 11008),
    ("qkv_dx", 4096, 4096, 12288), ("o_dx", 4096, 4096, 4096),
    ("gate_up_dx", 4096, 4096, 22016), ("down_dx", 4096, 11008, 4096),
]


def main(out_path):
    import torch.cuda.tunable as tn

    log = tempfile.mktemp(suffix=".log")
    tn.enable(True)
    tn.tuning_enable(True)
    tn.set_filename(tempfile.mktemp(suffix=".csv"), False)
    tn.set_max_tuning_duration(30)
    tn.set_max_tuning_iterations(30)
    tn.set_rotating_buffer_size(0)
    dev = torch.device("cuda")
    res = {}
    fd = os.dup(2)
    for name, M, N, K in SHAPES:
        x = torch.randn(M, K, device=dev).bfloat16()
        w = torch.randn(N, K, device=dev).bfloat16() * 0.02
        with open(log, "w") as f:
            os.dup2(f.fileno(), 2)
            os.dup2(f.fileno(), 1)
            torch.mm(x, w.t())
            torch.cuda.synchronize()
            sys.stdout.flush()
        os.dup2(fd, 2)
        os.dup2(fd, 1)
        text = open(log).read()
        cands = {}
        for m in re.finditer(r"(Gemm_(?:Hipblaslt|Rocblas)_\d+|Default)\S*\s.*?(\d+\.\d+)\s*ms", text):
            t = float(m.group(2))
            cands[m.group(1)] = min(t, cands.get(m.group(1), 1e9))
        best = sorted(cands.items(), key=lambda kv: kv[1])
        res[name] = {"shape": [M, N, K], "n_candidates": len(cands), "top": best[:8],
                     "log_head": text[:1500] if not cands else ""}
        print(name, len(cands), best[:4], flush=True)
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
