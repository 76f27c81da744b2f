#!/usr/bin/env python
"""Tune the hipBLASLt algorithm choice (PyTorch TunableOp) for the serving GEMM shapes and merge
the result into the shipped table (configs/tunableop/mi355x_gemms.csv).

    python scripts/tune_gemms.py --model llama2-7b --tp 1 [--out configs/tunableop/mi355x_gemms.csv]

Decode runs one GEMM per projection for every hipGraph batch bucket (1 ... 256 tokens) and the
prefill steps run 8192 / 16384 packed tokens; these shapes are tuned once here, offline, because
tuning inside a serving step would stall it (the engine only loads the table).  Training shapes
come from ``bench.py --tune_gemms``.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--tokens", default="1,2,4,8,16,32,64,96,128,160,192,224,256,8192,16384")
    a = ap.parse_args(argv)
    import torch

    from lumen.models import get_config
    from lumen.utils.gemm_tuning import DEFAULT_TABLE, start_gemm_tuning, tuned_entries

    out = a.out or DEFAULT_TABLE
    start_gemm_tuning(out)
    cfg = get_config(a.model)
    H, F, D = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    nh, nkv = cfg.num_attention_heads // a.tp, cfg.num_key_value_heads // a.tp
    shapes = [((nh + 2 * nkv) * D, H), (H, nh * D), (2 * F // a.tp, H), (H, F // a.tp),
              (cfg.vocab_size // a.tp, H)]
    dev = torch.device("cuda")
    ws = {s: torch.randn(*s, device=dev, dtype=torch.bfloat16) * 0.02 for s in shapes}
    for T in (int(t) for t in a.tokens.split(",")):
        for (N, K), w in ws.items():
            x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
            torch.matmul(x, w.t())
        torch.cuda.synchronize()
        print(f"tuned T={T} ({tuned_entries()} entries)", flush=True)
    print(f"table -> {out}")


if __name__ == "__main__":
    main()
