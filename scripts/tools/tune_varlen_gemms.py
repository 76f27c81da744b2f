"""Extend the shipped hipBLASLt (TunableOp) table to the packed-batch GEMM shapes.

Packed training rows (lumen.data.PackedCollator) carry sum(len) tokens rounded up to a multiple
of 256, so the frozen-weight GEMMs meet M in {256k}.  This runs the real model's forward and
backward once per M in [--m-min, --m-max] (step 256) with TunableOp tuning on, on top of the
existing table, and writes the merged table.

    python scripts/tools/tune_varlen_gemms.py --out configs/tunableop/mi355x_gemms.csv
"""
import argparse
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--m-min", type=int, default=1024)
    ap.add_argument("--m-max", type=int, default=6144)
    ap.add_argument("--out", required=True)
    ap.add_argument("--base", default=os.path.join(ROOT, "configs", "tunableop", "mi355x_gemms.csv"))
    args = ap.parse_args()
    if os.path.abspath(args.base) != os.path.abspath(args.out) and os.path.isfile(args.base):
        shutil.copyfile(args.base, args.out)
    import torch

    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model
    from lumen.utils.gemm_tuning import start_gemm_tuning, tuned_entries

    start_gemm_tuning(args.out)
    dev = torch.device("cuda")
    m = build_model(args.model, dtype=torch.bfloat16, device=dev, init="random", seed=0)
    apply_lora(m, LoraConfig(r=16, lora_dropout=0.05))
    from lumen.models.layers import configure_backward_layout

    configure_backward_layout(m)
    m.train()
    for p in m.parameters():
        if p.requires_grad:
            p.grad = torch.zeros_like(p)
    V = m.config.vocab_size
    for M in range(args.m_min, args.m_max + 1, 256):
        t0 = time.time()
        # two sequences per row (the packed path: varlen attention, per-sequence positions)
        cu = (0, M // 2, M)
        ids = torch.randint(3, V, (1, M), device=dev)
        labels = torch.roll(ids, -1, 1)
        pos = torch.cat([torch.arange(M // 2), torch.arange(M - M // 2)]).to(torch.int32).to(dev)
        loss = m(ids, labels, M, pos, cu_seqlens=cu)
        loss.backward()
        torch.cuda.synchronize()
        print(f"M={M}: {time.time() - t0:.1f}s, table entries {tuned_entries()}", flush=True)
    # TunableOp writes the table named by set_filename (start_gemm_tuning) at process exit
    print(f"{args.out}: {tuned_entries()} entries (written at exit)")


if __name__ == "__main__":
    main()
