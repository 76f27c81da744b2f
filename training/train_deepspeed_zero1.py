#!/usr/bin/env python3
"""LoRA + ZeRO-1 (reference training/train_deepspeed_zero1.py).

Same flags and defaults as the reference script; runs on lumen (MI355X RCCL / CPU gloo).
    python training/train_deepspeed_zero1.py --synthetic --max_steps 50
    torchrun --nproc_per_node 8 --master-addr 127.0.0.1 training/train_deepspeed_zero1.py ...
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lumen.cli.train import main  # noqa: E402

if __name__ == "__main__":
    main("zero1")
