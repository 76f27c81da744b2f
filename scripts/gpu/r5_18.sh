#!/bin/bash
# Round 5: activation recompute with per-layer granularity on the reference-compatible ZeRO-3 CLI
# (micro 2 x accum 4, seq 512): none / selective:16 / selective / full:16 / full
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5_18}; mkdir -p $O
for gc in false selective:16 selective full:16 full; do
  tag=${gc/:/_}
  timeout -k 10 400 python training/train_deepspeed_zero3.py --deepspeed configs/ds_config_zero3_mi355x.json \
      --synthetic --synthetic_samples 1024 --max_steps 40 --logging_steps 8 --save_strategy no \
      --gradient_checkpointing $gc --output_dir /tmp/ck_$tag --metrics_csv $O/m_$tag.csv > $O/zero3_gc_$tag.log 2>&1 || { tail -20 $O/zero3_gc_$tag.log; exit 1; }
  echo "== $gc $(grep -E "window_tokens" $O/zero3_gc_$tag.log | tail -1 | grep -o '"window_tokens_per_second": [0-9.]*') peak $(tail -1 $O/m_$tag.csv | cut -d, -f7)"
done
