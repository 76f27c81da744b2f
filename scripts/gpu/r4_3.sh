#!/bin/bash
# Round 4: activation checkpointing policies on the reference-compatible ZeRO-3 CLI (micro 2 x
# accum 4, seq 512, synthetic fixed-length rows): none / selective (gate|up recomputed) / full
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_3}; mkdir -p $O
for gc in false selective full; do
  timeout -k 10 400 python training/train_deepspeed_zero3.py --deepspeed configs/ds_config_zero3_mi355x.json \
      --synthetic --synthetic_samples 1024 --max_steps 40 --logging_steps 8 --save_strategy no \
      --gradient_checkpointing $gc --output_dir /tmp/ck_$gc --metrics_csv $O/m_$gc.csv > $O/zero3_gc_$gc.log 2>&1 || { tail -20 $O/zero3_gc_$gc.log; exit 1; }
  echo "== $gc"; grep -E "window_tokens" $O/zero3_gc_$gc.log | tail -3 | cut -c1-240; tail -1 $O/m_$gc.csv
done
