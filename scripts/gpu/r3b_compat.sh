#!/bin/bash
# reference-compatible CLI at its default flags (micro 2 x accum 4, seq 512, auto activation
# checkpointing) on the MI355X ZeRO-3 config, synthetic fixed-length rows; then with the
# reference's always-on checkpointing for comparison
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3b_compat}; mkdir -p $O
for gc in auto true; do
  timeout -k 10 400 python training/train_deepspeed_zero3.py --deepspeed configs/ds_config_zero3_mi355x.json \
      --synthetic --synthetic_samples 512 --max_steps 24 --logging_steps 8 --save_strategy no \
      --gradient_checkpointing $gc --output_dir /tmp/ck_$gc --metrics_csv /tmp/m_$gc.csv > $O/zero3_gc_$gc.log 2>&1 || { tail -20 $O/zero3_gc_$gc.log; exit 1; }
  grep -E "activation checkpointing|window_tokens" $O/zero3_gc_$gc.log | tail -2 | cut -c1-300
done
