#!/bin/bash
# Round 4: long-context training (same 4096 tokens per micro-step: 2 x 2048 and 1 x 4096; and
# 8 x 2048 = 16k tokens) -- Llama-2-7B ZeRO-3 + LoRA, one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_27}; mkdir -p $O
for cfg in "2048 2" "4096 1" "2048 8"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --no_serve --partitioned "" --seq_len $1 --micro_batch $2 --steps 10 --warmup 3 > $O/s$1_b$2.json 2> $O/s$1_b$2.err || { tail -5 $O/s$1_b$2.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/s$1_b$2.json')); e=d['extra']
print('seq $1 mb $2', d['value'], d['ms_per_step'], e['tflops_per_gpu'], e['peak_hbm_gb_max_rank'], d['config'])"
done
