#!/bin/bash
# Round 4: Llama-2-70B ZeRO-3 + LoRA on ONE GPU with the current tree (regression check of the
# memory logic: auto live budget, W^T budget, checkpointing auto)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_22}; mkdir -p $O
timeout -k 10 900 python bench.py --model llama2-70b --micro_batch 4 --steps ${STEPS:-3} --warmup ${WARM:-1} --no_serve --partitioned "" > $O/bench70b.json 2> $O/bench70b.err || { tail -20 $O/bench70b.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench70b.json')); e=d['extra']
print('70b', d['value'], d['ms_per_step'], d['config']['parallelism'], e['peak_hbm_gb_max_rank'], e['tflops_per_gpu'])"
