#!/bin/bash
# real-data path timing: variable-length (64-512) synthetic corpus, packed, through the
# reference-compatible zero3 entrypoint; GEMM table with packed M 1024-3072 vs heuristics; bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_11}; mkdir -p $O
run() {  # name, micro batch, env assignment, extra flag
  timeout -k 10 300 env $3 python training/train_deepspeed_zero3.py $4 --deepspeed configs/ds_config_zero3_mi355x.json \
    --synthetic --synthetic_min_len 64 --synthetic_samples 4096 --max_length 512 \
    --per_device_train_batch_size $2 --gradient_accumulation_steps 1 --max_steps 60 --logging_steps 20 \
    --save_strategy no --output_dir /tmp/lumen_varlen_$1 --metrics_csv $O/metrics.csv > $O/varlen_$1.log 2>&1 || return $?
  echo "$1: $(grep -E '^\{' $O/varlen_$1.log | tail -1 | cut -c1-300)"
}
run tok4096 8 LUMEN_X=1 --no_gradient_checkpointing\ --pack_tokens\ 4096 || exit $?
run mb8 8 LUMEN_X=1 --no_gradient_checkpointing || exit $?
run mb8_nopack 8 LUMEN_X=1 --no_gradient_checkpointing\ --no_packing || exit $?
run tok4096_ckpt 8 LUMEN_X=1 --pack_tokens\ 4096 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['value'])"
