#!/bin/bash
# real-data path: packed-vs-padded GPU test, GEMM table extended to packed M (256-multiples),
# variable-length (64-512) synthetic corpus through the reference-compatible zero3 entrypoint,
# and the bench on the same box for the comparison.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_10}; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_packing_gpu.py -v --timeout 120 --timeout-method thread > $O/pack_test.txt 2>&1
rc=$?; tail -3 $O/pack_test.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u scripts/tools/tune_varlen_gemms.py --m-min 1024 --m-max 6144 --out $O/mi355x_gemms_varlen.csv > $O/tune.log 2>&1 || exit $?
tail -3 $O/tune.log
export LUMEN_GEMM_TABLE=$O/mi355x_gemms_varlen.csv
for mb in 16 8; do
  timeout -k 10 300 python training/train_deepspeed_zero3.py --deepspeed configs/ds_config_zero3_mi355x.json \
    --synthetic --synthetic_min_len 64 --synthetic_samples 4096 --max_length 512 \
    --per_device_train_batch_size $mb --gradient_accumulation_steps 1 --max_steps 40 --logging_steps 10 \
    --save_strategy no --output_dir /tmp/lumen_varlen_$mb --metrics_csv $O/metrics.csv > $O/varlen_mb$mb.log 2>&1 || exit $?
  grep -E "tokens_per_second|samples_per_second|tok/s" $O/varlen_mb$mb.log | tail -3
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['value'])"
