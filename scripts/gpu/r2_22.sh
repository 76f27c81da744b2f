#!/bin/bash
# LoRA fold: numerics, GEMM table extended with the K+64 shapes, same-box bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_22}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_packing_gpu.py -k "fold or lora or packed or llama" -v --timeout 120 --timeout-method thread > $O/t.txt 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t.txt | tail -8; [ $rc -eq 0 ] || exit $rc
cp configs/tunableop/mi355x_gemms.csv $O/table.csv
timeout -k 10 400 python bench.py --steps 5 --warmup 3 --tune_gemms $O/table.csv > $O/tune.json 2> $O/tune.err || exit $?
grep -c . $O/table.csv
export LUMEN_GEMM_TABLE=$O/table.csv
for v in 0 1 0 1; do
  LUMEN_LORA_FOLD=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$v.json 2> $O/bench_$v.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('fold=$v', d['ms_per_step'], d['value'], d['extra']['gemm_table_entries'])"
done
