#!/bin/bash
# extend the TunableOp table with the LoRA-fold shapes: K = 4160 forward GEMMs at the packed M
# grid (1024..3072) and the NN backward of row-strided gathered weights (ZeRO-3 path)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_24}; mkdir -p $O
cp configs/tunableop/mi355x_gemms.csv $O/table.csv
LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=pipelined timeout -k 10 400 python bench.py --steps 3 --warmup 2 --tune_gemms $O/table.csv > $O/tune_pl.json 2> $O/tune_pl.err || exit $?
grep -c . $O/table.csv
timeout -k 10 600 python -u scripts/tools/tune_varlen_gemms.py --m-min 1024 --m-max 3072 --base $O/table.csv --out $O/table.csv > $O/tune_varlen.log 2>&1 || exit $?
tail -2 $O/tune_varlen.log
export LUMEN_GEMM_TABLE=$O/table.csv
for v in 0 1; do
  LUMEN_LORA_FOLD=$v LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=pipelined timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/pl_$v.json 2> $O/pl_$v.err || exit $?
  python -c "import json;d=json.load(open('$O/pl_$v.json'));print('pipelined fold=$v', d['ms_per_step'])"
done
