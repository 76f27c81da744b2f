#!/bin/bash
# LoRA fold on ZeRO-3-gathered weights (tail reserved in the partitioned layout, filled at bind):
# ZeRO-3 / fold GPU tests, then forced-partition pipelined bench A/B and the identity bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_23}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_zero3_gpu.py tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k "zero3 or fold or engine or fp16 or llama" -v --timeout 200 --timeout-method thread > $O/t.txt 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t.txt | tail -8; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  LUMEN_LORA_FOLD=$v LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=pipelined timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/pl_$v.json 2> $O/pl_$v.err || exit $?
  python -c "import json;d=json.load(open('$O/pl_$v.json'));print('pipelined fold=$v', d['ms_per_step'], d['extra']['peak_hbm_gb_max_rank'])"
done
LUMEN_ZERO3_SINGLE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config configs/ds_config_zero3_release.json > $O/rel_1.json 2> $O/rel_1.err || exit $?
python -c "import json;d=json.load(open('$O/rel_1.json'));print('release fold=1', d['ms_per_step'], d['extra']['peak_hbm_gb_max_rank'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/id.json 2> $O/id.err || exit $?
python -c "import json;d=json.load(open('$O/id.json'));print('identity', d['ms_per_step'], d['value'], d['extra']['peak_hbm_gb_max_rank'])"
