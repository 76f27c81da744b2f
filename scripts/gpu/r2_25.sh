#!/bin/bash
# fused dA + dx (lora3_dxa): numerics, per-kernel timing, same-box bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_25}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_zero3_gpu.py -k "lora or fold or llama or gathered" -v --timeout 120 --timeout-method thread > $O/t.txt 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t.txt | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/probes/lora_kernels.py > $O/kern.json 2> $O/kern.err || exit $?
cat $O/kern.json
for v in 0 1 0 1; do
  LUMEN_LORA_DXA=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$v.json 2> $O/bench_$v.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('dxa=$v', d['ms_per_step'], d['value'])"
done
