#!/bin/bash
# LoRA side-stream overlap (DOWN under the base GEMM, dY pass under the dX GEMM): numerics with
# overlap on, then same-box bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_17}; mkdir -p $O
LUMEN_LORA_OVERLAP=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_packing_gpu.py -k "lora or packed or llama" -v --timeout 120 --timeout-method thread > $O/t.txt 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t.txt | tail -5; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  LUMEN_LORA_OVERLAP=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$v.json 2> $O/bench_$v.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('overlap=$v', d['ms_per_step'], d['value'])"
done
