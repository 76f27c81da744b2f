#!/bin/bash
# LoRA v3 (DOWN + fused dY + dx, v2 UP): tests, per-kernel probe, layer probe, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_9}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lora" -v --timeout 120 --timeout-method thread > $O/lora_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/lora_tests.txt | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/probes/lora_kernels.py > $O/kern.json 2> $O/kern.err || exit $?
cat $O/kern.json
for v in 0 1; do
  LUMEN_LORA_V3=$v timeout -k 10 120 python scripts/probes/lora_train_shapes.py >> $O/probe.jsonl 2>> $O/probe.err || exit $?
done
cat $O/probe.jsonl
for v in 0 1 0 1; do
  LUMEN_LORA_V3=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_v3_$v.json 2> $O/bench_v3_$v.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_v3_$v.json'));print('v3=$v', d['ms_per_step'], d['value'])"
done
