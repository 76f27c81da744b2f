#!/bin/bash
# LoRA adapter kernels A/B: ab_so/A.so vs ab_so/B.so: numerics on B, kernel trace of the
# training step for both (per-kernel times), full bench step B A B, fp16 step B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_lora_ab}; mkdir -p $O
SO=lumen/_C.cpython-310-x86_64-linux-gnu.so
cp ab_so/B.so $SO
timeout -k 10 400 python -u -m pytest tests -m gpu -q -k "lora or fp16 or packing or zero3 or delta" --timeout 180 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.txt | head; tail -1 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for v in B A; do
  cp ab_so/$v.so $SO
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step_$v -o run -- python3 bench.py --no_serve --steps 4 --warmup 3 > $O/traced_$v.json 2> $O/traced_$v.err || { tail -5 $O/traced_$v.err; exit 1; }
  python3 scripts/tools/step_table.py $O/step_$v > $O/step_table_$v.txt && grep -E "wall|lv3|lv2" $O/step_table_$v.txt | sed "s/^/$v /"
done
for v in B A B; do
  cp ab_so/$v.so $SO
  timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('bench $v', d['ms_per_step'], d['value'])"
done
cp ab_so/B.so $SO
