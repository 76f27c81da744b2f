#!/bin/bash
# packed fp16 conversion: kernel numerics (fp16 + bf16), the dY-pass probe, fp16 / bf16 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_fp16fix}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/probes/dy3_dtype_probe.py > $O/dy3.jsonl 2>&1 || { tail -5 $O/dy3.jsonl; exit 1; }
grep -E "0.001, \"B_mag\": 0.01, \"Z_mag\": 1.0" $O/dy3.jsonl
for dt in fp16 bf16 fp16; do
  timeout -k 10 300 python bench.py --no_serve --dtype $dt --steps 20 --warmup 5 > $O/$dt.json 2> $O/$dt.err || { tail -5 $O/$dt.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$dt.json'));print('$dt', d['ms_per_step'], d['value'], d['extra']['timed_steps_skipped_nonfinite'])"
done
