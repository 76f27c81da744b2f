#!/bin/bash
# Round 4: device LR schedules vs host (rebuilt extension), fp16 / kernel sanity, then a short
# bench (the AdamW kernel changed: the step must not move)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_30}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_lr_sched_gpu.py tests/test_fp16_gpu.py tests/test_serving_gpu.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -n 2 $O/tests.txt
timeout -k 10 300 python bench.py --no_serve --partitioned "" --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'])"
