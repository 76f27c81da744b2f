#!/bin/bash
# grad-norm with at most 512 workgroups: numerics + kernel time, then the training bench twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_60; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_gpu.py tests/test_lr_sched_gpu.py -k "norm or adamw or fp16 or sched" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/k -o k -- python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 3 --warmup 2 > $O/kb.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 scripts/tools/rocpd_summary.py $O/k norm_sq
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 20 --warmup 5 > $O/bench_$i.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$i.json')); print('bench', d['value'], d['ms_per_step'])"
done
