#!/bin/bash
# LM-head dH scale as one vectorized device-scalar pass: numerics, kernel trace, step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_54; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k "lm_head or scale_dev or fp16 or engine" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/k -o k -- python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 3 --warmup 2 > $O/kb.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 scripts/tools/rocpd_summary.py $O/k scale_dev
python3 scripts/tools/rocpd_summary.py $O/k elementwise_kernel_manual
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 20 --warmup 5 > $O/bench_$i.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$i.json')); print('bench', d['value'], d['ms_per_step'], d['extra']['final_loss'])"
done
