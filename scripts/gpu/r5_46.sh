#!/bin/bash
# RoPE in place, 8 heads per thread: numerics, then the training step A/B (LUMEN_ROPE_HPT 8 / 1)
# with a kernel trace of each
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_46; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "rope" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for h in 8 1; do
  LUMEN_ROPE_HPT=$h timeout -k 10 300 rocprofv3 --kernel-trace -d $O/k$h -o k$h -- python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 3 --warmup 2 > $O/kb_$h.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 scripts/tools/rocpd_summary.py $O/k$h rope
done
for h in 8 1 8 1; do
  LUMEN_ROPE_HPT=$h timeout -k 10 300 python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 20 --warmup 5 > $O/bench_$h.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$h.json')); print('hpt $h', d['value'], d['ms_per_step'])"
done
