#!/bin/bash
# 256-query-tile flash-attention forward: numerics (vs fp32 and the 128-row kernel), kernel time
# at the training shape, then the training step A/B (LUMEN_FA_FWD256 0 / 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_42; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fwd256" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for f in 0 1; do
  LUMEN_FA_FWD256=$f timeout -k 10 120 rocprofv3 --kernel-trace -d $O/k$f -o k$f -- \
    python3 lumen/bench/attn_bench.py --only fwd --iters 30 > $O/k$f.json 2> $O/k$f.err || exit 1
  python3 scripts/tools/rocpd_summary.py $O/k$f fwd
done
for f in 0 1 0 1; do
  LUMEN_FA_FWD256=$f timeout -k 10 300 python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 20 --warmup 5 > $O/bench_$f.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$f.json')); print('fwd256 $f', d['value'], d['ms_per_step'])"
done
