#!/bin/bash
# MLP tail overlap: tune the down-projection dX split (11008 = 8192 + 2816 at T = 4096), GPU tests
# of the column-range SwiGLU and the overlapped MLP, then bench.py training A/B on one box
# (LUMEN_MLP_OVERLAP 0 / 1 / 2), the tuned table in place
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_40; mkdir -p $O
timeout -k 10 300 python -u scripts/probes/tune_serve_splits.py --out $O/gemms.csv --ms 4096 --only down_dx,gate_up > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
cat $O/tune.txt | grep '^{'
cp $O/gemms.csv configs/tunableop/mi355x_gemms.csv
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "swiglu or overlap_mlp" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for m in 0 1 2 0 1 2; do
  LUMEN_MLP_OVERLAP=$m timeout -k 10 300 python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 20 --warmup 5 > $O/bench_$m.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$m.json')); print('overlap $m', d['value'], d['ms_per_step'])"
done
