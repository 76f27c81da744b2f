#!/bin/bash
# dy3 with the Z operand loaded before the dY prefetch (counted waits, no drain): LoRA numerics,
# per-launch kernel times, training step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_52; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "lora or fold" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/k -o k -- python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 3 --warmup 2 > $O/kb.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 scripts/tools/rocpd_by_grid.py $O/k dy3
python3 scripts/tools/rocpd_by_grid.py $O/k dxa3
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 20 --warmup 5 > $O/bench_$i.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$i.json')); print('bench', d['value'], d['ms_per_step'])"
done
