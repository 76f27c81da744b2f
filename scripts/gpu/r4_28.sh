#!/bin/bash
# Round 4: memory traffic of the training step's kernels (two rocprofv3 counter passes:
# FETCH_SIZE, WRITE_SIZE; kernel trace for durations) -> achieved GB/s per kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_28}; mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/$c -o run -- python3 bench.py --no_serve --partitioned "" --steps 3 --warmup 1 > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
done
python3 scripts/tools/pmc_bw.py $O/FETCH_SIZE $O/WRITE_SIZE > $O/bw_table.txt 2>&1
head -32 $O/bw_table.txt
