#!/bin/bash
# Round 4 profiles: one traced training step (rocprofv3 kernel trace -> step table) and the
# serving burst (kernel trace: decode-step composition with the decode-batch GEMM plans)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_4}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o run -- python3 bench.py --no_serve --partitioned "" --steps 6 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 scripts/tools/step_table.py $O/step > $O/step_table.txt 2>&1 || true
head -30 $O/step_table.txt
