#!/bin/bash
# kernel stats: plain N=1 vs forced ZeRO-3 pipelined (local gathers + off-path transposes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/s2_prof1; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/plain -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 > $O/plain.log 2>&1
rc=$?; echo "plain rc=$rc"; tail -1 $O/plain.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=pipelined timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pipe -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 > $O/pipe.log 2>&1
rc=$?; echo "pipe rc=$rc"; tail -1 $O/pipe.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
find $O -name "*kernel_stats.csv" -o -name "*kernel_trace.csv" | head
