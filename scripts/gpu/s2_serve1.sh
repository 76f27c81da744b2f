#!/bin/bash
# serving: engine bench + kernel trace of the same run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/s2_serve1; mkdir -p $O
timeout -k 10 300 python lumen/bench/serve_bench.py > $O/engine.log 2>&1
rc=$?; echo "engine rc=$rc"; tail -1 $O/engine.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 lumen/bench/serve_bench.py > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
