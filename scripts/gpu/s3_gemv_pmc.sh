#!/bin/bash
# HBM bytes + time per batch-1 GEMV dispatch (counters in their own run, kernel trace only)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-s3_gemv_pmc}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc -o run -- python3 scripts/probes/gemv_pmc.py > $O/pmc.log 2>&1 || exit 1
find $O/pmc -name "*.csv" | head
