#!/bin/bash
# TunableOp candidate ranking for the training GEMM shapes (verbose tuning log)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3_9}; mkdir -p $O
PYTORCH_TUNABLEOP_VERBOSE=3 timeout -k 10 600 python -u -m lumen.bench.gemm_candidates $O/cands.json > $O/out.txt 2>&1; rc=$?
tail -12 $O/out.txt; exit $rc
