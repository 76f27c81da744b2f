#!/bin/bash
# Round 4: the driver's round-end GPU tiers -- full `pytest -m gpu`, smoke(), bench.py
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_11}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | tail -20; tail -1 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
