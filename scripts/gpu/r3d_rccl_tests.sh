#!/bin/bash
# RCCL multi-rank GPU tests (two ranks sharing the box's GPU), then the whole GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_rccl_tests}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_rccl_gpu.py -x -v --timeout 180 --timeout-method thread > $O/rccl_tests.txt 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/rccl_tests.txt | tail -12; [ $rc -eq 0 ] || { tail -40 $O/rccl_tests.txt; exit $rc; }
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt; exit $rc
