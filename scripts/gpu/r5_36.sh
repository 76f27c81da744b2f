#!/bin/bash
# custom all-reduce: collective calibration-timeout handling; RCCL / TP tests
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_36; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_rccl_gpu.py -k "calibration" > $O/tests.txt 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.txt | tail -15
exit $rc
