#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/s2_r4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_zero3_gpu.py -x -v --timeout 300 --timeout-method thread > $O/zero3_tests.log 2>&1
rc=$?; echo "zero3 gpu tests rc=$rc"; grep -E "PASS|FAIL|Error" $O/zero3_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
LUMEN_ZERO3_SINGLE=1 timeout -k 10 300 python bench.py --steps 8 --warmup 3 > $O/bench_auto.log 2>&1
rc=$?; echo "bench auto rc=$rc"; tail -1 $O/bench_auto.log | cut -c700-1200; exit $rc
