#!/bin/bash
# Round 4: diagnostics for the world-8 failures -- fp32 tiny-llama-deep NaN (module by module vs
# the CPU), the custom all-reduce at 2 / 4 / 8 ranks (bit-exact), TP=8 tokens per carrier
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_8}; mkdir -p $O
timeout -k 10 180 python scripts/probes/fp32_probe.py > $O/fp32_probe.txt 2>&1; rc=$?
cat $O/fp32_probe.txt | grep -v Warning | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_custom_ar_gpu.py -v --timeout 150 --timeout-method thread > $O/car_tests.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|assert" $O/car_tests.txt | tail -30; tail -1 $O/car_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python scripts/probes/tp_diag.py > $O/tp_diag.txt 2>&1; rc=$?
grep -vE "Warning|warn" $O/tp_diag.txt | tail -30; exit $rc
