#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s2_sk4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "skinny" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python lumen/bench/skinny_bench.py > $O/bench.jsonl 2>$O/bench.err; rc=$?
cat $O/bench.jsonl; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu/s2_serve4.sh s2_sk4_serve
