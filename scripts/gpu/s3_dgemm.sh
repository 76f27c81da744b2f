#!/bin/bash
# decode-batch MFMA GEMM: numerics then the per-M sweep against hipBLASLt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s3_dgemm}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "dgemm" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u lumen/bench/skinny_bench.py --dgemm > $O/dgemm.jsonl 2>&1 || exit 1
cat $O/dgemm.jsonl
