#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_serving_gpu.py tests/test_kernels_gpu.py -q -m gpu -x > gpurun_out/r24_tests.log 2>&1 || { tail -40 gpurun_out/r24_tests.log; exit 1; }
tail -2 gpurun_out/r24_tests.log
