#!/bin/bash
# paged decode: every (D, G) of the uniform / pipelined variants + the existing decode tests
set -o pipefail
mkdir -p gpurun_out/r6_05
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "paged_decode" > gpurun_out/r6_05/pytest.log 2>&1
