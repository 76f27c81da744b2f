#!/bin/bash
# split deterministic sums for down3 / dy3 / dxa3: tests, then the step-time A/B
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r6_25; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_deterministic_gpu.py tests/test_fp16_gpu.py tests/test_kernels_gpu.py -k "deterministic or fp16 or lora" > $O/tests.txt 2>&1 \
  || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
sed -e "s#gpurun_out/r6_24#gpurun_out/r6_25#" scripts/gpu/r6_24.sh > /tmp/ab.sh && bash /tmp/ab.sh
