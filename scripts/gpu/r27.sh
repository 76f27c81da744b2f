#!/bin/bash
# custom all-reduce (2 processes on the one GPU) + serving GPU tests after the TP graph changes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r27
timeout -k 10 300 python -m pytest tests/test_custom_ar_gpu.py -x -q -s > gpurun_out/r27/car.log 2>&1 && \
timeout -k 10 400 python -m pytest tests/test_serving_gpu.py -x -q > gpurun_out/r27/serve.log 2>&1
rc=$?
tail -5 gpurun_out/r27/car.log
tail -3 gpurun_out/r27/serve.log 2>/dev/null
exit $rc
