#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r29
timeout -k 10 400 python -m pytest tests/test_custom_ar_gpu.py -x -q > gpurun_out/r29/car.log 2>&1
rc=$?
grep -v "Gloo\|hostname\|amdgpu.ids" gpurun_out/r29/car.log | tail -40
exit $rc
