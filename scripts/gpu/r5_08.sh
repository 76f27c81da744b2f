#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_08
timeout -k 10 1000 python -u -m pytest -v -s --timeout 400 --timeout-method thread \
  tests/test_production_shapes_gpu.py \
  "tests/test_rccl_gpu.py::test_zero3_rccl_world8_llama70b_layers" \
  "tests/test_rccl_gpu.py::test_fp32_model_trains_on_gpu" \
  "tests/test_kernels_gpu.py::test_fp32_model_matches_cpu" \
  > gpurun_out/r5_08/tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|Error|oracle|decode logits" gpurun_out/r5_08/tests.txt | tail -40
exit $rc
