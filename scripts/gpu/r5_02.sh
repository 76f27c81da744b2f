#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_02
timeout -k 10 300 python -u scripts/probes/oracle_diag.py > gpurun_out/r5_02/diag.txt 2>&1
P=0 timeout -k 10 300 python -u scripts/probes/oracle_diag.py > gpurun_out/r5_02/diag_p0.txt 2>&1
timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  "tests/test_production_shapes_gpu.py::test_llama2_7b_shaped_decode_step_matches_fp32" \
  "tests/test_kernels_gpu.py::test_decode_gemm_variants" \
  "tests/test_kernels_gpu.py::test_llama_lora_fold_matches_unfolded" \
  tests/test_custom_ar_gpu.py \
  "tests/test_rccl_gpu.py::test_custom_allreduce_late_peer" \
  "tests/test_rccl_gpu.py::test_tp_serving_rccl_matches_tp1" \
  "tests/test_rccl_gpu.py::test_zero3_rccl_world8_llama70b_layers" \
  > gpurun_out/r5_02/tests.txt 2>&1
rc=$?
cat gpurun_out/r5_02/diag.txt gpurun_out/r5_02/diag_p0.txt; grep -E "PASS|FAIL|Error|car diag|skew|\[\{" gpurun_out/r5_02/tests.txt | tail -40
exit $rc
