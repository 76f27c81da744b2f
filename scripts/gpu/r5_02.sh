#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_02
timeout -k 10 300 python -u scripts/probes/oracle_diag.py > gpurun_out/r5_02/diag.txt 2>&1
P=0 timeout -k 10 300 python -u scripts/probes/oracle_diag.py > gpurun_out/r5_02/diag_p0.txt 2>&1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  "tests/test_production_shapes_gpu.py::test_llama2_7b_shaped_decode_step_matches_fp32" \
  "tests/test_kernels_gpu.py::test_decode_gemm_variants" \
  "tests/test_kernels_gpu.py::test_llama_lora_fold_matches_unfolded" \
  > gpurun_out/r5_02/tests.txt 2>&1
rc=$?
cat gpurun_out/r5_02/diag.txt gpurun_out/r5_02/diag_p0.txt; tail -25 gpurun_out/r5_02/tests.txt
exit $rc
