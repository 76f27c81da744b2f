#!/bin/bash
# round 5: production-shape fp32-oracle tests + the tests touched by the ADVICE fixes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_01
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_production_shapes_gpu.py \
  "tests/test_kernels_gpu.py::test_decode_gemm_variants" \
  "tests/test_kernels_gpu.py::test_llama_lora_fold_matches_unfolded" \
  > gpurun_out/r5_01/tests.txt 2>&1
rc=$?
tail -25 gpurun_out/r5_01/tests.txt
exit $rc
