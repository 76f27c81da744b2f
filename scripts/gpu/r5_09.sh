#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_09
timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread \
  "tests/test_production_shapes_gpu.py::test_llama2_7b_shaped_decode_step_matches_fp32" \
  > gpurun_out/r5_09/tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|Error|oracle|decode logits" gpurun_out/r5_09/tests.txt | tail -20
exit $rc
