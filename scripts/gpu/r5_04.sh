#!/bin/bash
# decode GEMM variants at M = 256 + their numerics test
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_04
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  "tests/test_kernels_gpu.py::test_decode_gemm_variants" > gpurun_out/r5_04/test.txt 2>&1 || { tail -30 gpurun_out/r5_04/test.txt; exit 1; }
timeout -k 10 600 python -u scripts/probes/dgemm_variants.py > gpurun_out/r5_04/variants.jsonl 2>&1
rc=$?
cat gpurun_out/r5_04/variants.jsonl
exit $rc
