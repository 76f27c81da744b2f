#!/bin/bash
# head-dim-64 flash attention (zero-padded), OPT on the GPU path, packing GPU test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_16}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_packing_gpu.py -k "small_head_dim or opt_gpu or packed" -v --timeout 120 --timeout-method thread > $O/t.txt 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/t.txt | tail -12; exit $rc
