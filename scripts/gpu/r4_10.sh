#!/bin/bash
# Round 4: fp32 kernel paths (RMSNorm / SwiGLU / CE / RoPE / whole toy models vs the CPU), then
# the serving scheduling-policy comparison (r4_7)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_10}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_rccl_gpu.py -v --timeout 200 --timeout-method thread -k "rmsnorm_fwd_bwd or swiglu or cross_entropy or rope or fp32" > $O/fp32_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/fp32_tests.txt | tail -20; tail -1 $O/fp32_tests.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu/r4_7.sh r4_10/serve
