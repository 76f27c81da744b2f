#!/bin/bash
# fold / fused-tail GPU tests + same-box A/B of the fused fold tail (no fences)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3_3}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -k "fold" -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
bash scripts/gpu/r3_ab.sh LUMEN_LORA_FUSED_TAIL ${1:-r3_3}/tail || exit $?
