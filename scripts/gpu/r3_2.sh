#!/bin/bash
# GPU suite + same-box A/Bs: split gate|up GEMM, fused fold tail in the LoRA DOWN kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3_2}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt
[ $rc -le 1 ] || exit $rc
bash scripts/gpu/r3_ab.sh LUMEN_GEMM_SPLIT ${1:-r3_2}/split || exit $?
bash scripts/gpu/r3_ab.sh LUMEN_LORA_FUSED_TAIL ${1:-r3_2}/tail || exit $?
