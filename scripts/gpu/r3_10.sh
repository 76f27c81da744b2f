#!/bin/bash
# partial-sum dY pass: LoRA tests first, full GPU suite, then same-box bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3_10}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "lora_linear_fwd_bwd or fold or delta" -q --timeout 120 --timeout-method thread > $O/new_tests.txt 2>&1 || { grep -E "FAILED|Error" $O/new_tests.txt | head -20; tail -3 $O/new_tests.txt; exit 1; }
tail -1 $O/new_tests.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt
[ $rc -le 1 ] || exit $rc
bash scripts/gpu/r3_ab.sh LUMEN_LORA_DY_PARTIAL ${1:-r3_10}/ab || exit $?
