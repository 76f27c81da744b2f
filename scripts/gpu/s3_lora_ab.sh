#!/bin/bash
# LoRA training-shape probe + LoRA GPU tests: ab_old/ (HEAD build) vs the working tree, same box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s3_lora_ab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lora" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  (cd ab_old && timeout -k 10 120 python scripts/probes/lora_train_shapes.py 2>&1 | grep "^{" | sed "s/^/old /") || exit 1
  timeout -k 10 120 python scripts/probes/lora_train_shapes.py 2>&1 | grep "^{" | sed "s/^/new /" || exit 1
done
