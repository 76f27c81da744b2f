#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2_41; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "lora or fold" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
PROBES="0 32" bash scripts/gpu/r2_atomprobe.sh r2_41/p
