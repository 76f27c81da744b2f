#!/bin/bash
# tune + time the down input-grad split (no rotating buffers), GPU CE / lm-head tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3_7}; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests -m gpu -k "xent or cross or lm_head or fp16 or loss" -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1; tail -1 $O/gpu_tests.txt
LUMEN_TUNE_ROTATING_MB=0 timeout -k 10 600 python -u -m lumen.bench.split_gemm_probe --tune $O/tuned.csv > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep -v split_kernels $O/probe.txt | grep -E "one|split" | head -12
