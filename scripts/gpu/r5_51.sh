#!/bin/bash
# production-shape numerics (2-layer Llama-2-7B training vs fp32, 256-row decode) on the final dxa3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_51; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_production_shapes_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
