#!/bin/bash
# batch-1 decode: SwiGLU fused into the down-projection GEMV (LUMEN_SWIGLU_GEMV) numerics + A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_35; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "skinny or gemv" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for v in 1 0 1 0; do
  LUMEN_SWIGLU_GEMV=$v timeout -k 10 300 python -u scripts/probes/decode_step_probe.py --rows 1 --steps 96 >> $O/b1_$v.txt 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
done
for v in 1 0; do echo "fused=$v $(grep ms_per $O/b1_$v.txt | tr '\n' ' ')"; done
