#!/bin/bash
# fused-delta dQ kernel: FA numerics tests, then same-box bench A/B (LUMEN_FA_DQ_DELTA=0/1)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/s4_dqdelta2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu/s4_envab.sh s4_dqdelta2/ab "sep|LUMEN_FA_DQ_DELTA=0" "fused|LUMEN_FA_DQ_DELTA=1" || exit 1
bash scripts/gpu/s4_prof.sh ${1:-s4_prof2}
