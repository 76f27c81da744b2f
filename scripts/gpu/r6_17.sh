#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6_17; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sampling or sample" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
sed -e "s#gpurun_out/r6_16#gpurun_out/r6_17#" scripts/gpu/r6_16.sh > /tmp/r6_17_prof.sh
bash /tmp/r6_17_prof.sh
