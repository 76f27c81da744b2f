#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2_50; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "flash or llama" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for ps in 1 0 1 0; do
  LUMEN_FA_PERSIST=$ps PROBES="0" bash scripts/gpu/r2_faprobe.sh r2_50/p$ps > $O/p$ps.txt || exit 1
  echo "persist $ps: $(cat $O/p$ps.txt)"
  rm -rf $O/p$ps
done
