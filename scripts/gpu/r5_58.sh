#!/bin/bash
# fp16 overflow-skip test under the LM-head TN path on / off (tolerance test on order-
# nondeterministic atomics: which of the round's changes moves it)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_58; mkdir -p $O
for w in 1 0 1 0; do
  LUMEN_LMHEAD_WT=$w timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_fp16_gpu.py -k "overflow" > $O/t_$w.txt 2>&1
  echo "wt=$w rc=$? $(grep -o 'AssertionError: (.*' $O/t_$w.txt | head -1 | cut -c1-150)"
done
exit 0
