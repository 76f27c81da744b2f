#!/bin/bash
# FA A/B on one box: ab_old/ (HEAD build) vs the working tree; FA GPU tests on the new tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s3_fa_ab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "flash" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for S in 512 4096; do
    B=$((4096 / S)); [ $S -eq 4096 ] && B=2
    (cd ab_old && timeout -k 10 120 python -m lumen.bench.attn_bench --B $B --S $S > ../$O/old_${S}_$i.log 2>&1) || exit 1
    timeout -k 10 120 python -m lumen.bench.attn_bench --B $B --S $S > $O/new_${S}_$i.log 2>&1 || exit 1
    echo "S=$S old: $(tail -1 $O/old_${S}_$i.log | cut -c1-200)"
    echo "S=$S new: $(tail -1 $O/new_${S}_$i.log | cut -c1-200)"
  done
done
