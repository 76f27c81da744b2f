#!/bin/bash
# 32x32x16 flash-attention kernels: numerics, then timings vs the 16x16x32 kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/s2_fa1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k flash_attention -x -v --timeout 120 --timeout-method thread > $O/fa_tests.log 2>&1
rc=$?; echo "fa tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" $O/fa_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
for v in "t1 v16" "v32 v32"; do set -- $v
  LUMEN_FA_FWD=$1 LUMEN_FA_BWD=$2 timeout -k 10 120 python lumen/bench/attn_bench.py --only all >> $O/bench.jsonl 2>$O/bench.err || exit 1
  LUMEN_FA_FWD=$1 LUMEN_FA_BWD=$2 timeout -k 10 120 python lumen/bench/attn_bench.py --only all --B 2 --S 4096 >> $O/bench.jsonl 2>>$O/bench.err || exit 1
done
cat $O/bench.jsonl
