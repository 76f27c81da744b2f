#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s2_fa8}; mkdir -p $O; rm -f $O/bench.jsonl
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "flash_attention" -x -q --timeout 120 --timeout-method thread > $O/fa_tests.log 2>&1
rc=$?; echo "fa tests rc=$rc"; tail -2 $O/fa_tests.log; [ $rc -eq 0 ] || exit $rc
for v in "v32 mix" "v32p mix"; do set -- $v
  LUMEN_FA_FWD=$1 LUMEN_FA_BWD=$2 timeout -k 10 120 python lumen/bench/attn_bench.py --only fwd >> $O/bench.jsonl 2>$O/bench.err || exit 1
  LUMEN_FA_FWD=$1 LUMEN_FA_BWD=$2 timeout -k 10 120 python lumen/bench/attn_bench.py --only fwd --B 2 --S 4096 >> $O/bench.jsonl 2>>$O/bench.err || exit 1
done
cut -c1-40,95-250 $O/bench.jsonl
