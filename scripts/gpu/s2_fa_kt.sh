#!/bin/bash
# per-kernel times of the flash-attention backward variants
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/s2_fa_kt; mkdir -p $O
for v in "t1 v16" "v32 v32"; do set -- $v
  for S in 512 4096; do B=$((4096 / S * 2)); [ $S = 512 ] && B=8
    LUMEN_FA_FWD=$1 LUMEN_FA_BWD=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$2_$S -o run -- python3 lumen/bench/attn_bench.py --only bwd --B $B --S $S --iters 5 > $O/$2_$S.log 2>&1 || exit 1
  done
done
