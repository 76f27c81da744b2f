#!/bin/bash
# Round 4: A/B of existing switches on the current tree (same box, back to back):
# RMSNorm backward waves per row, flash-attention persistence bits, LoRA dY tile height
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_21}; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no_serve --partitioned "" --steps 20 --warmup 5 > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'])"
}
run base LUMEN_NOOP=1 &&
run rms_wpr2 LUMEN_RMS_BWD_WPR=2 &&
run fa_persist7 LUMEN_FA_PERSIST=7 &&
run base2 LUMEN_NOOP=1
