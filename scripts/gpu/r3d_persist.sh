#!/bin/bash
# flash-attention forward persistent launch (LUMEN_FA_PERSIST bit 1) with the Q-by-DMA prologue
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_persist}; mkdir -p $O
for p in 11 9 11 9; do
  LUMEN_FA_PERSIST=$p timeout -k 10 120 python3 scripts/probes/fa_fwd_probe.py --shapes 8x512c,2x2048c > $O/p$p.jsonl 2>&1 || { tail -5 $O/p$p.jsonl; exit 1; }
  sed "s/^/persist=$p /" $O/p$p.jsonl | grep shape
done
