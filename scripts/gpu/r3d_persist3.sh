#!/bin/bash
# dQ-from-dS persistent launch (LUMEN_FA_PERSIST bit 2) on top of the new default (11)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_persist3}; mkdir -p $O
for p in 15 11 15 11; do
  LUMEN_FA_PERSIST=$p timeout -k 10 120 python3 scripts/probes/fa_fwd_probe.py --bwd --shapes 8x512c,2x2048c > $O/p$p.jsonl 2>&1 || { tail -5 $O/p$p.jsonl; exit 1; }
  sed "s/^/persist=$p /" $O/p$p.jsonl | grep shape
done
