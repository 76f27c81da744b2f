#!/bin/bash
# LM-head dX: NN vs TN (cached W^T), heuristic vs tuned
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_55; mkdir -p $O
timeout -k 10 400 python -u scripts/probes/lm_head_dx_probe.py --out $O/gemms.csv > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep '^{' $O/probe.txt
grep "32000_ld" $O/gemms.csv | grep "tn_4096_4096_32000" || true
