#!/bin/bash
# serving prefill / mixed-step projections: tune whole-wave split parts, time split vs single
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_21; mkdir -p $O
timeout -k 10 900 python -u scripts/probes/tune_serve_splits.py --out $O/gemms.csv > $O/tune.jsonl 2> $O/tune.err || { tail -20 $O/tune.err; exit 1; }
cat $O/tune.jsonl
