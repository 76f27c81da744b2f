#!/bin/bash
# LoRA per-kernel v2 vs v3 timing + rocprof kernel stats of the probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_7}; mkdir -p $O
timeout -k 10 120 python scripts/probes/lora_kernels.py > $O/kern.json 2> $O/kern.err || exit $?
cat $O/kern.json
TW=512 timeout -k 10 120 python scripts/probes/lora_kernels.py > $O/kern512.json 2>> $O/kern.err || exit $?
cat $O/kern512.json
