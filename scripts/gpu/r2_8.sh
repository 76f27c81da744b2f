#!/bin/bash
# down3 cost probes: 1 = no dropout hash, 2 = no A loads, 4 = no reduction/atomics
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_8}; mkdir -p $O
for pr in 0 8 4 7; do
  LUMEN_LV3_PROBE=$pr timeout -k 10 120 python scripts/probes/lora_kernels.py > $O/kern_$pr.json 2>> $O/kern.err || exit $?
  python -c "import json;d=json.load(open('$O/kern_$pr.json'));print($pr, d['qkv_down'], d['o_down'])"
done
