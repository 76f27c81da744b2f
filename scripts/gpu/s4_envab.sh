#!/bin/bash
# Same-box A/B of bench.py under env variants: s4_envab.sh OUT "NAME=ENV ..." ...
# each variant string is "label|VAR=val VAR2=val" (empty env = default)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s4_envab}; shift; mkdir -p $O
for i in 1 2; do
  for v in "$@"; do
    label=${v%%|*}; envs=${v#*|}
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/${label}_$i.log 2>&1 || exit 1
    echo "$label run$i $(tail -1 $O/${label}_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
