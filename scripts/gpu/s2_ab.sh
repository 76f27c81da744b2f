#!/bin/bash
# A/B on the same box: ab_old/ (older tree, own in-tree build) vs the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s2_ab}; mkdir -p $O
for i in 1 2; do
  (cd ab_old && timeout -k 10 300 python bench.py --steps 10 --warmup 3 > ../$O/old_$i.log 2>&1) || exit 1
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/new_$i.log 2>&1 || exit 1
  echo "old $(tail -1 $O/old_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')  new $(tail -1 $O/new_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
