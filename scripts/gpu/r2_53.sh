#!/bin/bash
# same-box A/B of the training step: persistent dK/dV on/off
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2_53; mkdir -p $O
for ps in 1 0 1 0; do
  LUMEN_FA_PERSIST=$ps timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b$ps.json 2> $O/b$ps.err || exit 1
  python3 -c "import json;d=json.load(open('$O/b$ps.json'));print('persist $ps', d['ms_per_step'], d['value'])"
done
