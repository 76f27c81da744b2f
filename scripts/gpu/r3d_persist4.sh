#!/bin/bash
# training step: persistent dQ (15, default) vs one-shot dQ (11), interleaved on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_persist4}; mkdir -p $O
for p in 15 11 15 11 15 11; do
  LUMEN_FA_PERSIST=$p timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/bench_$p.json 2> $O/bench_$p.err || { tail -5 $O/bench_$p.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$p.json'));print('train persist=$p', d['ms_per_step'], d['value'])"
done
