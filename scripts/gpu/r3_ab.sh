#!/bin/bash
# same-box A/B of one env switch on bench.py: off, on, off, on (20 steps each)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
VAR=$1; O=$GRAFT_REPO_ROOT/gpurun_out/${2:-r3_ab}; mkdir -p $O
for i in 1 2; do
  for v in ${VALS:-0 1}; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/bench_${v}_$i.json'));print('$VAR=$v run $i', d['ms_per_step'])"
  done
done
