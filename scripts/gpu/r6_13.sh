#!/bin/bash
# final tree: rocprofv3 kernel trace of the default training step -> step table; decode step table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_13; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o kt -- \
  python3 bench.py --steps 4 --warmup 2 --partitioned "" --no_serve --no_box > $O/bench_prof.json 2> $O/bench_prof.err \
  || { tail -20 $O/bench_prof.err; exit 1; }
python3 scripts/tools/step_table.py $O/prof > $O/step_table.txt 2>&1 || true
head -30 $O/step_table.txt
ls $O/prof
