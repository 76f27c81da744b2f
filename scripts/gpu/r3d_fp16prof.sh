#!/bin/bash
# fp16 (reference precision) vs bf16 steady-state step tables, same box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_fp16prof}; mkdir -p $O
for dt in fp16 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step_$dt -o run -- python3 bench.py --no_serve --dtype $dt --steps 4 --warmup 3 > $O/traced_$dt.json 2> $O/traced_$dt.err || { tail -5 $O/traced_$dt.err; exit 1; }
  python3 scripts/tools/step_table.py $O/step_$dt > $O/step_table_$dt.txt && head -30 $O/step_table_$dt.txt
done
