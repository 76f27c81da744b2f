#!/bin/bash
# kernel table of one forced-partition (pipelined) ZeRO-3 step: where the gather overhead goes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3_z3prof}; mkdir -p $O
LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=pipelined timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof -o step --output-format csv -- python3 bench.py --steps 4 --warmup 2 > $O/bench.json 2> $O/prof.log || exit $?
python scripts/tools/step_table.py $O/prof > $O/step_table.txt && head -30 $O/step_table.txt
ls $O/prof/*/ 2>/dev/null | head; find $O/prof -name "*memory_copy*" | head -3
