#!/bin/bash
# batch-1 decode: step time and kernel table
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_26; mkdir -p $O
timeout -k 10 300 python -u scripts/probes/decode_step_probe.py --rows 1 --steps 64 > $O/b1.txt 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
grep ms_per $O/b1.txt
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o b1 -- python3 scripts/probes/decode_step_probe.py --rows 1 --steps 64 > $O/prof_run.txt 2> $O/prof_err.txt || { tail -20 $O/prof_err.txt; exit 1; }
python3 scripts/tools/gap_table.py $O/prof 64 > $O/b1_table.txt
head -25 $O/b1_table.txt
