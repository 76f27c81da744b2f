#!/bin/bash
# mixed (chunked-prefill) step probe: wall per step, then a rocprof kernel table of the timed steps
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_20; mkdir -p $O
timeout -k 10 300 python -u scripts/probes/mixed_step_probe.py > $O/mixed.txt 2> $O/mixed.err || { tail -20 $O/mixed.err; exit 1; }
grep ms_per $O/mixed.txt
timeout -k 10 300 python -u scripts/probes/mixed_step_probe.py --decode 0 > $O/prefill_only.txt 2>> $O/mixed.err || { tail -20 $O/mixed.err; exit 1; }
grep ms_per $O/prefill_only.txt
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o mixed -- python3 scripts/probes/mixed_step_probe.py > $O/prof_run.txt 2> $O/prof_run.err || { tail -20 $O/prof_run.err; exit 1; }
python3 scripts/tools/gap_table.py $O/prof 24 > $O/mixed_table.txt
head -30 $O/mixed_table.txt
