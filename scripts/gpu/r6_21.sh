#!/bin/bash
# round-6 final tree: 256-row decode step (bf16, fp8) and its kernel table; batch-1 decode step
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_21; mkdir -p $O
timeout -k 10 300 python -u scripts/probes/decode_step_probe.py > $O/d256.txt 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
timeout -k 10 300 python -u scripts/probes/decode_step_probe.py --kv fp8 > $O/d256_fp8.txt 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
timeout -k 10 300 python -u scripts/probes/decode_step_probe.py --rows 1 --steps 64 > $O/d1.txt 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
grep -h ms_per $O/d256.txt $O/d256_fp8.txt $O/d1.txt
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o dec -- python3 scripts/probes/decode_step_probe.py > $O/prof_run.txt 2> $O/prof_err.txt || { tail -20 $O/prof_err.txt; exit 1; }
python3 scripts/tools/decode_table.py $O/prof > $O/decode_table.txt
head -12 $O/decode_table.txt
