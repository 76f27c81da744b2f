#!/bin/bash
# final tree: full GPU suite, bench, rocprofv3 kernel table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3_8}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o step --output-format csv -- python3 bench.py --steps 6 --warmup 2 > $O/prof_bench.json 2> $O/prof.log || exit $?
python scripts/tools/step_table.py $O/prof > $O/step_table.txt && head -24 $O/step_table.txt
