#!/bin/bash
# full GPU suite on the current tree, the 1-GPU bench, and a rocprofv3 kernel table of the step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_58}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o step --output-format csv -- python3 bench.py --steps 6 --warmup 2 > $O/prof_bench.json 2> $O/prof.log || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms (8 steps incl. init)", round(tot / 1e6, 1))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:24]:
    print("  ", round(float(r["TotalDurationNs"]) / 8e6, 3), "ms/step", r["Calls"], r["Name"][:90])
PY
