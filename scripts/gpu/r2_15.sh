#!/bin/bash
# kernel-time breakdown of the 256 x (512 in / 128 out) serving run (engine mode, budget 2048)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_15}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o serve --output-format csv -- python3 -m lumen.bench.serve_bench --mode engine --max-batched-tokens 2048 > $O/serve.json 2> $O/prof.log || exit $?
cut -c1-400 $O/serve.json
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms", round(tot / 1e6, 1))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(round(float(r["TotalDurationNs"]) / 1e6, 1), r["Calls"], r["Name"][:110])
PY
