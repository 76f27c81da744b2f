#!/bin/bash
# where the ZeRO-3 partitioned-path overhead goes: kernel stats of the forced-partition pipelined
# schedule (the N>1 code path at world 1) vs the identity schedule
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_18}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_id -o b --output-format csv -- python3 bench.py --steps 6 --warmup 2 > $O/id.json 2> $O/id.log || exit $?
LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=pipelined timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_pl -o b --output-format csv -- python3 bench.py --steps 6 --warmup 2 > $O/pl.json 2> $O/pl.log || exit $?
for k in id pl; do python -c "import json;d=json.load(open('$O/$k.json'));print('$k', d['ms_per_step'], d['config']['parallelism'])"; done
for k in id pl; do
f=$(find $O/prof_$k -name "*kernel_stats.csv" | head -1)
python - "$f" $k <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(sys.argv[2], "total kernel ms", round(tot / 1e6, 1))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print("  ", round(float(r["TotalDurationNs"]) / 1e6, 1), r["Calls"], r["Name"][:100])
PY
done
