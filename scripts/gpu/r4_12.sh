#!/bin/bash
# Round 4: smoke() + the driver's default bench (headline + partitioned + serving sections)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_12}; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - <<EOF2
import json
d = json.load(open("$O/bench.json"))
e = d["extra"]
print("train", d["value"], d["ms_per_step"], d["config"]["parallelism"], d["vs_baseline"])
for k in ("zero3_release", "zero3_hybrid", "serve", "serve_engine", "serve_chunked"):
    print(k, json.dumps(e.get(k)))
EOF2
