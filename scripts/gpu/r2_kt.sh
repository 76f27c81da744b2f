#!/bin/bash
# per-kernel time of the 1-GPU training step (rocprofv3 kernel trace), top kernels per step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r2_kt}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o step --output-format csv -- python3 bench.py --steps 6 --warmup 2 > $O/prof_bench.json 2> $O/prof.log || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" > $O/kernels.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
    print(f'{float(r["TotalDurationNs"]) / 8e6:8.3f} ms/step {r["Calls"]:>5} {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:90]}')
PY
grep -E "lv3|fa::|swiglu|rmsnorm|rope" $O/kernels.txt
