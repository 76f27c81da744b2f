#!/bin/bash
# kernel stats of the 256-request serving run (decode attention dominates the decode step)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s3_prof256}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 lumen/bench/serve_bench.py --num-requests 256 > $O/prof.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/s3_prof256/prof/**/run_kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/s3_prof256/prof/run_kernel_stats.csv")
for r in list(csv.DictReader(open(f[0])))[:14]:
    print(r["Name"][:90], r["Calls"], r["AverageNs"], r["Percentage"])
PY
