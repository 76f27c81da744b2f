#!/bin/bash
# current training step kernel stats (N=1 bench defaults, 2 warmup + 5 timed steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-s3_trainprof}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/plain -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 > $O/plain.log 2>&1
rc=$?; echo "plain rc=$rc"; tail -1 $O/plain.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
O=$O python3 - <<'PY'
import csv, glob
import os; f = glob.glob(os.environ["O"] + "/plain/**/run_kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:30]:
    print(r["Name"][:80], r["Calls"], round(float(r["TotalDurationNs"]) / 7e6, 2), "ms/step", r["AverageNs"][:8])
PY
