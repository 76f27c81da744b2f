#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2_45; mkdir -p $O
PROBES="0 6 22 23 54 16 32" bash scripts/gpu/r2_faprobe.sh r2_45/p || exit 1
for h in 0 1 0 1; do
  LUMEN_FA_DKDV_HEAVY=$h timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/h$h -o run -- python3 lumen/bench/attn_bench.py --only bwd --B 8 --S 512 --iters 20 > $O/h$h.log 2>&1 || exit 1
  f=$(find $O/h$h -name "*kernel_stats.csv" | head -1)
  python3 - "$f" $h <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "dkdv" in r["Name"]:
        print(f'heavy {sys.argv[2]}: {float(r["AverageNs"])/1e3:8.1f} us')
PY
  rm -rf $O/h$h
done
