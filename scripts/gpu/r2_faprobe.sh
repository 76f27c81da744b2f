#!/bin/bash
# FA dK/dV cost probes (LUMEN_FA_PROBE bits: 1 no DMA after step 1, 2 no S/dP, 4 no dV/dK, 8 no exp)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r2_faprobe}; mkdir -p $O
for pb in ${PROBES:-0 1 2 4 6 8}; do
  LUMEN_FA_PROBE=$pb timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$pb -o run -- python3 lumen/bench/attn_bench.py --only bwd --B 8 --S 512 --iters 20 > $O/p$pb.log 2>&1 || exit 1
  f=$(find $O/p$pb -name "*kernel_stats.csv" | head -1)
  python3 - "$f" $pb <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "dkdv" in r["Name"]:
        print(f'probe {sys.argv[2]}: {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:70]}')
PY
done
