#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2_55; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "flash or llama" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for ps in 1 9 1 9; do
  LUMEN_FA_PERSIST=$ps timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$ps -o run -- python3 lumen/bench/attn_bench.py --B 8 --S 512 --iters 20 > $O/k$ps.log 2>&1 || exit 1; python3 -c "import csv,glob;[print(round(float(r[\"AverageNs\"])/1e3,1), r[\"Name\"][:60]) for r in csv.DictReader(open(glob.glob(\"$O/k$ps/*kernel_stats.csv\")[0])) if \"lumen::fa\" in r[\"Name\"]]" > $O/p$ps.txt
  echo "persist $ps: $(cat $O/p$ps.txt)"
  rm -rf $O/k$ps
done
