#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s2_serve3; mkdir -p $O
for n in 1 16 64; do
  timeout -k 10 300 python lumen/bench/serve_bench.py --num-requests $n --max-num-seqs 256 > $O/serve_$n.log 2>&1 || exit 1
  tail -1 $O/serve_$n.log | cut -c1-260
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o run -- python3 lumen/bench/serve_bench.py --num-requests 1 > $O/prof1.log 2>&1
