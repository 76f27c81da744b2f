#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s2_serve2; mkdir -p $O
for mbt in 4096 8192; do
  timeout -k 10 300 python lumen/bench/serve_bench.py --max-batched-tokens $mbt > $O/serve_$mbt.log 2>&1 || exit 1
  tail -1 $O/serve_$mbt.log | cut -c1-300
done
