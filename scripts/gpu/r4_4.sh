#!/bin/bash
# Round 4 profiles: one traced training step (rocprofv3 kernel trace -> step table) and the
# serving burst (kernel trace: decode-step composition with the decode-batch GEMM plans)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_4}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o run -- python3 bench.py --no_serve --partitioned "" --steps 6 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 scripts/tools/step_table.py $O/step > $O/step_table.txt 2>&1 || true
head -30 $O/step_table.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serve -o run -- python3 -m lumen.bench.serve_bench --max-model-len 1024 > $O/serve.json 2> $O/serve.err || { tail -5 $O/serve.err; exit 1; }
tail -1 $O/serve.json | cut -c1-300
f=$(find $O/serve -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp $f $O/serve_kernel_stats.csv && head -25 $O/serve_kernel_stats.csv | cut -d, -f1-6
