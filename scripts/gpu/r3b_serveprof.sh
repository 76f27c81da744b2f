#!/bin/bash
# serving: engine bench (256 x 512 in / 128 out, budget 2048) with a rocprofv3 kernel trace, then
# the same through the OpenAI HTTP server + async client
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3b_serveprof}; mkdir -p $O
timeout -k 10 300 python -m lumen.bench.serve_bench > $O/engine.json 2> $O/engine.err || { tail -5 $O/engine.err; exit 1; }
tail -1 $O/engine.json | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -m lumen.bench.serve_bench > $O/engine_prof.json 2> $O/engine_prof.err || { tail -5 $O/engine_prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -30 $O/kernel_stats.csv | cut -d, -f1-8
timeout -k 10 400 python -m lumen.bench.serve_bench --mode http > $O/http.json 2> $O/http.err || { tail -5 $O/http.err; exit 1; }
tail -1 $O/http.json | cut -c1-400
