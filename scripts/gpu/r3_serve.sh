#!/bin/bash
# final-tree serving re-check: 256 requests x (512 in / 128 out), engine at budgets 2048 / 4096,
# fp8 KV at 2048, and the OpenAI HTTP path at 2048
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3_serve}; mkdir -p $O
for b in 2048 4096; do
  timeout -k 10 400 python -m lumen.bench.serve_bench --mode engine --max-batched-tokens $b >> $O/serve_engine.jsonl 2>> $O/serve.err || exit $?
  tail -1 $O/serve_engine.jsonl | cut -c1-300
done
timeout -k 10 400 python -m lumen.bench.serve_bench --mode engine --max-batched-tokens 2048 --kv-cache-dtype fp8 >> $O/serve_engine_fp8.jsonl 2>> $O/serve.err || exit $?
tail -1 $O/serve_engine_fp8.jsonl | cut -c1-300
timeout -k 10 600 python -m lumen.bench.serve_bench --mode http --max-batched-tokens 2048 > $O/serve_http.json 2>> $O/serve_http.err || exit $?
cut -c1-400 $O/serve_http.json
