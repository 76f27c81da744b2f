#!/bin/bash
# round 2: full GPU suite on the tree with chunked prefill, 1-GPU bench, serving bench
# (256 requests, 512 in / 128 out) with chunked prefill + mixed steps, engine + HTTP.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_5}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -2 $O/gpu_tests.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || exit $?
cut -c1-400 $O/bench_n1.json
for b in 2048 8192; do
  timeout -k 10 300 python -m lumen.bench.serve_bench --mode engine --max-batched-tokens $b >> $O/serve_engine.jsonl 2>> $O/serve.err || exit $?
  tail -1 $O/serve_engine.jsonl | cut -c1-500
done
timeout -k 10 400 python -m lumen.bench.serve_bench --mode http --max-batched-tokens 2048 > $O/serve_http.json 2>> $O/serve_http.err || exit $?
cut -c1-700 $O/serve_http.json
