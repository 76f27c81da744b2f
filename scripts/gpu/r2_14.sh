#!/bin/bash
# serving: async scheduling (step t+1 launched before step t's tokens reach the host).
# GPU serving tests, then engine-mode 256 x (512 in / 128 out) at token budgets, async vs sync,
# then HTTP mode at the chosen budget.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_14}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_serving_gpu.py -v --timeout 300 --timeout-method thread > $O/serve_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/serve_tests.txt | head; tail -1 $O/serve_tests.txt; [ $rc -eq 0 ] || exit $rc
for b in 1024 2048 4096; do
  for m in "" "--sync-scheduling"; do
    timeout -k 10 300 python -m lumen.bench.serve_bench --mode engine --max-batched-tokens $b $m >> $O/serve_engine.jsonl 2>> $O/serve.err || exit $?
    python -c "import json;d=[json.loads(l) for l in open('$O/serve_engine.jsonl')][-1];print(d['max_batched_tokens'], d['async_scheduling'], d['output_tok_s'], 'ttft50', d['ttft_p50_ms'], 'itl50', d['itl_p50_ms'], 'itl99', d['itl_p99_ms'], 'steps', d['steps'])"
  done
done
timeout -k 10 400 python -m lumen.bench.serve_bench --mode http --max-batched-tokens 2048 > $O/serve_http.json 2>> $O/serve_http.err || exit $?
cut -c1-600 $O/serve_http.json
