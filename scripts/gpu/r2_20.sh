#!/bin/bash
# fp8 KV cache: kernel numerics, embedding gather, serving GPU tests, then the 256-request
# serving bench with the fp8 cache at budgets 2048 / 4096 (engine) and 2048 (HTTP)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_20}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_serving_gpu.py -k "fp8 or embedding or paged or serving or engine" -v --timeout 120 --timeout-method thread > $O/t.txt 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/t.txt | tail -8; [ $rc -eq 0 ] || exit $rc
for b in 2048 4096; do
  timeout -k 10 300 python -m lumen.bench.serve_bench --mode engine --max-batched-tokens $b --kv-cache-dtype fp8 >> $O/serve_engine.jsonl 2>> $O/serve.err || exit $?
  python -c "import json;d=[json.loads(l) for l in open('$O/serve_engine.jsonl')][-1];print(d['max_batched_tokens'], d['kv_cache_dtype'], d['output_tok_s'], 'ttft50', d['ttft_p50_ms'], 'itl50', d['itl_p50_ms'], 'itl99', d['itl_p99_ms'], 'blocks', d['kv_blocks'])"
done
timeout -k 10 400 python -m lumen.bench.serve_bench --mode http --max-batched-tokens 2048 --kv-cache-dtype fp8 > $O/serve_http.json 2>> $O/serve_http.err || exit $?
cut -c1-500 $O/serve_http.json
