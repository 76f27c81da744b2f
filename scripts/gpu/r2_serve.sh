#!/bin/bash
# round 2: GPU tests (serving + kernels), then the 256-request serving bench (512 in / 128 out)
# at several per-step token budgets (chunked prefill + mixed steps), engine and HTTP mode.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_serve}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_serving_gpu.py tests/test_kernels_gpu.py tests/test_custom_ar_gpu.py -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -2 $O/gpu_tests.txt
[ $rc -le 1 ] || exit $rc
for b in 2048 4096 8192; do
  timeout -k 10 400 python -m lumen.bench.serve_bench --mode engine --max-batched-tokens $b >> $O/serve_engine.jsonl 2>> $O/serve.err || exit $?
  tail -1 $O/serve_engine.jsonl | cut -c1-400
done
timeout -k 10 600 python -m lumen.bench.serve_bench --mode http --max-batched-tokens 2048 > $O/serve_http.json 2>> $O/serve_http.err || exit $?
cut -c1-600 $O/serve_http.json
