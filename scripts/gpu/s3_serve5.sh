#!/bin/bash
# serving: kernel tests, serve bench at 1/16/64/256 requests, batch-1 decode kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s3_serve5}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_serving_gpu.py -k "rmsnorm or paged or engine or decode or serving or skinny or swiglu or rope_write" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for n in ${NREQ:-1 16 64 256}; do
  timeout -k 10 300 python lumen/bench/serve_bench.py --num-requests $n > $O/serve_$n.log 2>&1 || exit 1
  tail -1 $O/serve_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['output_tok_s'], 'ttft', d['ttft_p50_ms'], 'itl', d['itl_p50_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o run -- python3 lumen/bench/serve_bench.py --num-requests 1 > $O/prof1.log 2>&1 || exit 1
find $O/prof1 -name "*kernel_stats.csv" | head -1 | xargs -I{} head -20 {}
