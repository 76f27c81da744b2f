#!/bin/bash
# single-pass vs two-pass paged decode: numerics, then serve bench A/B on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s3_pa1}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_serving_gpu.py -k "paged or decode or serving or engine" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for n in 256 16 1; do
  for one in 0 1; do
    LUMEN_PA_1PASS=$one timeout -k 10 300 python lumen/bench/serve_bench.py --num-requests $n > $O/serve_${one}_$n.log 2>&1 || exit 1
    tail -1 $O/serve_${one}_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('one_pass=$one n=$n', d['output_tok_s'], 'ttft', d['ttft_p50_ms'], 'itl', d['itl_p50_ms'])"
  done
done
