#!/bin/bash
# Round 4: paged decode with raw-register K/V rows (fp8: 8 rows in flight per lane) -- kernel
# tests, then the engine-mode serving burst with bf16 and fp8 KV caches (prefill-first 4096)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_16}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_serving_gpu.py -q -x --timeout 120 --timeout-method thread -k "paged or fp8 or decode or serving" > $O/tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.txt | head; tail -1 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for kv in auto fp8; do
  timeout -k 10 300 python -m lumen.bench.serve_bench --max-model-len 1024 --kv-cache-dtype $kv \
    --scheduling-policy prefill_first --max-batched-tokens 4096 > $O/engine_$kv.json 2> $O/engine_$kv.err || { tail -20 $O/engine_$kv.err; exit 1; }
  python3 -c "
import json
d = json.loads([l for l in open('$O/engine_$kv.json') if l.startswith('{')][-1])
print('$kv', {k: d.get(k) for k in ('output_tok_s','ttft_p50_ms','itl_p50_ms','itl_p99_ms')})"
done
