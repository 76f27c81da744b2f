#!/bin/bash
# Round 4: prefix caching with same-step sharing -- shared-prefix burst and the plain burst
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_33}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_serving_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
B="python -m lumen.bench.serve_bench --max-model-len 1024 --scheduling-policy prefill_first --max-batched-tokens 4096 --enable-prefix-caching"
timeout -k 10 300 $B --shared-prefix 384 > $O/shared384_on.json 2> $O/shared384_on.err || { tail -5 $O/shared384_on.err; exit 1; }
timeout -k 10 300 $B > $O/plain_on.json 2> $O/plain_on.err || { tail -5 $O/plain_on.err; exit 1; }
for f in shared384_on plain_on; do
python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
print('$f', d['output_tok_s'], d['ttft_p50_ms'], d['itl_p99_ms'], d['prefix_hit_rate'], d['prefill_tokens_computed'])"
done
