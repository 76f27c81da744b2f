#!/bin/bash
# Round 4: final-tree serving variants (engine mode): fp8 KV cache, chunked prefill 2048
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_37}; mkdir -p $O
B="python -m lumen.bench.serve_bench --max-model-len 1024"
timeout -k 10 300 $B --scheduling-policy prefill_first --max-batched-tokens 4096 --kv-cache-dtype fp8 > $O/fp8.json 2> $O/fp8.err || { tail -5 $O/fp8.err; exit 1; }
timeout -k 10 300 $B --scheduling-policy chunked --max-batched-tokens 2048 > $O/chunked.json 2> $O/chunked.err || { tail -5 $O/chunked.err; exit 1; }
for f in fp8 chunked; do
python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
print('$f', d['output_tok_s'], d['ttft_p50_ms'], d['itl_p50_ms'], d['itl_p99_ms'])"
done
