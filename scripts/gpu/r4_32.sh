#!/bin/bash
# Round 4: serving soak over HTTP -- 3072 streamed requests at 32 req/s (~100 s) with prefix
# caching on, 4 API + 4 client processes; at the end every request must be done, every KV block
# back, no client errors
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_32}; mkdir -p $O
timeout -k 10 400 python -m lumen.bench.serve_bench --mode http --max-model-len 1024 \
  --scheduling-policy prefill_first --max-batched-tokens 4096 --api-servers 4 --client-procs 4 \
  --enable-prefix-caching --num-requests 3072 --request-rate 32 > $O/soak.json 2> $O/soak.err || { tail -10 $O/soak.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/soak.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('requests','ok','errors','output_tok_s','ttft_p50_ms','ttft_p99_ms','itl_p50_ms','itl_p99_ms','wall_s','kv_blocks','kv_blocks_free_at_end','engine_requests_left','prefix_hit_rate')})
assert d.get('errors', 0) == 0 and d['kv_blocks_free_at_end'] == d['kv_blocks'] and d['engine_requests_left'] == 0"
