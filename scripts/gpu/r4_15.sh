#!/bin/bash
# Round 4: serving variants over HTTP with the scaled-out front-end (4 API + 4 client processes):
# fp8 KV cache under prefill-first, and bf16 at Llama-2's full 4096 context (vLLM 0.6.0's defaults
# end to end: max_model_len 4096 -> 4096-token steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_15}; mkdir -p $O
for cfg in "fp8 1024" "auto 4096"; do
  set -- $cfg
  n=http_pf_kv$1_ctx$2
  timeout -k 10 300 python -m lumen.bench.serve_bench --mode both --max-model-len $2 --kv-cache-dtype $1 \
    --scheduling-policy prefill_first --max-batched-tokens 4096 --api-servers 4 --client-procs 4 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json
for l in open('$O/$n.json'):
    if l.startswith('{'):
        d = json.loads(l)
        for r in (d, d.get('engine') or {}):
            print('$n', r.get('mode'), {k: r.get(k) for k in ('output_tok_s','ttft_p50_ms','itl_p50_ms','itl_p90_ms','itl_p99_ms','itl_max_ms')})"
done
