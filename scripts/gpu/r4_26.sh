#!/bin/bash
# Round 4: latency vs offered load over the OpenAI HTTP path (Poisson arrivals, 256 requests of
# 512 / 128 tokens, Llama-2-7B, bf16 KV, vLLM 0.6 scheduling, 4 API + 4 client processes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_26}; mkdir -p $O
for r in ${RATES:-4 8 16 32}; do
  timeout -k 10 300 python -m lumen.bench.serve_bench --mode http --max-model-len 1024 \
    --scheduling-policy prefill_first --max-batched-tokens 4096 --api-servers 4 --client-procs 4 \
    --request-rate $r > $O/rate$r.json 2> $O/rate$r.err || { tail -5 $O/rate$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/rate$r.json').read().strip().splitlines()[-1])
print('rate $r', {k: d.get(k) for k in ('output_tok_s','ttft_p50_ms','ttft_p99_ms','itl_p50_ms','itl_p99_ms','wall_s')})"
done
