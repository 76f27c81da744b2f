#!/bin/bash
# Round 4: serving scheduling policies on Llama-2-7B TP=1 (256 x 512 in / 128 out, all at t=0):
# chunked (mixed decode + prefill-chunk steps) vs prefill_first (vLLM 0.6.0's default: prefill-only
# steps while prompts wait) at several step budgets; then chunked with the decode-GEMM plans off.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_7}; mkdir -p $O
run() {  # name, extra args...
  local n=$1; shift
  timeout -k 10 300 python -m lumen.bench.serve_bench --max-model-len 1024 "$@" > $O/$n.json 2> $O/$n.err \
    || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$O/$n.json') if l.startswith('{')][-1]); print('$n', {k: d.get(k) for k in ('output_tok_s','ttft_p50_ms','ttft_p99_ms','itl_p50_ms','itl_p99_ms','itl_max_ms','steps','wall_s')})"
}
run chunked_2048 --max-batched-tokens 2048 &&
run pf_2048 --max-batched-tokens 2048 --scheduling-policy prefill_first &&
run pf_4096 --max-batched-tokens 4096 --scheduling-policy prefill_first &&
run pf_8192 --max-batched-tokens 8192 --scheduling-policy prefill_first &&
run chunked_4096 --max-batched-tokens 4096 &&
LUMEN_DGEMM=0 run chunked_2048_nodgemm --max-batched-tokens 2048
