#!/bin/bash
# A/B of the serving decode fusions (fused split-context merge, SwiGLU-in-GEMV) on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s3_pa_ab}; mkdir -p $O
run() {  # tag env... : serve bench at n requests
  local tag=$1 n=$2; shift 2
  env "$@" timeout -k 10 300 python lumen/bench/serve_bench.py --num-requests $n > $O/serve_${tag}_$n.log 2>&1 || exit 1
  tail -1 $O/serve_${tag}_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', $n, d['output_tok_s'], 'ttft', d['ttft_p50_ms'], 'itl', d['itl_p50_ms'])"
}
for n in 1 16 256; do
  run off $n LUMEN_PA_FUSED_MERGE=0 LUMEN_SWIGLU_GEMV=0
  run merge $n LUMEN_PA_FUSED_MERGE=1 LUMEN_SWIGLU_GEMV=0
  run both $n LUMEN_PA_FUSED_MERGE=1 LUMEN_SWIGLU_GEMV=1
done
