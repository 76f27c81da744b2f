#!/bin/bash
# serving: prefill boost (x2 token budget while <= 64 sequences decode) vs off, interleaved;
# then the OpenAI HTTP path with the boost
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_boost}; mkdir -p $O
for b in 2 1 2 1; do
  timeout -k 10 300 python -m lumen.bench.serve_bench --prefill-boost $b > $O/engine_b$b.json 2> $O/engine_b$b.err || { tail -5 $O/engine_b$b.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/engine_b$b.json').read().splitlines()[-1]);print('boost $b', d['output_tok_s'], 'ttft p50/p99', d['ttft_p50_ms'], d['ttft_p99_ms'], 'itl p50/p99', d['itl_p50_ms'], d['itl_p99_ms'])"
done
timeout -k 10 400 python -m lumen.bench.serve_bench --mode http --prefill-boost 2 > $O/http_b2.json 2> $O/http_b2.err || { tail -5 $O/http_b2.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/http_b2.json').read().splitlines()[-1]);print('http boost 2', d['output_tok_s'], 'ttft p50', d['ttft_p50_ms'], 'itl p50/p99', d['itl_p50_ms'], d['itl_p99_ms'])"
