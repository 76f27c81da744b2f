#!/bin/bash
# Round 4: serving GPU tests (prefix caching, prompt scores / alternatives, speculative decoding)
# and the default serve burst with prompt-lookup drafting on (random prompts: what it costs when
# drafts are rarely right)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_25}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_serving_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -n 2 $O/tests.txt
B="python -m lumen.bench.serve_bench --max-model-len 1024 --scheduling-policy prefill_first --max-batched-tokens 4096"
timeout -k 10 300 $B --num-speculative-tokens 4 > $O/spec4.json 2> $O/spec4.err || { tail -5 $O/spec4.err; exit 1; }
timeout -k 10 300 $B --sync-scheduling > $O/sync.json 2> $O/sync.err || { tail -5 $O/sync.err; exit 1; }
for f in spec4 sync; do
python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
print('$f', d['output_tok_s'], d['ttft_p50_ms'], d['itl_p50_ms'], d['itl_p99_ms'], d.get('spec'))"
done
# batch-1 latency, long greedy generation (random weights tend to fall into loops, which prompt
# lookup then drafts): spec off vs on
B1="python -m lumen.bench.serve_bench --max-model-len 1024 --num-requests 1 --concurrency 1 --prompt-len 32 --max-tokens 512"
timeout -k 10 300 $B1 --sync-scheduling > $O/b1_sync.json 2> $O/b1_sync.err || { tail -5 $O/b1_sync.err; exit 1; }
timeout -k 10 300 $B1 > $O/b1_async.json 2> $O/b1_async.err || { tail -5 $O/b1_async.err; exit 1; }
timeout -k 10 300 $B1 --num-speculative-tokens 4 > $O/b1_spec4.json 2> $O/b1_spec4.err || { tail -5 $O/b1_spec4.err; exit 1; }
for f in b1_sync b1_async b1_spec4; do
python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
print('$f', d['output_tok_s'], d['itl_p50_ms'], d.get('spec'))"
done
