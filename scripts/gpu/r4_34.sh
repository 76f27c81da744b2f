#!/bin/bash
# Round 4: fresh-prompt prefill from the q|k|v rows -- serving GPU tests, then the serve burst
# (engine) with it on and off, and the default bench serve sections
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_34}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_serving_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
B="python -m lumen.bench.serve_bench --max-model-len 1024 --scheduling-policy prefill_first --max-batched-tokens 4096"
LUMEN_FRESH_PREFILL=0 timeout -k 10 300 $B --trace-steps > $O/paged.json 2> $O/paged.err || { tail -5 $O/paged.err; exit 1; }
timeout -k 10 300 $B --trace-steps > $O/fresh.json 2> $O/fresh.err || { tail -5 $O/fresh.err; exit 1; }
timeout -k 10 300 $B > $O/fresh_async.json 2> $O/fresh_async.err || { tail -5 $O/fresh_async.err; exit 1; }
for f in paged fresh fresh_async; do
python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
print('$f', d['output_tok_s'], d['ttft_p50_ms'], d['itl_p99_ms'], (d.get('step_trace') or {}).get('prefill'))"
done
