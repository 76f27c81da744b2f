#!/bin/bash
# Round 4: paged decode with q read in place -- kernel / serving / TP tests, then the serve burst
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_35}; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_serving_gpu.py tests/test_kernels_gpu.py tests/test_rccl_gpu.py -k "paged or decode or serving or prefill or tp or fp8 or spec or prefix or prompt" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
timeout -k 10 300 python -m lumen.bench.serve_bench --max-model-len 1024 --scheduling-policy prefill_first --max-batched-tokens 4096 --trace-steps > $O/trace.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
timeout -k 10 300 python -m lumen.bench.serve_bench --max-model-len 1024 --scheduling-policy prefill_first --max-batched-tokens 4096 > $O/engine.json 2> $O/engine.err || { tail -5 $O/engine.err; exit 1; }
for f in trace engine; do
python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
st=d.get('step_trace') or {}
print('$f', d['output_tok_s'], d['ttft_p50_ms'], d['itl_p50_ms'], d['itl_p99_ms'], (st.get('decode') or {}).get('ms_mean'), (st.get('prefill') or {}).get('ms_mean'))"
done
