#!/bin/bash
# Round 4: HTTP serving under both policies (lighter client parsing), then a rocprofv3
# kernel-stats profile of the prefill-first engine run (bench.py's extra.serve configuration)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_13}; mkdir -p $O
for cfg in "prefill_first 4096" "chunked 2048"; do
  set -- $cfg
  timeout -k 10 300 python -m lumen.bench.serve_bench --mode both --max-model-len 1024 \
    --scheduling-policy $1 --max-batched-tokens $2 > $O/http_$1_$2.json 2> $O/http_$1_$2.err || { tail -20 $O/http_$1_$2.err; exit 1; }
  python3 -c "
import json
for l in open('$O/http_$1_$2.json'):
    if l.startswith('{'):
        d = json.loads(l)
        for r in (d, d.get('engine') or {}):
            print('$1 $2', r.get('mode'), {k: r.get(k) for k in ('output_tok_s','ttft_p50_ms','itl_p50_ms','itl_p90_ms','itl_p95_ms','itl_p99_ms','itl_max_ms')})"
done
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o serve_pf -- python3 -m lumen.bench.serve_bench \
  --max-model-len 1024 --scheduling-policy prefill_first --max-batched-tokens 4096 > $O/prof_run.json 2> $O/prof_run.err || { tail -20 $O/prof_run.err; exit 1; }
find $O/prof -name "*kernel_stats.csv"
