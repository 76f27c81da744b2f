#!/bin/bash
# Round 4 rehearsal of the driver's round-end GPU tiers: the whole GPU suite, smoke(), bench.py
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_24}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_suite.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_suite.txt | head; tail -n 1 $O/gpu_suite.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -n 20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -n 20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); e=d['extra']
print(d['value'], d['ms_per_step'], d['vs_baseline'])
for k in ('serve', 'serve_engine', 'serve_chunked'):
    s = e.get(k) or {}
    print(k, s.get('output_tok_s'), s.get('ttft_p50_ms'), s.get('itl_p99_ms'))"
