#!/bin/bash
# grad-norm reduction with batched loads: numerics, kernel time, then the full suite + smoke + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_59; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "norm_sq or adamw" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/k -o k -- python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 3 --warmup 2 > $O/kb.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 scripts/tools/rocpd_summary.py $O/k norm_sq
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/gpu_suite.txt 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_suite.txt | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err2 || { tail -20 $O/bench.err2; exit 1; }
python3 -c "
import json
d = json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value', 'ms_per_step', 'vs_baseline')})
print({k: (d['extra'].get(k) or {}).get('output_tok_s') for k in ('serve', 'serve_engine', 'serve_chunked')})"
