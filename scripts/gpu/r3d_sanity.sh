#!/bin/bash
# round-3 re-entry sanity: GPU suite, smoke, default driver bench (train + extra.serve)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_sanity}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
