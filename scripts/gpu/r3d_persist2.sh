#!/bin/bash
# persistent forward attention as the default (training + paged prefill): numerics, the
# training step and the serving burst, persistent (11) vs one-shot forward (9) interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_persist2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
for p in 11 9 11 9; do
  LUMEN_FA_PERSIST=$p timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/bench_$p.json 2> $O/bench_$p.err || { tail -5 $O/bench_$p.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$p.json'));print('train persist=$p', d['ms_per_step'], d['value'])"
done
for p in 11 9 11 9; do
  LUMEN_FA_PERSIST=$p timeout -k 10 300 python -m lumen.bench.serve_bench > $O/serve_$p.json 2> $O/serve_$p.err || { tail -5 $O/serve_$p.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/serve_$p.json').read().splitlines()[-1]);print('serve persist=$p', d['output_tok_s'], 'ttft p50', d['ttft_p50_ms'], 'itl p50/p99', d['itl_p50_ms'], d['itl_p99_ms'])"
done
