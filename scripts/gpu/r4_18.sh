#!/bin/bash
# Round 4: bounded-grid world-1 gather copies -- copy / ZeRO-3 GPU tests, then the partitioned
# bench rows with LUMEN_GATHER_COPY_BLOCKS 32 / 64 / 0 (0 = the runtime's blit copy)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_18}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_zero3_gpu.py -q -x --timeout 150 --timeout-method thread -k "stream_copy or schedules or poison or transposed" > $O/tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.txt | head; tail -1 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for b in 32 64 0; do
  LUMEN_GATHER_COPY_BLOCKS=$b timeout -k 10 400 python bench.py --no_serve --steps 10 --warmup 3 > $O/bench_b$b.json 2> $O/bench_b$b.err || { tail -5 $O/bench_b$b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_b$b.json')); e=d['extra']
print('blocks=$b', d['value'], d['ms_per_step'], {k: (e[k]['ms_per_step'], e[k]['exposed_gather_wait_ms_per_step_max_rank']) for k in ('zero3_release','zero3_hybrid')})"
done
