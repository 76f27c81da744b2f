#!/bin/bash
# Round 4: q rotated inside the flash-attention forward (K-only RoPE pass) -- tests, then the
# training step table and the bench with it on / off
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_17}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -v --timeout 120 --timeout-method thread -k "rope or flash or llama" > $O/tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.txt | head; tail -1 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for rq in 1 0; do
  LUMEN_FA_ROPE_Q=$rq timeout -k 10 300 python bench.py --no_serve --partitioned "" --steps 20 --warmup 5 > $O/bench_rq$rq.json 2> $O/bench_rq$rq.err || { tail -5 $O/bench_rq$rq.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_rq$rq.json')); print('rope_q=$rq', d['value'], d['ms_per_step'])"
done
bash scripts/gpu/r4_4.sh ${1:-r4_17}/step
