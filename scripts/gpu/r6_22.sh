#!/bin/bash
# deterministic mode with the dY sums as a second launch: tests, then step tables det split / det in-kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_22; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_deterministic_gpu.py tests/test_fp16_gpu.py tests/test_kernels_gpu.py -k "deterministic or fp16 or lora" > $O/tests.txt 2>&1 \
  || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for split in 1 0; do
  LUMEN_LORA_DETERMINISTIC=1 LUMEN_DET_SPLIT=$split timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_s$split -o kt -- \
    python3 bench.py --steps 4 --warmup 2 --partitioned "" --no_serve --no_box > $O/bench_s$split.json 2> $O/bench_s$split.err \
    || { tail -20 $O/bench_s$split.err; exit 1; }
  python3 scripts/tools/step_table.py $O/prof_s$split > $O/step_table_s$split.txt 2>&1 || true
  head -1 $O/step_table_s$split.txt; grep -E "dy3|dxa3|down3" $O/step_table_s$split.txt | head -6
done
