#!/bin/bash
# step tables: deterministic adapter reductions (default) vs the f32-atomic form
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_04; mkdir -p $O
for det in 1; do
  LUMEN_LORA_DETERMINISTIC=$det timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_det$det -o kt -- \
    python3 bench.py --steps 4 --warmup 2 --partitioned "" --no_serve --no_box > $O/bench_det$det.json 2> $O/bench_det$det.err \
    || { tail -20 $O/bench_det$det.err; exit 1; }
  python3 scripts/tools/step_table.py $O/prof_det$det > $O/step_table_det$det.txt 2>&1 || true
  head -40 $O/step_table_det$det.txt
done
