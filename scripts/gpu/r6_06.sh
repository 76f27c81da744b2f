#!/bin/bash
# fused MLP GEMM end to end: bench A/B (LUMEN_FUSED_MLP 0 / 1, alternating) + a step table of 1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_06; mkdir -p $O
for fm in 0 1 0 1; do
  LUMEN_FUSED_MLP=$fm timeout -k 10 300 python bench.py --steps 10 --warmup 3 --partitioned "" --no_serve --no_box \
    > $O/bench_fm$fm.json 2> $O/bench_fm$fm.err || { tail -20 $O/bench_fm$fm.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_fm$fm.json'));print('fm $fm', d['value'], d['ms_per_step'], d['extra']['final_loss'])"
done
LUMEN_FUSED_MLP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_fm1 -o kt -- \
  python3 bench.py --steps 4 --warmup 2 --partitioned "" --no_serve --no_box > $O/bench_prof.json 2> $O/bench_prof.err \
  || { tail -20 $O/bench_prof.err; exit 1; }
python3 scripts/tools/step_table.py $O/prof_fm1 > $O/step_table_fm1.txt 2>&1 || true
head -40 $O/step_table_fm1.txt
