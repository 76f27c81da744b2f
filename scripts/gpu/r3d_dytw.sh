#!/bin/bash
# dY-pass rows per block (LUMEN_LORA_DY_TW): default (256 / 128 for o_proj) vs 512 / 1024
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_dytw}; mkdir -p $O
for tw in 0 512 1024; do
  LUMEN_LORA_DY_TW=$tw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step_$tw -o run -- python3 bench.py --no_serve --steps 4 --warmup 3 > $O/traced_$tw.json 2> $O/traced_$tw.err || { tail -5 $O/traced_$tw.err; exit 1; }
  python3 scripts/tools/step_table.py $O/step_$tw > $O/step_table_$tw.txt && grep -E "wall|dy3" $O/step_table_$tw.txt | sed "s/^/TW=$tw /"
done
for tw in 512 0 512; do
  LUMEN_LORA_DY_TW=$tw timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/bench_$tw.json 2> $O/bench_$tw.err || { tail -5 $O/bench_$tw.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$tw.json'));print('bench TW=$tw', d['ms_per_step'], d['value'])"
done
