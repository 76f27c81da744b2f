#!/bin/bash
# Llama-2-70B one GPU: persistent W^T for more projections (smaller activation reserve)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_70b_wt}; mkdir -p $O
for r in 40 0; do
  LUMEN_BWD_WT_RESERVE_GB=$r timeout -k 10 700 python bench.py --model llama2-70b --micro_batch 4 --no_serve --steps 4 --warmup 2 > $O/b70_r$r.json 2> $O/b70_r$r.err || { tail -20 $O/b70_r$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b70_r$r.json'));e=d['extra'];print('70b reserve=$r', d['ms_per_step'], d['value'], 'peak', e['peak_hbm_gb_max_rank'])"
done
