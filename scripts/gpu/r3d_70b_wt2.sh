#!/bin/bash
# Llama-2-70B one GPU after the W^T budget fix (allocator-cached blocks count as free), then the
# 7B bench to confirm it is unchanged
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_70b_wt2}; mkdir -p $O
timeout -k 10 700 python bench.py --model llama2-70b --micro_batch 4 --no_serve --steps 4 --warmup 2 > $O/b70.json 2> $O/b70.err || { tail -20 $O/b70.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b70.json'));e=d['extra'];print('70b', d['ms_per_step'], d['value'], 'peak', e['peak_hbm_gb_max_rank'])"
timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/b7.json 2> $O/b7.err || { tail -5 $O/b7.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b7.json'));e=d['extra'];print('7b', d['ms_per_step'], d['value'], 'peak', e['peak_hbm_gb_max_rank'])"
