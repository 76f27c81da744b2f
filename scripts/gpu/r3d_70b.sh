#!/bin/bash
# Llama-2-70B + LoRA r16 (q/k/v/o), 4 x 512 tokens per step, one MI355X (weights resident:
# the identity ZeRO-3 partition at world 1), current kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_70b}; mkdir -p $O
timeout -k 10 700 python bench.py --model llama2-70b --micro_batch 4 --no_serve --steps 4 --warmup 2 > $O/b70.json 2> $O/b70.err || { tail -20 $O/b70.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b70.json'));e=d['extra'];print('70b', d['ms_per_step'], d['value'], 'peak', e['peak_hbm_gb_max_rank'], 'tflops', e['tflops_per_gpu'])"
