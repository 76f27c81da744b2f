#!/bin/bash
# LM-head dH as TN against the cached W^T: numerics, trace, step A/B (LUMEN_LMHEAD_WT 1 / 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_56; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_gpu.py tests/test_zero3_gpu.py -k "lm_head or fp16 or engine or zero3" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for w in 1 0; do
  LUMEN_LMHEAD_WT=$w timeout -k 10 300 rocprofv3 --kernel-trace -d $O/k$w -o k$w -- python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 3 --warmup 2 > $O/kb_$w.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 scripts/tools/rocpd_by_grid.py $O/k$w Cijk | sort -k3 -n -r | head -8
done
for w in 1 0 1 0; do
  LUMEN_LMHEAD_WT=$w timeout -k 10 300 python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 20 --warmup 5 > $O/bench_$w.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print('lmhead_wt $w', d['value'], d['ms_per_step'], d['extra']['final_loss'], d['extra']['peak_hbm_gb_max_rank'])"
done
