#!/bin/bash
# dxa3 with the dropout masks shared through LDS (hashed once per element instead of twice):
# LoRA numerics (toy + production shapes vs fp32), kernel times and the step A/B
# (LUMEN_LV3_PROBE=128 = the former second hash)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_49; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "lora or production or fp32_model or fold" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for p in 0 128; do
  LUMEN_LV3_PROBE=$p timeout -k 10 300 rocprofv3 --kernel-trace -d $O/k$p -o k$p -- python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 3 --warmup 2 > $O/kb_$p.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 scripts/tools/rocpd_summary.py $O/k$p dxa3
done
for p in 0 128 0 128; do
  LUMEN_LV3_PROBE=$p timeout -k 10 300 python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 20 --warmup 5 > $O/bench_$p.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$p.json')); print('probe $p', d['value'], d['ms_per_step'])"
done
