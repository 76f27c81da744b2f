#!/bin/bash
# retune GEMMs with cold-cache (rotating buffer) timing, compare in-situ
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/tunableop
T=gpurun_out/tunableop/mi355x_gemms_cold.csv
rm -f $T
timeout -k 10 900 python bench.py --steps 5 --warmup 3 --tune_gemms $T > gpurun_out/r9_tune.log 2>&1 || { tail -20 gpurun_out/r9_tune.log; exit 1; }
grep -h '^{' gpurun_out/r9_tune.log | cut -c1-250
cat $T
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --gemm_table $T > gpurun_out/r9_cold.log 2>&1 || exit $?
echo "cold-tuned: $(grep -h '^{' gpurun_out/r9_cold.log | cut -c150-260)"
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r9_warm.log 2>&1 || exit $?
echo "warm-tuned: $(grep -h '^{' gpurun_out/r9_warm.log | cut -c150-260)"
