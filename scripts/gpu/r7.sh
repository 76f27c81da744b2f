#!/bin/bash
# TN backward GEMM layout: numerics test, tune the new shapes, A/B the policies
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/tunableop
T=gpurun_out/tunableop/mi355x_gemms.csv
cp configs/tunableop/mi355x_gemms.csv $T
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "transposed or lora" > gpurun_out/r7_tests.log 2>&1 || { tail -30 gpurun_out/r7_tests.log; exit 1; }
tail -2 gpurun_out/r7_tests.log
LUMEN_BWD_WT=all timeout -k 10 900 python bench.py --steps 5 --warmup 3 --tune_gemms $T > gpurun_out/r7_tune_all.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r7_tune_all.log | cut -c1-300
for pol in default all none; do
  if [ $pol = default ]; then unset LUMEN_BWD_WT; else export LUMEN_BWD_WT=$pol; fi
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 --gemm_table $T > gpurun_out/r7_b_$pol.log 2>&1 || exit $?
  echo "$pol: $(grep -h '^{' gpurun_out/r7_b_$pol.log | cut -c1-260)"
done
cat $T
