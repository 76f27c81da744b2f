#!/bin/bash
# tune serving GEMM shapes into the shipped table, re-run the serve bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/tunableop
cp configs/tunableop/mi355x_gemms.csv gpurun_out/tunableop/mi355x_gemms.csv
timeout -k 10 900 python scripts/tune_gemms.py --out gpurun_out/tunableop/mi355x_gemms.csv > gpurun_out/r21_tune.log 2>&1 || { tail -20 gpurun_out/r21_tune.log; exit 1; }
tail -3 gpurun_out/r21_tune.log
wc -l gpurun_out/tunableop/mi355x_gemms.csv
LUMEN_GEMM_TABLE=gpurun_out/tunableop/mi355x_gemms.csv timeout -k 10 600 python lumen/bench/serve_bench.py --num-requests 256 --prompt-len 512 --max-tokens 128 > gpurun_out/r21_serve.log 2>&1 || { tail -30 gpurun_out/r21_serve.log; exit 1; }
grep -h '^{' gpurun_out/r21_serve.log
LUMEN_GEMM_TABLE=gpurun_out/tunableop/mi355x_gemms.csv timeout -k 10 600 python bench.py --steps 10 --warmup 3 --gemm_table gpurun_out/tunableop/mi355x_gemms.csv > gpurun_out/r21_bench.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r21_bench.log | cut -c100-200
