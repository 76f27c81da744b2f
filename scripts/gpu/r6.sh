#!/bin/bash
# GEMM tuning (TunableOp) for the training bench shapes + before/after bench + profile
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/tunableop
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --gemm_table off > gpurun_out/b_heur.log 2>&1 || exit $?
grep '^{' gpurun_out/b_heur.log
timeout -k 10 900 python bench.py --steps 10 --warmup 3 --tune_gemms gpurun_out/tunableop/mi355x_gemms.csv > gpurun_out/b_tune.log 2>&1 || exit $?
grep '^{' gpurun_out/b_tune.log
ls -la gpurun_out/tunableop
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --gemm_table gpurun_out/tunableop/mi355x_gemms.csv > gpurun_out/b_tuned.log 2>&1 || exit $?
grep '^{' gpurun_out/b_tuned.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train2 -o train --output-format csv -- python3 bench.py --steps 4 --warmup 2 --gemm_table gpurun_out/tunableop/mi355x_gemms.csv > gpurun_out/prof_train2.log 2>&1
echo "prof rc=$?"
