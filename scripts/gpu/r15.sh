#!/bin/bash
# BASELINE.md configs on 1 GPU: ZeRO-2 bs1 (apples-to-apples samples/s), ZeRO-1 bf16, 70B ZeRO-3
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config configs/ds_config_zero2.json --micro_batch 1 --steps 30 --warmup 5 > gpurun_out/r15_zero2_bs1.log 2>&1 || { tail -20 gpurun_out/r15_zero2_bs1.log; exit 1; }
grep -h '^{' gpurun_out/r15_zero2_bs1.log
timeout -k 10 600 python bench.py --config configs/ds_config_zero1.json --steps 10 --warmup 3 > gpurun_out/r15_zero1.log 2>&1 || { tail -20 gpurun_out/r15_zero1.log; exit 1; }
grep -h '^{' gpurun_out/r15_zero1.log
timeout -k 10 900 python bench.py --model llama2-70b --micro_batch 4 --steps 3 --warmup 2 > gpurun_out/r15_70b.log 2>&1 || { tail -30 gpurun_out/r15_70b.log; exit 1; }
grep -h '^{' gpurun_out/r15_70b.log
