#!/bin/bash
# direct LoRA grad accumulation + zero arena: numerics, bench, profile
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "lora or engine or transposed or rms or llama or flash" > gpurun_out/r23_tests.log 2>&1 || { tail -40 gpurun_out/r23_tests.log; exit 1; }
tail -2 gpurun_out/r23_tests.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r23_bench.log 2>&1 || { tail -30 gpurun_out/r23_bench.log; exit 1; }
grep -h '^{' gpurun_out/r23_bench.log | cut -c100-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r23 -o train --output-format csv -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/prof_r23.log 2>&1
echo "prof rc=$?"
