#!/bin/bash
# LoRA v2 (16-bit MFMA) kernels: numerics, micro timing, training bench, profile
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "lora or transposed" > gpurun_out/r10_tests.log 2>&1 || { tail -40 gpurun_out/r10_tests.log; exit 1; }
tail -2 gpurun_out/r10_tests.log
timeout -k 10 300 python -m lumen.bench.lora_bench > gpurun_out/r10_lora_bench.log 2>&1 || { cat gpurun_out/r10_lora_bench.log; exit 1; }
cat gpurun_out/r10_lora_bench.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r10_bench.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r10_bench.log | cut -c1-330
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r10 -o train --output-format csv -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/prof_r10.log 2>&1
echo "prof rc=$?"
