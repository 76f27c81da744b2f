#!/bin/bash
# pair-hash dropout: numerics + bench; FA PMC counters at the training shape
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "lora or transposed or llama" > gpurun_out/r12_tests.log 2>&1 || { tail -40 gpurun_out/r12_tests.log; exit 1; }
tail -2 gpurun_out/r12_tests.log
timeout -k 10 300 python -m lumen.bench.lora_bench > gpurun_out/r12_lora_bench.log 2>&1 || { cat gpurun_out/r12_lora_bench.log; exit 1; }
cat gpurun_out/r12_lora_bench.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r12_bench.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r12_bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pmc12 -o attn --output-format csv -- python3 lumen/bench/attn_bench.py --iters 2 > gpurun_out/pmc12.log 2>&1
echo "pmc rc=$?"
