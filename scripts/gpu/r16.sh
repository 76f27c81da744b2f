#!/bin/bash
# register-resident P/dS in the flash-attention backward: numerics, attention timing, bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "flash or llama" > gpurun_out/r16_tests.log 2>&1 || { tail -40 gpurun_out/r16_tests.log; exit 1; }
tail -2 gpurun_out/r16_tests.log
timeout -k 10 200 python lumen/bench/attn_bench.py > gpurun_out/r16_attn.log 2>&1 || { cat gpurun_out/r16_attn.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r16_attn.log
timeout -k 10 200 python lumen/bench/attn_bench.py --B 1 --S 4096 > gpurun_out/r16_attn_long.log 2>&1 && grep -v amdgpu.ids gpurun_out/r16_attn_long.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r16_bench.log 2>&1 || exit $?
grep -h '^{' gpurun_out/r16_bench.log | cut -c100-200
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pmc16 -o attn --output-format csv -- python3 lumen/bench/attn_bench.py --iters 2 > gpurun_out/pmc16.log 2>&1
echo "pmc rc=$?"
