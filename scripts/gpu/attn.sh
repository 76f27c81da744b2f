#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -k "flash or llama_layer" > gpurun_out/fa_tests.log 2>&1
rc=$?; echo "fa tests rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
LUMEN_FA_MT=1 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -k "flash" > gpurun_out/fa_tests_mt1.log 2>&1
rc=$?; echo "fa tests mt1 rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
LUMEN_FA_MT=2 timeout -k 10 300 python lumen/bench/attn_bench.py > gpurun_out/attn.log 2>&1 || exit $?
LUMEN_FA_MT=1 timeout -k 10 300 python lumen/bench/attn_bench.py --only fwd >> gpurun_out/attn.log 2>&1 || exit $?
timeout -k 10 300 python lumen/bench/attn_bench.py --B 1 --S 4096 >> gpurun_out/attn.log 2>&1 || exit $?
