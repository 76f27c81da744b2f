#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -m gpu -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python lumen/bench/attn_bench.py > gpurun_out/attn.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 900 python lumen/bench/serve_bench.py --num-requests 256 --prompt-len 512 --max-tokens 128 > gpurun_out/serve.log 2>&1
echo "serve rc=$?"
