#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -m gpu -q -k "paged or serving or engine" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python lumen/bench/serve_bench.py --num-requests 256 --prompt-len 512 --max-tokens 128 > gpurun_out/serve.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_serve -o serve --output-format csv -- python3 lumen/bench/serve_bench.py --num-requests 128 --prompt-len 512 --max-tokens 64 > gpurun_out/prof_serve.log 2>&1
echo "prof rc=$?"
