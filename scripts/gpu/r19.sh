#!/bin/bash
# serving: headline run + kernel trace for decode-step gap analysis
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python lumen/bench/serve_bench.py --num-requests 256 --prompt-len 512 --max-tokens 128 > gpurun_out/r19_serve.log 2>&1 || { tail -30 gpurun_out/r19_serve.log; exit 1; }
grep -h '^{' gpurun_out/r19_serve.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r19 -o serve --output-format csv -- python3 lumen/bench/serve_bench.py --num-requests 256 --prompt-len 512 --max-tokens 128 > gpurun_out/prof_r19.log 2>&1
echo "prof rc=$?"
