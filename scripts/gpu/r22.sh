#!/bin/bash
# serving through the OpenAI HTTP API + async client (the reference's declared path)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python lumen/bench/serve_bench.py --mode http --num-requests 256 --concurrency 256 --prompt-len 512 --max-tokens 128 > gpurun_out/r22_http.log 2>&1 || { tail -40 gpurun_out/r22_http.log; exit 1; }
grep -h '^{' gpurun_out/r22_http.log
