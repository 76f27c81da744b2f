#!/bin/bash
# decode GEMM cost probe (where its time goes at M = 256), then the full bench with the pipelined paged decode default
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_14
timeout -k 10 400 python -u scripts/probes/dgemm_costprobe.py > gpurun_out/r5_14/costprobe.jsonl 2> gpurun_out/r5_14/costprobe.err || { tail -20 gpurun_out/r5_14/costprobe.err; exit 1; }
timeout -k 10 900 python -u bench.py > gpurun_out/r5_14/bench.json 2> gpurun_out/r5_14/bench.err || { tail -20 gpurun_out/r5_14/bench.err; exit 1; }
cat gpurun_out/r5_14/costprobe.jsonl
tail -c 1500 gpurun_out/r5_14/bench.json
