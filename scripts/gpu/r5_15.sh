#!/bin/bash
# decode GEMM cost probe with graph-replayed timing
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_15
timeout -k 10 400 python -u scripts/probes/dgemm_costprobe.py > gpurun_out/r5_15/costprobe.jsonl 2> gpurun_out/r5_15/costprobe.err || { tail -20 gpurun_out/r5_15/costprobe.err; exit 1; }
cat gpurun_out/r5_15/costprobe.jsonl
