#!/bin/bash
# serving M = 2048 o / down as whole-GEMM split-K on the hand-written GEMM vs the library
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6_07
timeout -k 10 300 python -u scripts/probes/mlp_gemm_probe.py --only serve --rounds 5 --reps 20 > gpurun_out/r6_07/probe.txt 2>&1
cat gpurun_out/r6_07/probe.txt | tail -5
