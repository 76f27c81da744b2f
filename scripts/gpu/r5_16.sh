#!/bin/bash
# load-path ceiling of the decode GEMM's access pattern (plain loads, no LDS / MFMA)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5_16
timeout -k 10 120 ./build_probe/l2p > gpurun_out/r5_16/l2p.jsonl 2>&1; rc=$?
cat gpurun_out/r5_16/l2p.jsonl
exit $rc
