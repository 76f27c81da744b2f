#!/bin/bash
# decode GEMM staging pipeline without math: LDS-DMA ring vs register staging
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5_24
timeout -k 10 120 ./build_probe/spp > gpurun_out/r5_24/spp.jsonl 2>&1; rc=$?
cat gpurun_out/r5_24/spp.jsonl
exit $rc
