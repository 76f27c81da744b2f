#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_12
hipcc --offload-arch=gfx950 -O3 -o /tmp/hbm_read scripts/probes/hbm_read_probe.cpp > /dev/null 2>&1 || exit 1
timeout -k 10 120 /tmp/hbm_read > gpurun_out/r5_12/hbm_read.jsonl 2>&1
rc=$?
cat gpurun_out/r5_12/hbm_read.jsonl
exit $rc
