#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6_14
timeout -k 10 120 python scripts/probes/sampler_probe.py > gpurun_out/r6_14/sampler.json 2> gpurun_out/r6_14/err.txt || { tail -5 gpurun_out/r6_14/err.txt; exit 1; }
cat gpurun_out/r6_14/sampler.json
