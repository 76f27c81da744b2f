#!/bin/bash
# sampler with batched row loads: numerics tests, then timing
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6_15; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k sampling > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 120 python scripts/probes/sampler_probe.py > $O/sampler.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
cat $O/sampler.json
