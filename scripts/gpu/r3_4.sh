#!/bin/bash
# RMSNorm occupancy-cap probe, then bench A/B of the best cap
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3_4}; mkdir -p $O
timeout -k 10 120 python -u -m lumen.bench.rmsnorm_probe > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt | grep lds
timeout -k 10 200 python -u -m pytest tests -m gpu -k "rmsnorm or rms_norm" -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1; tail -1 $O/gpu_tests.txt
