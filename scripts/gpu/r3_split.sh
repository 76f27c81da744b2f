#!/bin/bash
# wave-quantisation probe: one-piece vs column-split MLP GEMMs (tunes the new shapes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3_split}; mkdir -p $O
timeout -k 10 600 python -u -m lumen.bench.split_gemm_probe --tune $O/tuned.csv > $O/probe.txt 2>&1 || exit $?
tail -3 $O/probe.txt
