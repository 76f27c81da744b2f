#!/bin/bash
# Round 4: fp32 backward probe (module-output gradients GPU vs CPU), then the world-8 bench
# rehearsal and TP=1 vs TP=2 serving (the tail of r4_6)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_9}; mkdir -p $O
timeout -k 10 180 python scripts/probes/fp32_probe.py > $O/fp32_probe.txt 2>&1 || { tail -20 $O/fp32_probe.txt; exit 1; }
grep -E "DOUT|GRAD|loss|done" $O/fp32_probe.txt | head -60
sed -n '/^export LUMEN_SHARED_GPU_REHEARSAL=1 LUMEN_DIST_TIMEOUT/,$p' scripts/gpu/r4_6.sh | sed "s#\$O#$O#g" > $O/rest.sh
bash $O/rest.sh
