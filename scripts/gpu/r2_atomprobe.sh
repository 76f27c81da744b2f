#!/bin/bash
# LoRA kernel cost probes: dy3 / dxa3 with their global f32 atomics switched off (probe bits)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r2_atom}; mkdir -p $O
for pb in ${PROBES:-0 16 32 48 64}; do
  LUMEN_LV3_PROBE=$pb timeout -k 10 120 python3 scripts/probes/lora_kernels.py > $O/probe_$pb.json 2> $O/probe_$pb.err || exit 1
  echo "probe $pb: $(cat $O/probe_$pb.json)"
done
