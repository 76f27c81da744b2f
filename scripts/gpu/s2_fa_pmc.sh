#!/bin/bash
# PMC counters of the flash-attention kernels (fwd v32 vs t1, bwd v32 vs v16), S=4096
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/s2_fa_pmc; mkdir -p $O
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
for v in "t1 v16" "v32 v32"; do set -- $v
  LUMEN_FA_FWD=$1 LUMEN_FA_BWD=$2 timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/$1 -o run -- python3 lumen/bench/attn_bench.py --only bwd --B 2 --S 4096 --iters 3 > $O/$1.log 2>&1 || exit 1
done
ls -R $O | head
