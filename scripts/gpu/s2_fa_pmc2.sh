#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/s2_fa_pmc2; mkdir -p $O
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
C2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA"
for v in v32 v32p; do
  for c in 1 2; do
    CC=$C1; [ $c = 2 ] && CC=$C2
    LUMEN_FA_FWD=$v timeout -s KILL 90 rocprofv3 --pmc $CC --output-format csv -d $O/${v}_$c -o run -- python3 lumen/bench/attn_bench.py --only fwd --B 2 --S 4096 --iters 3 > $O/${v}_$c.log 2>&1 || exit 1
  done
done
