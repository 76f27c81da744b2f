#!/bin/bash
# PMC counters of the LoRA adapter kernels at the training shapes (one counter set per run)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-s3_lora_pmc}; mkdir -p $O
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS"
timeout -s KILL 120 rocprofv3 --pmc $C1 --output-format csv -d $O/p1 -o run -- python3 scripts/probes/lora_train_shapes.py > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/p2 -o run -- python3 scripts/probes/lora_train_shapes.py > $O/p2.log 2>&1 || exit 1
ls $O/p1 $O/p2
