#!/bin/bash
# FA stall breakdown: wave-parked vs issue-stall vs active
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc26 -o attn --output-format csv -- python3 lumen/bench/attn_bench.py --iters 2 > gpurun_out/pmc26.log 2>&1
echo "pmc rc=$?"
