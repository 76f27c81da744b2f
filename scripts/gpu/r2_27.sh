#!/bin/bash
# FA at the training shape (B=8, S=512): attn_bench timings + two PMC passes over fwd+bwd; fp16 test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2_27; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_fp16_gpu.py -x -q --timeout 120 --timeout-method thread > $O/fp16.txt 2>&1; tail -2 $O/fp16.txt
timeout -k 10 120 python lumen/bench/attn_bench.py --B 8 --S 512 --iters 50 > $O/attn.json 2>&1 || exit 1
cat $O/attn.json
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
C2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_MFMA"
for c in 1 2; do
  CC=$C1; [ $c = 2 ] && CC=$C2
  timeout -s KILL 90 rocprofv3 --pmc $CC --output-format csv -d $O/pmc_$c -o run -- python3 lumen/bench/attn_bench.py --only bwd --B 8 --S 512 --iters 3 > $O/pmc_$c.log 2>&1 || exit 1
done
