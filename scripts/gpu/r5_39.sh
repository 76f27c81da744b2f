#!/bin/bash
# FA forward cost split, second pass: probes 0 / 3 (no key loop) / 5 (no softmax) + an LDS / VALU
# counter pass on the production kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_39; mkdir -p $O
for p in 0 3 5; do
  LUMEN_FA_PROBE=$p timeout -k 10 120 rocprofv3 --kernel-trace -d $O/p$p -o p$p -- \
    python3 lumen/bench/attn_bench.py --only fwd --iters 30 > $O/p$p.json 2> $O/p$p.err || exit 1
  python3 scripts/tools/rocpd_summary.py $O/p$p fwd32
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d $O/pmc -o pmc -- \
  python3 lumen/bench/attn_bench.py --only fwd --iters 10 > $O/pmc.json 2> $O/pmc.err || exit 1
python3 scripts/tools/rocpd_summary.py $O/pmc fwd32
