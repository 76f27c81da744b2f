#!/bin/bash
# decode-step probe: bf16 KV, new uniform-block-id nt kernel (LUMEN_PA_1PASS=2, default) vs the
# round-4 kernel (=1); then a kernel trace of the decode steps
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_03
for v in 2 1 2 1; do
  LUMEN_PA_1PASS=$v timeout -k 10 300 python -u scripts/probes/decode_step_probe.py >> gpurun_out/r5_03/ab_v$v.txt 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_03/prof -o dec --output-format csv -- python3 scripts/probes/decode_step_probe.py > gpurun_out/r5_03/prof.log 2>&1 || exit 1
python3 scripts/tools/decode_table.py gpurun_out/r5_03/prof > gpurun_out/r5_03/decode_table.txt
grep -h ms_per gpurun_out/r5_03/ab_v*.txt; head -30 gpurun_out/r5_03/decode_table.txt
