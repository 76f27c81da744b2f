#!/bin/bash
# split (two-stream) decode: numerics test, then A/B on the 7B decode-step probe
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_07
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  "tests/test_serving_gpu.py::test_split_decode_two_streams_matches" > gpurun_out/r5_07/test.txt 2>&1 || { tail -30 gpurun_out/r5_07/test.txt; exit 1; }
for v in 256 0 256 0; do
  LUMEN_DECODE_SPLIT=$v timeout -k 10 300 python -u scripts/probes/decode_step_probe.py >> gpurun_out/r5_07/split_$v.txt 2>&1 || exit 1
done
LUMEN_DECODE_SPLIT=256 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_07/prof -o dec --output-format csv -- python3 scripts/probes/decode_step_probe.py > gpurun_out/r5_07/prof.log 2>&1 || exit 1
python3 scripts/tools/decode_table.py gpurun_out/r5_07/prof > gpurun_out/r5_07/decode_table.txt
tail -3 gpurun_out/r5_07/test.txt; grep -h ms_per gpurun_out/r5_07/split_*.txt; head -12 gpurun_out/r5_07/decode_table.txt
