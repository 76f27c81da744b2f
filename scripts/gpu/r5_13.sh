#!/bin/bash
# paged decode variants: numerics (all variants), then decode-step A/B 2 (uniform nt) vs 3 (pipelined)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_13
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  "tests/test_kernels_gpu.py::test_paged_decode" "tests/test_kernels_gpu.py::test_fp8_kv_cache_kernels" \
  > gpurun_out/r5_13/test.txt 2>&1 || { tail -30 gpurun_out/r5_13/test.txt; exit 1; }
for v in 3 2 3 2; do
  LUMEN_PA_1PASS=$v timeout -k 10 300 python -u scripts/probes/decode_step_probe.py >> gpurun_out/r5_13/pa_v$v.txt 2>&1 || exit 1
done
for v in 3 2; do
  LUMEN_PA_1PASS=$v timeout -k 10 300 python -u scripts/probes/decode_step_probe.py --kv fp8 >> gpurun_out/r5_13/fp8_v$v.txt 2>&1 || exit 1
done
LUMEN_PA_1PASS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_13/prof -o dec --output-format csv -- python3 scripts/probes/decode_step_probe.py > gpurun_out/r5_13/prof.log 2>&1 || exit 1
python3 scripts/tools/decode_table.py gpurun_out/r5_13/prof > gpurun_out/r5_13/decode_table_v3.txt
tail -2 gpurun_out/r5_13/test.txt
for f in gpurun_out/r5_13/pa_v*.txt gpurun_out/r5_13/fp8_v*.txt; do echo $f; grep ms_per $f; done
head -5 gpurun_out/r5_13/decode_table_v3.txt
