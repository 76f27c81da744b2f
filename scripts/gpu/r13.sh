#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
( for i in $(seq 1 16); do rocm-smi --showclocks --showpower 2>/dev/null | grep -E "sclk|Power|fclk|mclk" | tr '\n' ' '; echo; sleep 1; done ) > gpurun_out/r13_smi.log 2>&1 &
SMI=$!
timeout -k 10 120 python -m lumen.bench.power_probe > gpurun_out/r13_probe.log 2>&1
rc=$?
wait $SMI
cat gpurun_out/r13_probe.log | grep -v amdgpu.ids
cat gpurun_out/r13_smi.log
exit $rc
