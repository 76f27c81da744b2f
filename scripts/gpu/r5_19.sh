#!/bin/bash
# full GPU suite on the current tree + smoke
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_19
timeout -k 10 1080 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
  > gpurun_out/r5_19/gpu_suite.txt 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5_19/gpu_suite.txt | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r5_19/smoke.txt 2>&1; rc=$?
tail -3 gpurun_out/r5_19/smoke.txt
exit $rc
