#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
rm -rf build/lumen_native lumen/_C*.so
timeout -k 10 900 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/r25_build.log 2>&1 || { tail -20 gpurun_out/r25_build.log; exit 1; }
tail -2 gpurun_out/r25_build.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids
