#!/bin/bash
# kernel numerics + rocprofv3 kernel-trace/stats of the headline bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q > gpurun_out/kernels.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 3 --warmup 1 ${BENCH_ARGS} > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
