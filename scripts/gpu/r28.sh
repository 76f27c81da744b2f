#!/bin/bash
# custom all-reduce: correctness after the W-templated kernel + latency sweep (shared GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r28
timeout -k 10 300 python -m pytest tests/test_custom_ar_gpu.py -x -q -s > gpurun_out/r28/car.log 2>&1 && \
timeout -k 10 300 python -m lumen.bench.car_bench --world 2 --out gpurun_out/r28/car_w2.json > gpurun_out/r28/bench_w2.log 2>&1 && \
timeout -k 10 300 python -m lumen.bench.car_bench --world 4 --out gpurun_out/r28/car_w4.json > gpurun_out/r28/bench_w4.log 2>&1
rc=$?
tail -3 gpurun_out/r28/car.log; cat gpurun_out/r28/bench_w2.log gpurun_out/r28/bench_w4.log 2>/dev/null | grep -v Gloo
exit $rc
