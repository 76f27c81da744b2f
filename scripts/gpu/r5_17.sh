#!/bin/bash
# LoRA backward: dY pass on a side stream beside the input-gradient GEMM (LUMEN_LORA_BWD_OVERLAP), numerics + A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_17
LUMEN_LORA_BWD_OVERLAP=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py -k "lora or engine_lora" tests/test_production_shapes_gpu.py::test_llama2_7b_shaped_training_step_matches_fp32 \
  > gpurun_out/r5_17/tests.txt 2>&1 || { tail -30 gpurun_out/r5_17/tests.txt; exit 1; }
tail -2 gpurun_out/r5_17/tests.txt
for v in 1 0 1 0; do
  LUMEN_LORA_BWD_OVERLAP=$v timeout -k 10 300 python -u bench.py --no_serve --partitioned "" --no_comm_probe --steps 20 --warmup 5 > gpurun_out/r5_17/bench_ov$v.json 2>>gpurun_out/r5_17/bench.err || exit 1
  echo "overlap=$v $(python3 -c "import json,sys;d=json.loads(open('gpurun_out/r5_17/bench_ov$v.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
