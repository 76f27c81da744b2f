#!/bin/bash
# dy3 with Z rows prefetched one stage ahead: LoRA numerics + determinism tests, then the probe
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r6_11; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_deterministic_gpu.py tests/test_kernels_gpu.py -k "lora or deterministic" > $O/tests.txt 2>&1 \
  || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for i in 1 2; do
  timeout -k 10 120 python scripts/probes/lora_train_shapes.py > $O/probe$i.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
  cat $O/probe$i.json
done
