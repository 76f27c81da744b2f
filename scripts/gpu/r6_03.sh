#!/bin/bash
# deterministic adapter reductions: determinism + numerics tests, the LoRA kernel tests, the
# production-shape fp32 oracle, fp16; then the bench (dy3 / dxa3 cost)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_03; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_deterministic_gpu.py tests/test_production_shapes_gpu.py tests/test_fp16_gpu.py \
  "tests/test_kernels_gpu.py::test_lora_linear_fwd_bwd" "tests/test_kernels_gpu.py::test_lora3_dxa_delta_handoff_kernel" \
  tests/test_zero3_gpu.py > $O/tests.txt 2>&1 || { tail -60 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --partitioned "" --no_serve > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - <<PY
import json
d = json.load(open("$O/bench.json"))
x = d["extra"]
print("value", d["value"], "ms", d["ms_per_step"], "loss", x["final_loss"])
print("box", json.dumps(x.get("box"))[:1200])
PY
