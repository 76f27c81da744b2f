#!/bin/bash
# round 6: new GPU tests (fused MLP GEMM, radix sampler, fp16 skip, custom-AR fallback) + a bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_01; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_kernels_gpu.py -k "mlp_gemm or fused_mlp or sampling" > $O/tests_kernels.txt 2>&1 \
  || { tail -40 $O/tests_kernels.txt; exit 1; }
tail -3 $O/tests_kernels.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_fp16_gpu.py "tests/test_rccl_gpu.py::test_custom_allreduce_calibration_timeout_falls_back" \
  > $O/tests_misc.txt 2>&1 || { tail -40 $O/tests_misc.txt; exit 1; }
tail -3 $O/tests_misc.txt
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - <<PY
import json
d = json.load(open("$O/bench.json"))
x = d["extra"]
print("value", d["value"], "ms", d["ms_per_step"])
print("box", json.dumps(x.get("box"))[:1500])
print("budget", json.dumps(x.get("budget")))
print("serve", (x.get("serve") or {}).get("output_tok_s"), "chunked", (x.get("serve_chunked") or {}).get("output_tok_s"))
PY
