#!/bin/bash
# Round 4: hybrid GPU tests (fixed), the driver's bench (headline + partitioned release / hybrid
# + HTTP serving), then the activation-checkpointing policies on the compat CLI
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_5}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_zero3_gpu.py tests/test_kernels_gpu.py -v --timeout 180 --timeout-method thread -k "hybrid or transposed or grad_paths" > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/gpu_tests.txt | tail -20; tail -1 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - <<EOF2
import json
d = json.load(open("$O/bench.json"))
e = d["extra"]
print("train", d["value"], d["ms_per_step"], d["config"]["parallelism"], "peak", e["peak_hbm_gb_max_rank"])
for k in ("zero3_release", "zero3_hybrid", "serve", "serve_engine", "native_build"):
    print(k, json.dumps(e.get(k)))
EOF2
bash scripts/gpu/r4_3.sh r4_5/ckpt
