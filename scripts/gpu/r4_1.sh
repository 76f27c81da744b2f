#!/bin/bash
# Round 4, first call: decode-GEMM numerics, ZeRO-3 hybrid + RCCL async-offload tests, the decode
# GEMM sweep vs hipBLASLt (plan table), then the driver's bench (headline + partitioned release /
# hybrid timings + HTTP serving section)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_1}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode_gemm_variants" -v --timeout 120 --timeout-method thread > $O/dgemm_tests.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|Error" $O/dgemm_tests.txt | tail -20; tail -1 $O/dgemm_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m lumen.bench.decode_gemm_probe --plans $O/decode_gemm_plans.json > $O/decode_probe.jsonl 2> $O/decode_probe.err || { tail -5 $O/decode_probe.err; exit 1; }
grep -v sweep $O/decode_probe.jsonl
timeout -k 10 600 python -u -m pytest tests/test_zero3_gpu.py tests/test_rccl_gpu.py -v --timeout 180 --timeout-method thread -k "not world8 and not tp_serving_rccl_matches" > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/gpu_tests.txt | tail -40; tail -1 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - <<EOF
import json
d = json.load(open("$O/bench.json"))
e = d["extra"]
print("train", d["value"], d["ms_per_step"], d["config"]["parallelism"])
for k in ("zero3_release", "zero3_hybrid", "serve", "serve_engine"):
    print(k, json.dumps(e.get(k)))
EOF
