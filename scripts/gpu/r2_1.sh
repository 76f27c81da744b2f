#!/bin/bash
# round 2, call 1: GPU test suite, 1-GPU bench (identity ZeRO-3), forced-partition schedules
# (pipelined / keep / release at the reference live budget) with peak HBM, reference offload
# config.  r2_1.sh OUT
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_1}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -2 $O/gpu_tests.txt
# test failures (rc 1) still let the benches run; a crash / timeout / abort ends the call
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || exit $?
cat $O/bench_n1.json | cut -c1-400
for sch in pipelined keep; do
  LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=$sch timeout -k 10 300 python bench.py --steps 10 --warmup 3 >> $O/forced.jsonl 2>> $O/forced.err || exit $?
done
LUMEN_ZERO3_SINGLE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config configs/ds_config_zero3_release.json >> $O/forced.jsonl 2>> $O/forced.err || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config configs/ds_config_zero2_fp16.json > $O/fp16_zero2.json 2> $O/fp16.err || exit $?
cut -c1-300 $O/fp16_zero2.json
timeout -k 10 600 python bench.py --steps 4 --warmup 2 --config configs/ds_config_zero3.json > $O/offload_ref_config.json 2> $O/offload.err || exit $?
python - <<PY
import json
for l in open("$O/forced.jsonl"):
    d = json.loads(l); x = d["extra"]
    print(x["zero3"]["schedule"], d["ms_per_step"], "ms", x["peak_hbm_gb_max_rank"], "GB", x["zero3_exposed_wait_ms_per_step_max_rank"], "exposed ms", x["zero3"]["pool_size"], x["zero3"]["turn_keep"], x["zero3"]["depth"])
d = json.load(open("$O/offload_ref_config.json")); print("offload", d["ms_per_step"], d["extra"]["peak_hbm_gb_max_rank"])
PY
