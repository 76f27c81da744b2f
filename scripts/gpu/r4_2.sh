#!/bin/bash
# Round 4: multi-rank RCCL rehearsals on the box's one GPU (LUMEN_SHARED_GPU_REHEARSAL: every
# rank its own RCCL host id, socket transport).  RCCL test suite (world 2 and 8, TP 2 / 8 vs
# TP 1), then bench.py at world 8 on the reduced-depth Llama-2-7B (keep headline + release /
# hybrid partitioned steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rccl_gpu.py -v --timeout 300 --timeout-method thread > $O/rccl_tests.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/rccl_tests.txt | tail -20; tail -1 $O/rccl_tests.txt; [ $rc -eq 0 ] || exit $rc
export LUMEN_SHARED_GPU_REHEARSAL=1 LUMEN_DIST_TIMEOUT=300
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 8 --model llama2-7b-2l --steps 3 --warmup 1 --seq_len 256 \
  --micro_batch 2 --partitioned_steps 2 > $O/bench_w8.json 2> $O/bench_w8.err || { tail -30 $O/bench_w8.err; exit 1; }
python3 - <<EOF
import json
d = json.load(open("$O/bench_w8.json"))
e = d["extra"]
print("w8", d["n_gpus"], d["value"], d["ms_per_step"], d["config"]["parallelism"], "rccl_world", e["rccl_world"])
for k in ("zero3", "zero3_release", "zero3_hybrid"):
    print(k, json.dumps(e.get(k)))
EOF
