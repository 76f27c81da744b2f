#!/bin/bash
# world-4 rehearsal of the FULL Llama-2-7B bench.py N > 1 path (four ranks sharing the box's one
# GPU, RCCL over loopback): every record field -- extra.comm incl. the peer-access matrix and the
# custom all-reduce setup, extra.box per rank, the wall budget, partitioned schedules, TP = 4 serve
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_20; mkdir -p $O
export LUMEN_SHARED_GPU_REHEARSAL=1 LUMEN_DIST_TIMEOUT=300
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29643 bench.py --gpus 4 --model llama2-7b --steps 5 --warmup 2 \
  --partitioned_steps 1 --partitioned release --serve_tp_shape 32,256,16 > $O/bench_w4.json 2> $O/bench_w4.err \
  || { tail -30 $O/bench_w4.err; exit 1; }
echo "json lines: $(grep -c '^{' $O/bench_w4.json)"
python3 - <<PY
import json
d = json.load(open("$O/bench_w4.json"))
e = d["extra"]
print("w4", d["n_gpus"], d["value"], d["ms_per_step"], d["config"]["parallelism"], "rccl_world", e["rccl_world"])
for k in ("budget", "box", "comm", "zero3", "zero3_release", "zero3_hybrid", "serve_tp"):
    print(k, json.dumps(e.get(k))[:1800])
PY
