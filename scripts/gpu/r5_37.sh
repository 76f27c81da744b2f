#!/bin/bash
# world-8 bench.py rehearsal (8 ranks sharing the GPU, 2-layer Llama-2-7B shapes): every record
# field incl. extra.comm (transport probe) and the partitioned link-time estimates, TP = 8 serve
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_37; mkdir -p $O
export LUMEN_SHARED_GPU_REHEARSAL=1 LUMEN_DIST_TIMEOUT=300
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29641 bench.py --gpus 8 --model llama2-7b-2l --steps 3 --warmup 1 --seq_len 256 \
  --micro_batch 2 --partitioned_steps 2 > $O/bench_w8.json 2> $O/bench_w8.err || { tail -30 $O/bench_w8.err; exit 1; }
echo "json lines: $(grep -c '^{' $O/bench_w8.json)"
python3 - <<EOF
import json
d = json.load(open("$O/bench_w8.json"))
e = d["extra"]
print("w8", d["n_gpus"], d["value"], d["ms_per_step"], d["config"]["parallelism"], "rccl_world", e["rccl_world"])
print("comm", json.dumps(e.get("comm"))[:1500])
for k in ("zero3_release", "zero3_hybrid"):
    print(k, json.dumps(e.get(k))[:600])
print("serve_tp", json.dumps(e.get("serve_tp"))[:600])
EOF
