#!/bin/bash
# Round 4: bench.py's TP = N serving section, rehearsed with 2 and 4 RCCL ranks sharing the one
# GPU (2-layer Llama-2-7B-shaped model; the driver's 8-GPU run uses Llama-2-7B over xGMI)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_19}; mkdir -p $O
export LUMEN_SHARED_GPU_REHEARSAL=1 LUMEN_DIST_TIMEOUT=300
for n in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2963$n bench.py --gpus $n --model llama2-7b-2l --steps 3 --warmup 1 --seq_len 256 \
    --micro_batch 2 --partitioned "" > $O/bench_tp$n.json 2> $O/bench_tp$n.err || { tail -30 $O/bench_tp$n.err; exit 1; }
  python3 -c "
import json
d = json.load(open('$O/bench_tp$n.json'))
print('n=$n', d['value'], d['ms_per_step'], json.dumps(d['extra'].get('serve_tp')))"
done
