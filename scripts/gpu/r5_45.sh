#!/bin/bash
# world-8 shared-GPU rehearsal of the bucketed (overlapped) LoRA gradient reduce-scatter:
# 2-layer Llama-2-7B shapes with LUMEN_DP_BUCKET_MB=1 (4 buckets) vs 0 (one bucket), RCCL
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_45; mkdir -p $O
export LUMEN_SHARED_GPU_REHEARSAL=1 LUMEN_DIST_TIMEOUT=300
for mb in 1 0; do
  LUMEN_DP_BUCKET_MB=$mb timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 2965$mb bench.py --gpus 8 --model llama2-7b-2l --steps 3 --warmup 1 --seq_len 256 \
    --micro_batch 2 --partitioned "" --no_comm_probe --serve_tp 0 > $O/w8_$mb.json 2> $O/w8_$mb.err || { tail -30 $O/w8_$mb.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/w8_$mb.json')); e=d['extra']; print('bucket_mb $mb', d['value'], d['ms_per_step'], 'buckets', e['dp_grad_buckets'], 'loss', e['final_loss'])"
done
