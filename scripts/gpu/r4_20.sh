#!/bin/bash
# Round 4: bench.py's TP section at world 2 (two ranks on the one GPU): normal, then with a
# 5-second deadline (the JSON line must still come out, with extra.serve_tp = the timeout)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_20}; mkdir -p $O
export LUMEN_SHARED_GPU_REHEARSAL=1 LUMEN_DIST_TIMEOUT=300
for dl in 420 5; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 2964${dl:0:1} bench.py --gpus 2 --model llama2-7b-2l --steps 3 --warmup 1 --seq_len 256 \
    --micro_batch 2 --partitioned "" --serve_tp_deadline $dl > $O/bench_dl$dl.json 2> $O/bench_dl$dl.err
  rc=$?
  echo "deadline=$dl rc=$rc lines=$(grep -c '^{' $O/bench_dl$dl.json)"
  python3 -c "
import json
d = json.loads(open('$O/bench_dl$dl.json').readline())
print('deadline=$dl', d['value'], json.dumps(d['extra'].get('serve_tp'))[:300])" || exit 1
done
