#!/bin/bash
# Round 4: world-8 / TP-8 RCCL tests (fixed), then the world-8 bench rehearsal and TP serving
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_6}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_kernels_gpu.py tests/test_rccl_gpu.py -v --timeout 300 --timeout-method thread -k "rope or fp32 or world8 or matches_tp1" > $O/rccl_tests.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/rccl_tests.txt | tail -20; tail -1 $O/rccl_tests.txt; [ $rc -eq 0 ] || exit $rc
sed -n '/^export LUMEN_SHARED_GPU_REHEARSAL/,$p' scripts/gpu/r4_2.sh > $O/rest.sh
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
# TP serving: TP=1 vs TP=2 with both ranks on the one GPU (the host header over gloo, the payload
# over RCCL, decode graphs with the custom all-reduce); reduced-depth Llama-2-7B, 64 x 256 / 64
unset LUMEN_SHARED_GPU_REHEARSAL
timeout -k 10 300 python -m lumen.bench.serve_bench --model llama2-7b-2l --num-requests 64 --prompt-len 256 \
  --max-tokens 64 --max-model-len 512 --num-blocks 4096 > $O/serve_tp1.json 2> $O/serve_tp1.err || { tail -10 $O/serve_tp1.err; exit 1; }
export LUMEN_SHARED_GPU_REHEARSAL=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29621 -m lumen.bench.serve_bench --tp 2 --model llama2-7b-2l --num-requests 64 --prompt-len 256 \
  --max-tokens 64 --max-model-len 512 --num-blocks 4096 > $O/serve_tp2.json 2> $O/serve_tp2.err || { tail -20 $O/serve_tp2.err; exit 1; }
python3 - <<EOF2
import json
for t in ("tp1", "tp2"):
    d = json.loads([l for l in open("$O/serve_" + t + ".json") if l.startswith("{")][-1])
    print(t, {k: d.get(k) for k in ("output_tok_s", "ttft_p50_ms", "itl_p50_ms", "itl_p99_ms", "graphs")})
EOF2
