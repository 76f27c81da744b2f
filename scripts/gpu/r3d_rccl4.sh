#!/bin/bash
# Multi-rank RCCL rehearsals on the box's one GPU (LUMEN_SHARED_GPU_REHEARSAL=1):
# 1) bench.py at world 4 (ZeRO-3 keep), 2) the reference-compatible ZeRO-3 CLI at world 2 through
# lumen.launch with a checkpoint at step 4, 3) resume of that checkpoint at world 2 to step 6
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export LUMEN_SHARED_GPU_REHEARSAL=1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_rccl4}; mkdir -p $O
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29621 \
  bench.py --gpus 4 --steps 4 --warmup 2 --no_serve > $O/bench_w4.json 2> $O/bench_w4.err || { tail -30 $O/bench_w4.err; exit 1; }
cat $O/bench_w4.json
CLI="training/train_deepspeed_zero3.py --deepspeed configs/ds_config_zero3_mi355x.json --synthetic --synthetic_samples 256 --logging_steps 2 --save_strategy steps --save_steps 4 --output_dir /tmp/ck_w2 --metrics_csv $O/m_w2.csv"
timeout -k 10 400 python -m lumen.launch --nproc_per_node 2 --master_port 29622 $CLI --max_steps 4 > $O/cli_w2.log 2>&1 || { tail -30 $O/cli_w2.log; exit 1; }
grep -E "loss|checkpoint|saved" $O/cli_w2.log | tail -6
ls /tmp/ck_w2 /tmp/ck_w2/checkpoint-4 | head -20
timeout -k 10 400 python -m lumen.launch --nproc_per_node 2 --master_port 29623 $CLI --max_steps 6 --resume_from_checkpoint > $O/cli_w2_resume.log 2>&1 || { tail -30 $O/cli_w2_resume.log; exit 1; }
grep -E "loss|resum|checkpoint" $O/cli_w2_resume.log | tail -6
