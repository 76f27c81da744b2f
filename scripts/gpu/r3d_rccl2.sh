#!/bin/bash
# First multi-rank RCCL runs on hardware: 2 ranks sharing the box's one GPU
# (LUMEN_SHARED_GPU_REHEARSAL=1: per-rank NCCL_HOSTID, RCCL socket transport over loopback).
# 1) collective semantics probe, 2) bench.py ZeRO-3 (keep) at world 2, 3) the release schedule
# at world 2 (per-use all-gathers of the frozen weights on their own communicator).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export LUMEN_SHARED_GPU_REHEARSAL=1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_rccl2}; mkdir -p $O
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 180 $RUN --master-port 29611 scripts/probes/rccl_probe.py > $O/probe.log 2>&1 || { tail -30 $O/probe.log; exit 1; }
grep -E "rccl_probe" $O/probe.log
timeout -k 10 400 $RUN --master-port 29612 bench.py --gpus 2 --steps 6 --warmup 3 --no_serve > $O/bench_keep.json 2> $O/bench_keep.err || { tail -30 $O/bench_keep.err; exit 1; }
cat $O/bench_keep.json
grep -E "zero3|schedule" $O/bench_keep.err | head -5
timeout -k 10 400 $RUN --master-port 29613 bench.py --gpus 2 --steps 4 --warmup 2 --no_serve --config configs/ds_config_zero3_release.json > $O/bench_release.json 2> $O/bench_release.err || { tail -30 $O/bench_release.err; exit 1; }
cat $O/bench_release.json
