#!/bin/bash
# kernel trace of the training step: per-GEMM-call durations in launch order (one layer's fwd/bwd GEMMs)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r5_25; mkdir -p $O
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o train -- python3 $GRAFT_REPO_ROOT/bench.py --no_serve --partitioned "" --no_comm_probe --steps 3 --warmup 2 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
ls $O/prof
