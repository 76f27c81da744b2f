#!/bin/bash
# step time A/B (no profiler): atomic default, deterministic split, deterministic in-kernel
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r6_24; mkdir -p $O
for rep in 1 2; do
  for mode in atomic split inkernel; do
    case $mode in
      atomic) env_="LUMEN_LORA_DETERMINISTIC=0" ;;
      split) env_="LUMEN_LORA_DETERMINISTIC=1 LUMEN_DET_SPLIT=1" ;;
      inkernel) env_="LUMEN_LORA_DETERMINISTIC=1 LUMEN_DET_SPLIT=0" ;;
    esac
    env $env_ timeout -k 10 300 python bench.py --steps 20 --warmup 3 --partitioned "" --no_serve --no_box \
      > $O/$mode$rep.json 2> $O/$mode$rep.err || { tail -10 $O/$mode$rep.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/$mode$rep.json').read().strip().splitlines()[-1]);print('$mode', $rep, d['value'], d['ms_per_step'])"
  done
done
