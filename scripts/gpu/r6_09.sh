#!/bin/bash
# LoRA backward pass tile heights: dY rows per lora3_dy block x x rows per lora3_dxa block
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r6_10; mkdir -p $O
for dy in 0 256 512 1024; do
  for dxa in 0 256 512 1024; do
    LUMEN_LORA_DY_TW=$dy LUMEN_LORA_DXA_TW=$dxa timeout -k 10 120 python scripts/probes/lora_train_shapes.py > $O/dy${dy}_dxa${dxa}.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "dy=$dy dxa=$dxa $(cat $O/dy${dy}_dxa${dxa}.json)"
  done
done
