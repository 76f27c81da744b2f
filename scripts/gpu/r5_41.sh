#!/bin/bash
# MLP tail overlap, why slower: kernel traces of LUMEN_MLP_OVERLAP 0 / 1 (3 steps each), and the
# bench with the round-5 table (no down-dX split rows) vs the new table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_41; mkdir -p $O
cp configs/tunableop/mi355x_gemms.csv $O/new.csv
grep -v "tn_2816_4096_4096_ld_4096_4096_11008\|tn_8192_4096_4096_ld_4096_4096_11008" $O/new.csv > $O/old.csv
for m in 0 1; do
  LUMEN_MLP_OVERLAP=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t$m -o t$m -- python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 3 --warmup 2 > $O/tb_$m.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
done
for t in old new old new; do
  cp $O/$t.csv configs/tunableop/mi355x_gemms.csv
  LUMEN_MLP_OVERLAP=0 timeout -k 10 300 python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 20 --warmup 5 > $O/bench_$t.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$t.json')); print('table $t', d['value'], d['ms_per_step'])"
done
