#!/bin/bash
# tune the NN input-gradient GEMMs of gathered (ZeRO-3) weights, then A/B the layouts
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/s2_tune; mkdir -p $O
cp configs/tunableop/mi355x_gemms.csv $O/table.csv
LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=pipelined LUMEN_BWD_WT=none timeout -k 10 900 python bench.py --steps 2 --warmup 2 --tune_gemms $O/table.csv > $O/tune.log 2>&1
rc=$?; echo "tune rc=$rc"; tail -1 $O/tune.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
grep -c . $O/table.csv
for pol in default none; do
  if [ $pol = default ]; then unset LUMEN_BWD_WT; else export LUMEN_BWD_WT=none; fi
  LUMEN_GEMM_TABLE=$O/table.csv LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=pipelined timeout -k 10 300 python bench.py --steps 8 --warmup 3 > $O/bench_$pol.log 2>&1
  rc=$?; echo "bench $pol rc=$rc"; tail -1 $O/bench_$pol.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
done
unset LUMEN_BWD_WT
LUMEN_GEMM_TABLE=$O/table.csv timeout -k 10 300 python bench.py --steps 8 --warmup 3 > $O/bench_plain.log 2>&1
rc=$?; echo "bench plain rc=$rc"; tail -1 $O/bench_plain.log | cut -c1-260; exit $rc
