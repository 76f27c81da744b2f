#!/bin/bash
# RMSNorm: 4 waves per row (fwd: the workgroup-per-row kernel; bwd: WPR 4) vs the defaults
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_rms}; mkdir -p $O
LUMEN_RMS_FWD_WPR=4 LUMEN_RMS_BWD_WPR=4 timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "rmsnorm or norm" --timeout 180 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -1 $O/tests.txt; [ $rc -eq 0 ] || { tail -30 $O/tests.txt; exit $rc; }
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step_$n -o run -- python3 bench.py --no_serve --steps 4 --warmup 3 > $O/traced_$n.json 2> $O/traced_$n.err || { tail -5 $O/traced_$n.err; return 1; }
  python3 scripts/tools/step_table.py $O/step_$n > $O/step_table_$n.txt && grep -E "wall|rmsnorm" $O/step_table_$n.txt | sed "s/^/$n /"
}
run base LUMEN_RMS_FWD_WPR=2 && run w4 LUMEN_RMS_FWD_WPR=4 LUMEN_RMS_BWD_WPR=4 || exit 1
for v in w4 base w4 base; do
  if [ $v = w4 ]; then E="LUMEN_RMS_FWD_WPR=4 LUMEN_RMS_BWD_WPR=4"; else E="LUMEN_RMS_FWD_WPR=2"; fi
  env $E timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('bench $v', d['ms_per_step'], d['value'])"
done
