#!/bin/bash
# flash-attention A/B: ab_so/A.so (before) vs ab_so/B.so (after): FA numerics on B, per-shape
# timing interleaved B A B, kernel trace of the training shape, full bench step B A B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_fa_ab}; mkdir -p $O
SO=lumen/_C.cpython-310-x86_64-linux-gnu.so
cp ab_so/B.so $SO
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_serving_gpu.py -q -k "flash or attention or paged or prefill" --timeout 120 --timeout-method thread > $O/fa_tests.txt 2>&1
rc=$?; tail -3 $O/fa_tests.txt; [ $rc -eq 0 ] || exit $rc
for v in B A B A; do
  cp ab_so/$v.so $SO
  timeout -k 10 120 python3 scripts/probes/fa_fwd_probe.py --bwd --shapes 8x512c,8x512n,2x2048n > $O/shapes_$v.jsonl 2> $O/shapes_$v.err || { tail -5 $O/shapes_$v.err; exit 1; }
  sed "s/^/$v /" $O/shapes_$v.jsonl
done
for v in B A; do
  cp ab_so/$v.so $SO
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python3 scripts/probes/fa_fwd_probe.py --bwd --shapes 8x512c --iters 20 > $O/kt_$v.log 2>&1 || { tail -5 $O/kt_$v.log; exit 1; }
  python3 - $O/kt_$v $v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "lumen::fa" in r["Name"]:
        print(sys.argv[2], f'{float(r["AverageNs"])/1e3:8.1f} us x {r["Calls"]:>4}  {r["Name"][:80]}')
PY
done
for v in B A B; do
  cp ab_so/$v.so $SO
  timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('bench $v', d['ms_per_step'], d['value'])"
done
cp ab_so/B.so $SO
