#!/bin/bash
# GPU suite + forced-partition keep (the N > 1 code path) vs identity, after the W^T budget change
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_keep}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
for v in keep identity; do
  if [ $v = keep ]; then E="LUMEN_ZERO3_SINGLE=1"; else E="LUMEN_ZERO3_SINGLE=0"; fi
  env $E timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$v.json'));e=d['extra'];print('$v', d['ms_per_step'], d['value'], 'peak', e['peak_hbm_gb_max_rank'], e['zero3']['schedule'], 'gathered MB total', e.get('zero3_gathered_mb_total'))"
done
