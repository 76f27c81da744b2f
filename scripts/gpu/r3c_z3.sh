#!/bin/bash
# Resident keep schedule (frozen weights gathered once) + FA register fixes: GPU suite, then
# identity vs forced-partition keep / release (the N > 1 code path) on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3c_z3}; mkdir -p $O
summ() { python -c "import json,sys;d=json.load(open('$1'));e=d['extra'];z=e['zero3'] or {};print('$2', d['ms_per_step'], 'ms/step', d['value'], 'tok/s', 'peak GB', e['peak_hbm_gb_max_rank'], 'gathered MB/step', e['zero3_gathered_mb_per_step'], 'total MB', e.get('zero3_gathered_mb_total'), 'exposed ms', e['zero3_exposed_wait_ms_per_step_max_rank'], 'sched', z.get('schedule'))"; }
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; return 1; }
  summ $O/$name.json $name
}
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
B="timeout -k 10 400 python bench.py --no_serve"
run identity $B --steps 20 --warmup 5 || exit 1
run keep LUMEN_ZERO3_SINGLE=1 $B --steps 20 --warmup 5 || exit 1
run release LUMEN_ZERO3_SINGLE=1 $B --config configs/ds_config_zero3_release.json --steps 20 --warmup 5 || exit 1
run identity2 $B --steps 20 --warmup 5 || exit 1
