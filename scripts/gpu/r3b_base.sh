#!/bin/bash
# round 3 start: smoke, GPU suite, default bench, forced-partition ZeRO-3 schedules (the N > 1 path)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3b_base}; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_identity.json 2> $O/bench_identity.err || exit $?
python -c "import json;d=json.load(open('$O/bench_identity.json'));print('identity', d['ms_per_step'], d['value'], 'peak GB', d['extra']['peak_hbm_gb_max_rank'])"
for sch in pipelined keep release; do
  LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=$sch timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$sch.json 2> $O/bench_$sch.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_$sch.json'));e=d['extra'];print('$sch', d['ms_per_step'], 'peak GB', e['peak_hbm_gb_max_rank'], 'gathered MB/step', e['zero3_gathered_mb_per_step'], 'exposed ms', e['zero3_exposed_wait_ms_per_step_max_rank'], 'skipped', e['timed_steps_skipped_nonfinite'])"
done
