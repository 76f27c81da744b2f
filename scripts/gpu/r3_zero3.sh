#!/bin/bash
# ZeRO-3 schedules on the final tree with partitioning forced at world size 1 (the code path of
# the N > 1 runs: every step re-gathers the frozen weights through the coordinator)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3_zero3}; mkdir -p $O
for sch in pipelined keep release; do
  LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=$sch timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$sch.json 2> $O/bench_$sch.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_$sch.json'));e=d['extra'];print('$sch', d['ms_per_step'], 'peak GB', e['peak_hbm_gb_max_rank'], 'gathered MB/step', e['zero3_gathered_mb_per_step'], 'exposed ms', e['zero3_exposed_wait_ms_per_step_max_rank'], 'skipped', e['timed_steps_skipped_nonfinite'])"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_identity.json 2> $O/bench_identity.err || exit $?
python -c "import json;d=json.load(open('$O/bench_identity.json'));print('identity', d['ms_per_step'], 'peak GB', d['extra']['peak_hbm_gb_max_rank'])"
