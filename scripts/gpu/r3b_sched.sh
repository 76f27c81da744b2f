#!/bin/bash
# ZeRO-3 schedules (forced partition at world 1 = the N > 1 code path): 7B keep (lead units) /
# pipelined / release and gathered-W^T variants; optimizer offload sync vs async; Llama-2-70B
# with the reference's live budget (release)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3b_sched}; mkdir -p $O
summ() { python -c "import json,sys;d=json.load(open('$1'));e=d['extra'];z=e['zero3'] or {};print('$2', d['ms_per_step'], 'ms/step', d['value'], 'tok/s', 'peak GB', e['peak_hbm_gb_max_rank'], 'gathered MB/step', e['zero3_gathered_mb_per_step'], 'exposed ms', e['zero3_exposed_wait_ms_per_step_max_rank'], 'skipped', e['timed_steps_skipped_nonfinite'], 'sched', z.get('schedule'), 'lead', z.get('lead_units'))"; }
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
run keep LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=keep $B --steps 20 --warmup 5 || exit 1
run keep_lead0 LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=keep LUMEN_ZERO3_LEAD=0 $B --steps 20 --warmup 5 || exit 1
run pipelined LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=pipelined $B --steps 20 --warmup 5 || exit 1
run keep_tn_all LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=keep LUMEN_GATHERED_TN=q_proj,down_proj,o_proj,gate_proj $B --steps 20 --warmup 5 || exit 1
run keep_tn_none LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=keep LUMEN_GATHERED_TN= $B --steps 20 --warmup 5 || exit 1
run keep_offpath LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=keep LUMEN_ZERO3_OFFPATH_WT=1 $B --steps 20 --warmup 5 || exit 1
run release LUMEN_ZERO3_SINGLE=1 $B --config configs/ds_config_zero3_release.json --steps 20 --warmup 5 || exit 1
run offload_opt_sync LUMEN_OFFLOAD_ASYNC=0 $B --config configs/ds_config_zero3_offload_opt_mi355x.json --steps 10 --warmup 3 || exit 1
run offload_opt_async LUMEN_OFFLOAD_ASYNC=1 $B --config configs/ds_config_zero3_offload_opt_mi355x.json --steps 10 --warmup 3 || exit 1
run r70b_release LUMEN_ZERO3_SINGLE=1 timeout -k 10 900 python bench.py --no_serve --model llama2-70b --micro_batch 4 --config configs/ds_config_zero3_release.json --steps 4 --warmup 2 || exit 1
