#!/bin/bash
# round-3 closing measurements, part 2: fp16 with the tuned split parts (same box as bf16),
# forced-partition keep, serving over HTTP, reference-compatible ZeRO-3 CLI
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3c_final2}; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
summ() { python3 -c "import json;d=json.load(open('$1'));e=d['extra'];print('$2', d['ms_per_step'], 'ms/step', d['value'], 'tok/s', 'peak GB', e['peak_hbm_gb_max_rank'], 'sched', (e['zero3'] or {}).get('schedule'), 'gathered total MB', e.get('zero3_gathered_mb_total'))"; }
for v in bf16 fp16 bf16b fp16b; do
  dt=${v%b}
  timeout -k 10 300 python bench.py --no_serve --dtype $dt --steps 20 --warmup 5 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  summ $O/$v.json $v
done
LUMEN_ZERO3_SINGLE=1 timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/keep_forced.json 2> $O/keep_forced.err || { tail -5 $O/keep_forced.err; exit 1; }
summ $O/keep_forced.json keep_forced
timeout -k 10 400 python -m lumen.bench.serve_bench --mode http > $O/http.json 2> $O/http.err || { tail -5 $O/http.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/http.json').read().splitlines()[-1]);print('http', d['output_tok_s'], 'ttft p50', d['ttft_p50_ms'], 'itl p50/p99', d['itl_p50_ms'], d['itl_p99_ms'])"
timeout -k 10 400 python training/train_deepspeed_zero3.py --deepspeed configs/ds_config_zero3_mi355x.json \
    --synthetic --synthetic_samples 512 --max_steps 24 --logging_steps 8 --save_strategy no \
    --output_dir /tmp/ck_fused --metrics_csv /tmp/m_fused.csv > $O/zero3_cli.log 2>&1 || { tail -20 $O/zero3_cli.log; exit 1; }
grep -E "window_tokens" $O/zero3_cli.log | tail -1 | cut -c1-300
