#!/bin/bash
# round-3 closing measurements: default bench (train + extra.serve), bf16 vs fp16 same box,
# forced-partition keep, serving engine + HTTP, reference-compatible ZeRO-3 CLI
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3c_final}; mkdir -p $O
summ() { python3 -c "import json;d=json.load(open('$1'));e=d['extra'];print('$2', d['ms_per_step'], 'ms/step', d['value'], 'tok/s', 'peak GB', e['peak_hbm_gb_max_rank'], 'sched', (e['zero3'] or {}).get('schedule'), 'serve', (e.get('serve') or {}).get('output_tok_s'))"; }
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
summ $O/bench_default.json default
timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/bf16.json 2> $O/bf16.err || { tail -5 $O/bf16.err; exit 1; }
summ $O/bf16.json bf16
timeout -k 10 300 python bench.py --no_serve --dtype fp16 --steps 20 --warmup 5 > $O/fp16.json 2> $O/fp16.err || { tail -5 $O/fp16.err; exit 1; }
summ $O/fp16.json fp16
LUMEN_ZERO3_SINGLE=1 timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/keep_forced.json 2> $O/keep_forced.err || { tail -5 $O/keep_forced.err; exit 1; }
summ $O/keep_forced.json keep_forced
timeout -k 10 400 python -m lumen.bench.serve_bench --mode http > $O/http.json 2> $O/http.err || { tail -5 $O/http.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/http.json').read().splitlines()[-1]);print('http', d['output_tok_s'], 'ttft p50', d['ttft_p50_ms'], 'itl p50/p99', d['itl_p50_ms'], d['itl_p99_ms'])"
timeout -k 10 400 python training/train_deepspeed_zero3.py --deepspeed configs/ds_config_zero3_mi355x.json \
    --synthetic --synthetic_samples 512 --max_steps 24 --logging_steps 8 --save_strategy no \
    --output_dir /tmp/ck_fused --metrics_csv /tmp/m_fused.csv > $O/zero3_cli.log 2>&1 || { tail -20 $O/zero3_cli.log; exit 1; }
grep -E "window_tokens" $O/zero3_cli.log | tail -1 | cut -c1-300
