#!/bin/bash
# LoRA kernel iteration: LoRA GPU tests, 1-GPU bench, PMC LDS-conflict survey of the step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r2_lora}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "lora or fold" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['value'])"
bash scripts/gpu/r2_pmc_bench.sh ${1:-r2_lora}/pmcb > /dev/null || exit $?
grep "lv3\|lv2" $O/pmcb/summary.txt
