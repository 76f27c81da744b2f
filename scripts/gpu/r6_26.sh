#!/bin/bash
# round 6 tree: full GPU suite, smoke, bench (default flags)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_26; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/gpu_suite.txt 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_suite.txt | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - <<PY
import json
d = json.loads(open("$O/bench.json").read().strip().splitlines()[-1])
print({k: d[k] for k in ("value", "ms_per_step", "vs_baseline")}); print("box", json.dumps(d["extra"].get("box"))[:900]); print("budget", json.dumps(d["extra"].get("budget")))
for k in ("serve", "serve_engine", "serve_chunked", "serve_sampled", "zero3_release", "zero3_hybrid"):
    v = d["extra"].get(k) or {}
    print(k, {kk: v.get(kk) for kk in ("output_tok_s", "itl_p99_ms", "ms_per_step")})
PY
