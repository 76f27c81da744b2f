#!/bin/bash
# in-step A/B: the down projection (N 4096, K 11008) at the 256-row decode bucket on decode_gemm
# (BN 64, S 4, 8 waves) vs hipBLASLt; the plan table is edited on the box copy only
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_34; mkdir -p $O
timeout -k 10 300 python -u scripts/probes/decode_step_probe.py > $O/lib.txt 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
python3 - <<PY
import json
p = "configs/kernels/decode_gemm_plans.json"
d = json.load(open(p))
d["plans"].append({"N": 4096, "K": 11008, "BM": 256, "BN": 64, "S": 4, "NW": 8, "M_measured": 256, "us": 0, "lib_us": 0})
d["plans"].append({"N": 4096, "K": 4096, "BM": 256, "BN": 64, "S": 4, "NW": 8, "M_measured": 256, "us": 0, "lib_us": 0})
json.dump(d, open(p, "w"))
PY
timeout -k 10 300 python -u scripts/probes/decode_step_probe.py > $O/dg.txt 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
timeout -k 10 300 python -u scripts/probes/decode_step_probe.py > $O/dg2.txt 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
git -C "$GRAFT_REPO_ROOT" checkout configs/kernels/decode_gemm_plans.json 2>/dev/null || python3 - <<PY
import json
p = "configs/kernels/decode_gemm_plans.json"
d = json.load(open(p)); d["plans"] = [e for e in d["plans"] if e.get("BM") != 256]; json.dump(d, open(p, "w"), indent=1)
PY
timeout -k 10 300 python -u scripts/probes/decode_step_probe.py > $O/lib2.txt 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
for f in lib dg dg2 lib2; do echo "$f $(grep ms_per $O/$f.txt)"; done
