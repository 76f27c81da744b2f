#!/bin/bash
# re-tune the fp16 training GEMM shapes from scratch (TunableOp, rotating buffers), merge the
# Half rows into a copy of the shipped table, A/B the fp16 step on both tables
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_fp16tune}; mkdir -p $O
timeout -k 10 900 python bench.py --no_serve --dtype fp16 --steps 2 --warmup 2 --tune_gemms $O/tuned_fp16.csv > $O/tune.json 2> $O/tune.err || { tail -5 $O/tune.err; exit 1; }
grep -c Half $O/tuned_fp16.csv
LUMEN_TUNE_ROTATING_MB=0 timeout -k 10 600 python -m lumen.bench.split_gemm_probe --dtype fp16 --tune $O/tuned_fp16.csv > $O/tune_split.log 2>&1 || { tail -5 $O/tune_split.log; exit 1; }
grep -c Half $O/tuned_fp16.csv
python3 - $O <<'PY'
import sys
o = sys.argv[1]
old = [l.rstrip("\n") for l in open("configs/tunableop/mi355x_gemms.csv")]
new = {tuple(l.split(",")[:2]): l.rstrip("\n") for l in open(f"{o}/tuned_fp16.csv")
       if l.startswith("GemmTunableOp_Half")}
out, seen = [], set()
for l in old:
    k = tuple(l.split(",")[:2])
    if k in new:
        old_t, new_t = float(l.split(",")[3]), float(new[k].split(",")[3])
        print("retuned", k[1], "old", old_t, "new", new_t, new[k].split(",")[2])
        out.append(new[k]); seen.add(k)
    else:
        out.append(l)
for k, l in new.items():
    if k not in seen:
        print("added", k[1]); out.append(l)
open(f"{o}/merged.csv", "w").write("\n".join(out) + "\n")
PY
for t in new old new old; do
  if [ $t = new ]; then TB=$O/merged.csv; else TB=configs/tunableop/mi355x_gemms.csv; fi
  LUMEN_GEMM_TABLE=$TB timeout -k 10 300 python bench.py --no_serve --dtype fp16 --steps 20 --warmup 5 > $O/fp16_$t.json 2> $O/fp16_$t.err || { tail -5 $O/fp16_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/fp16_$t.json'));print('fp16 $t', d['ms_per_step'], d['value'], d['extra']['gemm_table_entries'])"
done
