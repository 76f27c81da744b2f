#!/bin/bash
# in-step GEMM solution A/B: swap one big training-shape entry of the TunableOp table for the
# runner-up of a fresh tuning probe (profiles/r2_gemm_split/candidates_r3_9.txt) and time bench.py
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3_insitu}; mkdir -p $O
T=configs/tunableop/mi355x_gemms.csv
run() {  # name table
  LUMEN_GEMM_TABLE=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$1.json 2> $O/bench_$1.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_$1.json'));print('$1', d['ms_per_step'], d['extra']['gemm_table_entries'])"
}
variant() {  # name signature solution
  sed "s/^\(GemmTunableOp_BFloat16_TN,$2,\)[^,]*,/\1$3,/" $T > $O/table_$1.csv
  grep -c ",$2,$3," $O/table_$1.csv > /dev/null || { echo "no entry for $2"; return 0; }
  run $1 $O/table_$1.csv
}
run base0 $T
variant gu_dx tn_4096_4096_22016_ld_22016_22016_4096 Gemm_Hipblaslt_627945
variant gu_part tn_20480_4096_4096_ld_4096_4096_22016 Gemm_Hipblaslt_618463
variant dn_dx tn_11008_4096_4096_ld_4096_4096_11008 Gemm_Rocblas_618611
variant qkv_fwd tn_12288_4096_4160_ld_4160_4160_12288 Gemm_Rocblas_618464
variant qkv_dx tn_4096_4096_12288_ld_12288_12288_4096 Gemm_Rocblas_618611
variant dn_fwd tn_4096_4096_11008_ld_11008_11008_4096 Gemm_Hipblaslt_618463
run base1 $T
