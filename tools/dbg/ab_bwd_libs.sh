#!/bin/bash
# Interleaved A/B of the RoIPool backward across library builds (cfg5, sampled RoIs):
#   bash tools/dbg/ab_bwd_libs.sh OUTDIR PATHS lib_a.so lib_b.so ...   ("" = the in-tree library)
out=$1; paths=$2; shift 2
mkdir -p "$out"
for rep in 1 2; do
  for L in "$@"; do
    FRCNN_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_roi_pool_bwd.py --paths "$paths" --rounds 5 \
      > "$out/ab.json" 2> "$out/ab.err" || { tail -5 "$out/ab.err"; exit 1; }
    python3 -c "import json; s=open('$out/ab.json').read(); d=json.loads(s[s.index('{'):]); print('rep $rep lib ${L:-default}', {k: round(v['us_median'],1) for k,v in d['paths'].items()})"
  done
done
