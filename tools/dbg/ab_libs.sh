#!/bin/bash
# Interleaved A/B of the RoIPool forward across library builds:
#   bash tools/dbg/ab_libs.sh OUTDIR "cfg2 cfg3" lib_a.so lib_b.so ...
# ("" = the in-tree library).  Each run is bounded; the first failure ends the script.
out=$1; cfgs=$2; shift 2
mkdir -p "$out"
for rep in 1 2; do
  for L in "$@"; do
    for c in $cfgs; do
      FRCNN_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_roi_pool.py --config $c --variants wave \
        > "$out/ab.json" 2> "$out/ab.err" || { tail -5 "$out/ab.err"; exit 1; }
      python3 -c "import json,sys; d=json.load(open('$out/ab.json')); v=d['variants']['wave']; print('rep $rep lib ${L:-default} $c', round(v['us_median'],1), round(v['us_min'],1))"
    done
  done
done
