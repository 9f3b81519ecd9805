#!/bin/bash
# Interleaved A/B of whole bench runs across library builds:
#   bash tools/dbg/ab_bench_libs.sh OUTDIR "BENCH ARGS" lib_a.so lib_b.so ...   ("" = the in-tree library)
out=$1; bargs=$2; shift 2
mkdir -p "$out"
for rep in 1 2 3; do
  for L in "$@"; do
    FRCNN_LIB_PATH=$L timeout -k 10 300 python -u bench.py $bargs > "$out/b.json" 2> "$out/b.err" || { tail -5 "$out/b.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/b.json').read().strip().splitlines()[-1]); print('rep $rep lib ${L:-default}', round(d['value'],1), round(d['ms_per_step']*1e3,1))"
  done
done
