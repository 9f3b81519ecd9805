#!/bin/bash
# Interleaved bench A/B across library builds: bash tools/dbg/ab_bench.sh OUT REPS "bench args" lib_a.so lib_b.so ...
# ("" = the in-tree library)
out=$1; reps=$2; args=$3; shift 3
mkdir -p "$out"
for rep in $(seq 1 $reps); do
  for L in "$@"; do
    FRCNN_LIB_PATH=$L timeout -k 10 200 python -u bench.py --cpu-seconds 0 $args > "$out/b.json" 2> "$out/b.err" || { tail -5 "$out/b.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/b.json').read().strip().splitlines()[-1]); print('rep $rep ${L:-default}', round(d['value']), 'img/s', round(d['ms_per_step']*1e3,1), 'us/step')"
  done
done
