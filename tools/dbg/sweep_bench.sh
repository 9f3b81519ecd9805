#!/bin/bash
# Interleaved bench sweep: bash tools/dbg/sweep_bench.sh OUT REPS "args A" "args B" ...
out=$1; reps=$2; shift 2
mkdir -p "$out"
for rep in $(seq 1 $reps); do
  i=0
  for A in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python -u bench.py --cpu-seconds 0 $A > "$out/b_$i.json" 2> "$out/b_$i.err" || { tail -5 "$out/b_$i.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/b_$i.json').read().strip().splitlines()[-1]); print('rep $rep [$A]', round(d['value']), 'img/s', round(d['ms_per_step']*1e3,1), 'us/step')"
  done
done
