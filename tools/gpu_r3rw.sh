# GPU-box script: cfg5 draws' stream waits, front vs split, interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3rw}
mkdir -p "$OUT"
for i in 1 2; do
  for w in split front; do
    timeout -k 10 200 python -u bench.py --config cfg5 --cpu-seconds 0 --rng-waits $w > "$OUT/cfg5_${w}_$i.json" 2>"$OUT/cfg5_${w}_$i.err" || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/cfg5_${w}_$i.json').read().strip().splitlines()[-1]); print('$w', round(d['value'],1), round(d['ms_per_step']*1000,1))"
  done
done
