# GPU-box script: cfg2 bench images/s vs timed steps K for 2 / 3 step streams.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-k}
mkdir -p "$OUT"
for rnd in 1 2; do
  for ps in 2 3; do
    for k in 20 50 300; do
      timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps $k --prop-streams $ps > "$OUT/b_${ps}_${k}_$rnd.json" 2>"$OUT/b_${ps}_${k}_$rnd.err" || { tail -5 "$OUT/b_${ps}_${k}_$rnd.err"; exit 1; }
      python3 - "$OUT/b_${ps}_${k}_$rnd.json" "streams=$ps K=$k" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("  ", sys.argv[2], round(d["value"]), "img/s", round(d["ms_per_step"]*1e3,1), "us/step")
PY
    done
  done
done
