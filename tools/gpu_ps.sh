# GPU-box script: cfg2 bench over the number of alternating step streams.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-ps}
mkdir -p "$OUT"
for rnd in 1 2; do
  for v in ${VARIANTS:-2 3 4}; do
    timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 300 --prop-streams $v ${EXTRA:-} > "$OUT/bench_${v}_$rnd.json" 2>"$OUT/bench_${v}_$rnd.err" || { tail -5 "$OUT/bench_${v}_$rnd.err"; exit 1; }
    python3 - "$OUT/bench_${v}_$rnd.json" "streams=$v" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("  ", sys.argv[2], round(d["value"]), "img/s", round(d["ms_per_step"]*1e3,1), "us/step; pool", round(d["roofline"]["kernel_us"],1), "us; issue", round(d["host_issue_us_per_step"],1))
PY
  done
done
