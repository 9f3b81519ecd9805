# GPU-box script: cfg2 bench A/B of where the RoIPool runs (--pool-on prop|own),
# alternating rounds, then a kernel trace of the default.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-poolon}
mkdir -p "$OUT"
for rnd in 1 2 3; do
  for v in prop own; do
    timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 300 --pool-on $v ${EXTRA:-} > "$OUT/bench_${v}_$rnd.json" 2>"$OUT/bench_${v}_$rnd.err" || { tail -5 "$OUT/bench_${v}_$rnd.err"; exit 1; }
    python3 - "$OUT/bench_${v}_$rnd.json" $v <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("  ", sys.argv[2], round(d["value"]), "img/s", round(d["ms_per_step"]*1e3,1), "us/step; pool", round(d["roofline"]["kernel_us"],1), "us; issue", round(d["host_issue_us_per_step"],1))
PY
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --cpu-seconds 0 --steps 30 --warmup 5 > "$OUT/trace.log" 2>&1
