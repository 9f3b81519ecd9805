# GPU-box script: cfg2 bench over a list of option sets (one line each), plus
# an optional RoIPool A/B first.  Usage: bash tools/gpu_bench_sweep.sh TAG "opts1" "opts2" ...
set -u
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*"; }
if [ -n "${AB:-}" ]; then
  st "ab $AB"
  timeout -k 10 200 python -u tools/ab_roi_pool.py $AB > "$OUT/ab.json" 2>&1 || { cat "$OUT/ab.json"; exit 1; }
  mv "$OUT/ab.json" "$OUT/ab_1.log"; python tools/ab_summary.py "$OUT"
fi
i=0
for a in "$@"; do
  i=$((i+1))
  st "bench $a"
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 $a > "$OUT/bench_$i.json" 2>"$OUT/bench_$i.err" || { tail -20 "$OUT/bench_$i.err"; exit 1; }
  python - "$OUT/bench_$i.json" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("   ", round(d["value"]), "img/s", round(d["ms_per_step"]*1e3,1), "us/step; dom kernel", round(d["roofline"]["kernel_us"],1), "us; issue", round(d["host_issue_us_per_step"],1), "us")
PY
done
