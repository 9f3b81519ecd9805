# GPU-box script: full GPU tests, then the bench with rotating input sets (default)
# vs one input set, at cfg2 / cfg5 / cfg3 on 2 ranks.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-sets}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -gt 1 ] && exit $rc
b() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --cpu-seconds 0 "$@" > "$OUT/$name.json" 2>"$OUT/$name.err" || { tail -5 "$OUT/$name.err"; return 1; }
  python3 - "$OUT/$name.json" "$name" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("  ", sys.argv[2], round(d["value"]), "img/s", round(d["ms_per_step"]*1e3,1), "us/step;", d["roofline"]["kernel"], round(d["roofline"]["kernel_us"],1), "us;", d["data"])
PY
}
b cfg2_sets && b cfg2_one --input-sets 1 && b cfg2_sets2 && b cfg2_one2 --input-sets 1 && b cfg5_sets --config cfg5 && b cfg3_g2 --gpus 2
