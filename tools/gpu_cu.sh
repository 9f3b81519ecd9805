# GPU-box script: RoIPool parity after the flat-partition change, the CU-mask
# probe, pool A/B at cfg1/2/4 and the cfg2 bench with CU reservations.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-cu}
mkdir -p "$OUT"
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*"; }
st pytest
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -x -q -k "roi_pool or dist" \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
st probe
timeout -k 10 120 python -u tools/cu_probe.py > "$OUT/probe.log" 2>&1 || { cat "$OUT/probe.log"; exit 1; }
cat "$OUT/probe.log"
for c in cfg2 cfg1 cfg4; do
  st "ab $c"
  timeout -k 10 200 python -u tools/ab_roi_pool.py --config $c --variants wave,wave@2,wave@4,dense > "$OUT/ab_$c.json" 2>&1 || { cat "$OUT/ab_$c.json"; exit 1; }
  python - "$OUT/ab_$c.json" <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print(d["config"], {k: round(v["us_median"],1) for k,v in d["variants"].items()})
PY
done
for a in "--prop-cus 0" "--prop-cus 16" "--prop-cus 32" "--prop-cus 16 --cu-order blk" "--prop-cus 32 --cu-order blk"; do
  st "bench $a"
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 200 $a > "$OUT/bench.json" 2>"$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
  python - "$OUT/bench.json" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(round(d["value"]), "img/s", round(d["ms_per_step"]*1e3,1), "us/step pool", round(d["roofline"]["kernel_us"],1), "issue", round(d["host_issue_us_per_step"],1))
PY
done
